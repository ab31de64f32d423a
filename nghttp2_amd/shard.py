"""Sharding a batch of header strings across GPUs.

Every string is independent, so a batch shards into contiguous string ranges
balanced by bytes (a prefix sum over lengths), one range per rank / GPU, with
no data-path collective: each rank encodes / decodes its own shard and the
host rebases offsets with a prefix sum over the shard output sizes.  xGMI is
unused because the path has no exchange step.
"""
import numpy as np


def byte_balanced_bounds(off, world):
    """String-index bounds [(s0, s1)] * world so that each shard holds about
    total/world bytes (contiguous ranges, every string in exactly one)."""
    off = np.asarray(off, dtype=np.int64)
    n = len(off) - 1
    base, total = int(off[0]), int(off[-1] - off[0])
    cuts = [0]
    for r in range(1, world):
        target = base + (total * r) // world
        # first string whose start offset is >= target
        cuts.append(int(np.searchsorted(off[:n], target, side="left")))
    cuts.append(n)
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def shard(pool, off, s0, s1, pad=16):
    """A shard as its own SoA batch: (pool bytes padded to `pad`, offsets
    rebased to 0)."""
    off = np.asarray(off, dtype=np.int64)
    a, b = int(off[s0]), int(off[s1])
    sub = np.zeros((b - a) + (-(b - a)) % pad + pad, dtype=np.uint8)
    sub[:b - a] = pool[a:b]
    return sub, (off[s0:s1 + 1] - a).astype(np.uint32)


def merge(parts):
    """Reassemble per-shard outputs [(out_pool, out_off)] in rank order into
    one batch: concatenated pools, offsets rebased by the running total."""
    pools, offs = [], [np.zeros(1, dtype=np.int64)]
    base = 0
    for p, o in parts:
        o = np.asarray(o, dtype=np.int64)
        pools.append(np.asarray(p[:int(o[-1])], dtype=np.uint8))
        offs.append(o[1:] + base)
        base += int(o[-1])
    return (np.concatenate(pools) if pools else np.zeros(0, np.uint8),
            np.concatenate(offs).astype(np.uint64))
