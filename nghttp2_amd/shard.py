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


class ShardedCodec:
    """One batch over several devices in ONE process: the
    batch is cut into byte-balanced contiguous shards, one per entry of
    `devices`; each shard runs on its own host thread with its own HIP stream
    and its own HuffmanBatchCodec, and the host rebases the shards' output
    offsets into one batch (`merge`).  This is the reference's threading
    model (doc/programmers-guide.rst:36-40: one nghttp2 session per thread,
    no shared state) with a device behind each thread.  No collective: the
    shards never exchange data.

    `devices` may repeat a device (e.g. [0, 0]: two shards, two threads and
    two streams on one GPU).  Inputs and merged outputs are host numpy
    arrays; the device parts stay available from the last call
    (`last_parts`) for callers that keep the results resident."""

    def __init__(self, devices):
        import threading
        import torch

        from .hd import HuffmanBatchCodec
        self.torch = torch
        self.devices = [torch.device("cuda", d) if isinstance(d, int) else torch.device(d)
                        for d in devices]
        if not self.devices:
            raise ValueError("ShardedCodec needs at least one device")
        self.codecs, self.streams = [], []
        for d in self.devices:
            with torch.cuda.device(d):
                self.codecs.append(HuffmanBatchCodec(d))
                self.streams.append(torch.cuda.Stream(device=d))
        self._lock = threading.Lock()
        self.last_parts = None

    def _run(self, fn, n):
        """fn(k) for every shard k, each on its own host thread; re-raises the
        first failure after every thread has finished."""
        import threading
        out, err = [None] * n, []

        def body(k):
            try:
                with self.torch.cuda.device(self.devices[k]), \
                        self.torch.cuda.stream(self.streams[k]):
                    out[k] = fn(k)
                    self.streams[k].synchronize()
            except BaseException as e:  # reported after the join
                with self._lock:
                    err.append((k, e))
        ts = [threading.Thread(target=body, args=(k,)) for k in range(n)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if err:
            k, e = sorted(err, key=lambda x: x[0])[0]
            raise RuntimeError("shard %d (%s) failed: %s" % (k, self.devices[k], e)) from e
        return out

    def _scatter(self, pool, off):
        off = np.asarray(off, dtype=np.int64)
        bounds = byte_balanced_bounds(off, len(self.devices))
        return bounds, [shard(pool, off, s0, s1) for s0, s1 in bounds]

    def _to_dev(self, k, sp, so):
        t = self.torch
        src = t.from_numpy(sp).to(self.devices[k], non_blocking=False)
        src_off = t.from_numpy(so.astype(np.uint32).view(np.int32)).to(self.devices[k])
        return src, src_off

    def encode(self, pool, off):
        """Huffman-encode the batch across the devices: returns the merged
        (encoded pool uint8, offsets uint64[n+1]), equal to a single-device
        encode of the whole batch."""
        _, parts = self._scatter(pool, off)

        def work(k):
            sp, so = parts[k]
            src, src_off = self._to_dev(k, sp, so)
            enc, eoff = self.codecs[k].encode(src, src_off, raw_bytes=int(so[-1]),
                                              stream=self.streams[k])
            return enc, eoff
        dev_parts = self._run(work, len(parts))
        self.last_parts = dev_parts
        host = [(e.cpu().numpy(), o.cpu().numpy().view(np.uint32)) for e, o in dev_parts]
        return merge(host)

    def decode_auto(self, enc_pool, enc_off):
        """Decode the batch (final=1 per string) across the devices into the
        dense layout of each shard, merged: returns (decoded pool uint8,
        dst_off uint64[n+1], status int32[n]); string i's bytes are
        pool[dst_off[i] : dst_off[i] + status[i]] when status[i] >= 0."""
        _, parts = self._scatter(enc_pool, enc_off)

        def work(k):
            sp, so = parts[k]
            src, src_off = self._to_dev(k, sp, so)
            return self.codecs[k].decode_auto(src, src_off, enc_bytes=int(so[-1]),
                                              stream=self.streams[k])
        dev_parts = self._run(work, len(parts))
        self.last_parts = dev_parts
        host, status = [], []
        for d, o, st in dev_parts:
            oh = o.cpu().numpy().view(np.uint32)
            host.append((d[:int(oh[-1])].cpu().numpy(), oh))
            status.append(st.cpu().numpy())
        pool_m, off_m = merge(host)
        return pool_m, off_m, (np.concatenate(status) if status else np.zeros(0, np.int32))
