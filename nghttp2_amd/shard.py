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


def _lib():
    import ctypes
    from .hd import lib
    L = lib()
    if not getattr(L, "_sharded_bound", False):
        vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
        L.nghttp2_amd_hd_shard_bounds.argtypes = [vp, u32, u32, vp]
        L.nghttp2_amd_hd_sharded_new.argtypes = [ctypes.POINTER(vp), vp, u32]
        L.nghttp2_amd_hd_sharded_del.argtypes = [vp]
        L.nghttp2_amd_hd_sharded_del.restype = None
        L.nghttp2_amd_hd_sharded_count.argtypes = [vp]
        L.nghttp2_amd_hd_sharded_count.restype = u32
        L.nghttp2_amd_hd_sharded_encode.argtypes = [vp, vp, vp, u32, vp, sz, vp]
        L.nghttp2_amd_hd_sharded_decode.argtypes = [vp, vp, vp, u32, vp, sz, vp, vp, vp, vp]
        L._sharded_bound = True
    return L


def _ptr(a):
    import ctypes
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _padded(pool, end):
    """The pool readable to align_up(end, 16) + 16, as every batch call needs."""
    need = end + (-end) % 16 + 16
    pool = np.ascontiguousarray(pool, dtype=np.uint8)
    if pool.size >= need:
        return pool
    out = np.zeros(need, dtype=np.uint8)
    out[:pool.size] = pool
    return out


class ShardedCodec:
    """One batch over several devices in ONE process, through
    the library's sharded engine (include/nghttp2_amd_hd.h
    nghttp2_amd_hd_sharded_*): the batch is cut into byte-balanced contiguous
    shards, one per entry of `devices`; each shard runs on the engine's
    worker thread for its device, with its own HIP stream and device buffers
    (H2D, the kernels, D2H straight to the merged position), and the shards'
    offsets are rebased into one batch.  This is the reference's threading
    model (doc/programmers-guide.rst:36-40: one nghttp2 session per thread,
    no shared state) with a device behind each thread, in native code.  No
    collective: the shards never exchange data.

    `devices` may repeat a device (e.g. [0, 0]: two shards, two threads and
    two streams on one GPU).  Inputs and outputs are host numpy arrays."""

    def __init__(self, devices):
        import ctypes
        self.devices = [d if isinstance(d, int) else (d.index or 0) for d in devices]
        if not self.devices:
            raise ValueError("ShardedCodec needs at least one device")
        self.L = _lib()
        h = ctypes.c_void_p()
        ids = (ctypes.c_int * len(self.devices))(*self.devices)
        rv = self.L.nghttp2_amd_hd_sharded_new(ctypes.byref(h), ids, len(self.devices))
        if rv != 0:
            raise RuntimeError("nghttp2_amd: sharded_new failed with nghttp2 error %d" % rv)
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            self.L.nghttp2_amd_hd_sharded_del(self.h)
            self.h = None

    def encode(self, pool, off):
        """Huffman-encode the batch across the devices: returns the merged
        (encoded pool uint8, offsets uint64[n+1]), equal to a single-device
        encode of the whole batch."""
        from .hd import _check
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = len(off) - 1
        src = _padded(pool, int(off[-1]))
        cap = self.L.nghttp2_amd_hd_huff_encode_bound(int(off[-1]) - int(off[0]), n)
        dst = np.empty(cap, dtype=np.uint8)
        doff = np.empty(n + 1, dtype=np.uint32)
        _check(self.L.nghttp2_amd_hd_sharded_encode(self.h, _ptr(src), _ptr(off), n, _ptr(dst), cap,
                                                    _ptr(doff)), "sharded_encode")
        return dst[:int(doff[-1])], doff.astype(np.uint64)

    def decode_auto(self, enc_pool, enc_off):
        """Decode the batch (final=1 per string) across the devices, each
        shard in decode_batch_auto's dense layout, merged: returns (decoded
        pool uint8, dst_off uint64[n+1], status int32[n]); string i's bytes are
        pool[dst_off[i] : dst_off[i] + status[i]] when status[i] >= 0."""
        from .hd import _check
        off = np.ascontiguousarray(enc_off, dtype=np.uint32)
        n = len(off) - 1
        src = _padded(enc_pool, int(off[-1]))
        cap = self.L.nghttp2_amd_hd_huff_decode_bound(int(off[-1]) - int(off[0]), n) + 32 * len(self.devices)
        dst = np.empty(cap, dtype=np.uint8)
        doff = np.empty(n + 1, dtype=np.uint32)
        st = np.empty(max(1, n), dtype=np.int32)
        _check(self.L.nghttp2_amd_hd_sharded_decode(self.h, _ptr(src), _ptr(off), n, _ptr(dst), cap,
                                                    _ptr(doff), _ptr(st), None, None), "sharded_decode")
        return dst[:int(doff[-1])], doff.astype(np.uint64), st[:n]
