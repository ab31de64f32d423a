"""ctypes binding of include/nghttp2_amd_hd.h (the engine's C ABI).

HuffmanBatchCodec mirrors, for batches of strings, the reference's internal
Huffman API (lib/nghttp2_hd.h:385-440):

  ==========================================  ==================================
  reference (lib/nghttp2_hd_huffman.c)        batched engine call
  ==========================================  ==================================
  nghttp2_hd_huff_encode_count  :34-43        encode_count(src, src_off)
  nghttp2_hd_huff_encode        :45-104       encode(src, src_off)
  nghttp2_hd_huff_decode_context_init :106    (implicit per string)
  nghttp2_hd_huff_decode(fin=1) :111-143      decode(src, src_off) -> status
  nghttp2_hd_huff_decode_failure_state :145   fstate == 0x100
  nghttp2_huff_estimate_decode_length (.h:76) decode_slots(src_off)
  ==========================================  ==================================

Tensors are torch CUDA (HIP) tensors: uint8 pools, int32 tensors holding
uint32 offsets.  Errors follow nghttp2: negative nghttp2_error codes raise
RuntimeError; per-string decode status is an int32 tensor.
"""
import collections
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libnghttp2_amd_hd.so"

NGHTTP2_ERR_INVALID_ARGUMENT = -501
NGHTTP2_ERR_BUFFER_ERROR = -502
NGHTTP2_ERR_HEADER_COMP = -523
NGHTTP2_ERR_INSUFF_BUFSIZE = -525
NGHTTP2_ERR_FATAL = -900

_lib = None


def lib_path():
    return os.path.join(HERE, "lib", LIB_NAME)


def lib():
    """Load the HIP library; raises if it was not built (no fallback)."""
    global _lib
    if _lib is None:
        # NGHTTP2_AMD_LIB: an ablation build of the same library (tools/diag)
        path = os.environ.get("NGHTTP2_AMD_LIB") or lib_path()
        if not os.path.exists(path):
            raise RuntimeError(
                "nghttp2_amd: HIP library %s is missing -- run "
                "`python -c 'import __graft_entry__ as g; g.build()'`" % path)
        # torch first: its HIP runtime (torch/lib/libamdhip64.so, soname
        # libamdhip64.so.7) then also serves this library, so the process
        # holds ONE runtime and torch's streams are valid here.  Loaded the
        # other way round, torch brings a second runtime copy.
        import torch  # noqa: F401
        L = ctypes.CDLL(path)
        vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
        L.nghttp2_amd_hd_version.restype = ctypes.c_char_p
        L.nghttp2_amd_hd_huff_tables.argtypes = [vp, vp]
        L.nghttp2_amd_hd_huff_encode_bound.restype = sz
        L.nghttp2_amd_hd_huff_encode_bound.argtypes = [ctypes.c_uint64, u32]
        L.nghttp2_amd_hd_huff_workspace_size.restype = sz
        L.nghttp2_amd_hd_huff_workspace_size.argtypes = [u32]
        L.nghttp2_amd_hd_huff_encode_workspace_size.restype = sz
        L.nghttp2_amd_hd_huff_encode_workspace_size.argtypes = [ctypes.c_uint64, u32]
        L.nghttp2_amd_hd_huff_encode_batch.argtypes = [vp, vp, u32, vp, sz, vp, vp, sz, vp]
        L.nghttp2_amd_hd_huff_encode_count_batch.argtypes = [vp, vp, u32, vp, vp]
        L.nghttp2_amd_hd_huff_decode_slots.argtypes = [vp, u32, vp, vp, sz, vp]
        L.nghttp2_amd_hd_huff_decode_batch.argtypes = [vp, vp, u32, vp, vp, vp, vp, vp, vp]
        L.nghttp2_amd_hd_huff_decode_bound.restype = sz
        L.nghttp2_amd_hd_huff_decode_bound.argtypes = [ctypes.c_uint64, u32]
        u64 = ctypes.c_uint64
        L.nghttp2_amd_hd_huff_decode_batch_auto.argtypes = [vp, vp, u32, u64, vp, sz, vp, vp,
                                                            vp, vp, vp]
        L.nghttp2_amd_hd_huff_decode_fsm_batch.argtypes = [vp, vp, u32, vp, vp, vp, vp, vp,
                                                           vp, vp, ctypes.c_int, vp]
        L.nghttp2_amd_hd_emit_strings_bound.restype = sz
        L.nghttp2_amd_hd_emit_strings_bound.argtypes = [u64, u32]
        L.nghttp2_amd_hd_emit_strings_workspace_size.restype = sz
        L.nghttp2_amd_hd_emit_strings_workspace_size.argtypes = [u64, u32]
        L.nghttp2_amd_hd_emit_strings_batch.argtypes = [vp, vp, u32, u64, vp, sz, vp, vp, sz, vp]
        L.nghttp2_amd_hd_name_tokens_batch.argtypes = [vp, vp, u32, vp, vp, vp]
        L.nghttp2_amd_hd_lookup_token.argtypes = [ctypes.c_char_p, sz]
        L.nghttp2_amd_hd_lookup_token.restype = ctypes.c_int32
        L.nghttp2_amd_hd_name_hash.argtypes = [ctypes.c_char_p, sz]
        L.nghttp2_amd_hd_name_hash.restype = ctypes.c_uint32
        _lib = L
    return _lib


def lookup_token(name):
    """Host lookup_token (lib/nghttp2_hd.c:137): -1 or NGHTTP2_TOKEN_*."""
    name = bytes(name)
    return lib().nghttp2_amd_hd_lookup_token(name, len(name))


def name_hash(name):
    """Host FNV-1a name hash (lib/nghttp2_hd.c:536-547)."""
    name = bytes(name)
    return lib().nghttp2_amd_hd_name_hash(name, len(name))


def tables_ref_layout():
    """The engine's tables in the reference struct layouts (host-only)."""
    sym = ctypes.create_string_buffer(257 * 8)
    dec = ctypes.create_string_buffer(257 * 16 * 4)
    lib().nghttp2_amd_hd_huff_tables(sym, dec)
    return sym.raw, dec.raw


def _check(rv, what):
    if rv != 0:
        raise RuntimeError("nghttp2_amd: %s failed with nghttp2 error %d" % (what, rv))


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class HuffmanBatchCodec:
    """Batched HPACK Huffman codec on one device.

    All calls are asynchronous on the given (default: current) torch stream.
    A codec may be used from several streams: each stream gets its own device
    workspaces (tile sums, the framing pool), allocated on that stream and
    grown there, so calls on different streams never share scratch and a
    regrown block is only reused in the order of its own stream.  Calls on one
    stream run in issue order, as any work on a stream does.
    """

    _SCRATCH_KEEP = 16  # per-stream workspaces kept (two kinds per stream)

    def __init__(self, device=None):
        import torch
        self.torch = torch
        self.device = torch.device(device if device is not None else "cuda")
        self.L = lib()
        # (stream handle, kind) -> uint8 tensor allocated on that stream; the
        # least recently used entries past _SCRATCH_KEEP are dropped, so
        # short-lived streams do not pin device workspace (a dropped block
        # returns to the caching allocator on the stream it was allocated on)
        self._scratch = collections.OrderedDict()

    def _on(self, stream):
        return stream if stream is not None else self.torch.cuda.current_stream(self.device)

    def _scratch_for(self, kind, need, stream):
        s = self._on(stream)
        key = (s.cuda_stream, kind)
        t = self._scratch.get(key)
        if t is not None:
            self._scratch.move_to_end(key)
        if t is None or t.numel() < need:
            # Uninitialised on purpose: the kernels write every scratch word
            # they read (a zero fill would be one more kernel).  Allocated
            # under the call's own stream, so the caching allocator ties the
            # block to it.
            with self.torch.cuda.stream(s):
                t = self.torch.empty(need, dtype=self.torch.uint8, device=self.device)
            self._scratch[key] = t
            while len(self._scratch) > self._SCRATCH_KEEP:
                self._scratch.popitem(last=False)
        return t

    def _empty(self, n, dtype, stream):
        """An output tensor allocated under the call's stream (so the caching
        allocator never hands its block to another stream while the call's
        kernels may still write it)."""
        with self.torch.cuda.stream(self._on(stream)):
            return self.torch.empty(n, dtype=dtype, device=self.device)

    def _workspace(self, n, raw_bytes=None, stream=None):
        return self._scratch_for("ws", self.L.nghttp2_amd_hd_huff_workspace_size(n), stream)

    def encode_bound(self, raw_bytes, n):
        return self.L.nghttp2_amd_hd_huff_encode_bound(int(raw_bytes), int(n))

    def encode(self, src, src_off, raw_bytes=None, dst=None, dst_off=None, stream=None):
        """Encode strings; returns (dst pool, dst_off int32[n+1])."""
        torch = self.torch
        n = src_off.numel() - 1
        if raw_bytes is None:
            raw_bytes = src.numel()
        cap = self.encode_bound(raw_bytes, n)
        if dst is None:
            dst = self._empty(cap, torch.uint8, stream)
        if dst_off is None:
            dst_off = self._empty(n + 1, torch.int32, stream)
        ws = self._workspace(n, raw_bytes, stream)
        rv = self.L.nghttp2_amd_hd_huff_encode_batch(
            _p(src), _p(src_off), n, _p(dst), dst.numel(), _p(dst_off), _p(ws),
            ws.numel(), _stream(stream))
        _check(rv, "encode_batch")
        return dst, dst_off

    def encode_count(self, src, src_off, enc_len=None, stream=None):
        n = src_off.numel() - 1
        if enc_len is None:
            enc_len = self._empty(max(1, n), self.torch.int32, stream)
        rv = self.L.nghttp2_amd_hd_huff_encode_count_batch(
            _p(src), _p(src_off), n, _p(enc_len), _stream(stream))
        _check(rv, "encode_count_batch")
        return enc_len[:n]

    def name_tokens(self, names, name_off, token=None, hash=None, stream=None):
        """lookup_token + name_hash (lib/nghttp2_hd.c:137, :536) for every
        name of the batch: returns (token int32[n], hash int32[n] holding the
        uint32 FNV-1a bits)."""
        torch = self.torch
        n = name_off.numel() - 1
        if token is None:
            token = self._empty(max(1, n), torch.int32, stream)
        if hash is None:
            hash = self._empty(max(1, n), torch.int32, stream)
        rv = self.L.nghttp2_amd_hd_name_tokens_batch(
            _p(names), _p(name_off), n, _p(token), _p(hash), _stream(stream))
        _check(rv, "name_tokens_batch")
        return token[:n], hash[:n]

    def emit_strings(self, src, src_off, raw_bytes=None, dst=None, dst_off=None, stream=None):
        """HPACK string literals (emit_string, lib/nghttp2_hd.c:1001-1044) for
        every string: returns (dst pool, dst_off int32[n+1]); literal i is
        dst[dst_off[i]:dst_off[i+1]]."""
        torch = self.torch
        n = src_off.numel() - 1
        if raw_bytes is None:
            raw_bytes = src.numel()
        cap = self.L.nghttp2_amd_hd_emit_strings_bound(int(raw_bytes), n)
        if dst is None:
            dst = self._empty(cap, torch.uint8, stream)
        if dst_off is None:
            dst_off = self._empty(n + 1, torch.int32, stream)
        need = self.L.nghttp2_amd_hd_emit_strings_workspace_size(int(raw_bytes), n)
        ews = self._scratch_for("ews", need, stream)
        rv = self.L.nghttp2_amd_hd_emit_strings_batch(
            _p(src), _p(src_off), n, int(raw_bytes), _p(dst), dst.numel(), _p(dst_off),
            _p(ews), ews.numel(), _stream(stream))
        _check(rv, "emit_strings_batch")
        return dst, dst_off

    def decode_slots(self, src_off, dst_off=None, stream=None):
        n = src_off.numel() - 1
        if dst_off is None:
            dst_off = self._empty(n + 1, self.torch.int32, stream)
        ws = self._workspace(n, stream=stream)
        rv = self.L.nghttp2_amd_hd_huff_decode_slots(
            _p(src_off), n, _p(dst_off), _p(ws), ws.numel(), _stream(stream))
        _check(rv, "decode_slots")
        return dst_off

    def decode_bound(self, enc_bytes, n):
        return self.L.nghttp2_amd_hd_huff_decode_bound(int(enc_bytes), int(n))

    def decode_auto(self, src, src_off, enc_bytes=None, dst=None, dst_off=None, status=None,
                    want_ctx=False, stream=None, pick=None):
        """Decode into a dense pool (one launch): the strings of each task of
        64 consecutive strings (or of a task split into two of 32) back to
        back from the task's base auto_slot(x_t0, t0).  enc_bytes = src_off[n] - src_off[0] sizes dst and
        picks the kernel instance by the mean string length; when it is not
        given it is read from src_off on the call's stream (a host
        synchronisation of that stream: pass it to keep the call
        asynchronous).  pick = "items64" (the short-string instance: whole
        strings of up to 96 bytes as one item since round 6) / "pieces40" forces one instance
        through that same argument (tests).  Returns
        (dst, dst_off, status[, fstate, flags])."""
        torch = self.torch
        n = src_off.numel() - 1
        if enc_bytes is None:
            with torch.cuda.stream(self._on(stream)):
                ends = src_off[[0, n]].cpu().numpy().view("uint32").astype("int64")
            enc_bytes = int(ends[1] - ends[0])
        sel = {None: int(enc_bytes), "items64": 0, "pieces40": 49 * max(1, n)}[pick]
        if dst is None:
            dst = self._empty(self.decode_bound(enc_bytes, n), torch.uint8, stream)
        if dst_off is None:
            dst_off = self._empty(n + 1, torch.int32, stream)
        if status is None:
            status = self._empty(max(1, n), torch.int32, stream)
        fstate = flags = None
        if want_ctx:
            fstate = self._empty(max(1, n), torch.int16, stream)
            flags = self._empty(max(1, n), torch.uint8, stream)
        rv = self.L.nghttp2_amd_hd_huff_decode_batch_auto(
            _p(src), _p(src_off), n, sel, _p(dst), dst.numel(), _p(dst_off), _p(status),
            _p(fstate), _p(flags), _stream(stream))
        _check(rv, "decode_batch_auto")
        if want_ctx:
            return dst, dst_off, status[:n], fstate[:n], flags[:n]
        return dst, dst_off, status[:n]

    def decode_fsm(self, src, src_off, dst_off, dst, init_fstate=None, init_flags=None,
                   final=True, stream=None):
        """The reference nibble FSM, batched (streaming-capable).  Returns
        (status, fstate, flags)."""
        torch = self.torch
        n = src_off.numel() - 1
        status = self._empty(max(1, n), torch.int32, stream)
        fstate = self._empty(max(1, n), torch.int16, stream)
        flags = self._empty(max(1, n), torch.uint8, stream)
        rv = self.L.nghttp2_amd_hd_huff_decode_fsm_batch(
            _p(src), _p(src_off), n, _p(dst), _p(dst_off), _p(status), _p(fstate),
            _p(flags), _p(init_fstate), _p(init_flags), 1 if final else 0, _stream(stream))
        _check(rv, "decode_fsm_batch")
        return status[:n], fstate[:n], flags[:n]

    def decode(self, src, src_off, dst_off=None, dst=None, dst_cap=None, status=None,
               want_ctx=False, stream=None):
        """Decode strings (fin=1 each).  Returns (dst, dst_off, status[, fstate, flags]).

        dst_off defaults to the reference's floor(8E/5)+1 slots; dst_cap must
        then be given (or is derived from src size: 8*E_total/5 + n + 16).
        """
        torch = self.torch
        n = src_off.numel() - 1
        if dst_off is None:
            dst_off = self.decode_slots(src_off, stream=stream)
            if dst_cap is None:
                dst_cap = (src.numel() * 8) // 5 + n + 16
        if dst is None:
            if dst_cap is None:
                dst_cap = int(dst_off[-1].item()) + 16
            dst = self._empty(dst_cap, torch.uint8, stream)
        if status is None:
            status = self._empty(max(1, n), torch.int32, stream)
        fstate = flags = None
        if want_ctx:
            fstate = self._empty(max(1, n), torch.int16, stream)
            flags = self._empty(max(1, n), torch.uint8, stream)
        rv = self.L.nghttp2_amd_hd_huff_decode_batch(
            _p(src), _p(src_off), n, _p(dst), _p(dst_off), _p(status), _p(fstate),
            _p(flags), _stream(stream))
        _check(rv, "decode_batch")
        if want_ctx:
            return dst, dst_off, status[:n], fstate[:n], flags[:n]
        return dst, dst_off, status[:n]


# ---------------------------------------------------------------------------
# Batched HPACK inflate front-end (nghttp2_amd_hd_inflate_*)
# ---------------------------------------------------------------------------
class _Nv(ctypes.Structure):
    _fields_ = [("block", ctypes.c_uint32), ("name_off", ctypes.c_uint32),
                ("name_len", ctypes.c_uint32), ("value_off", ctypes.c_uint32),
                ("value_len", ctypes.c_uint32), ("flags", ctypes.c_uint8)]


def _inflate_lib():
    L = lib()
    if not getattr(L, "_inflate_bound", False):
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.nghttp2_amd_hd_inflate_new.argtypes = [ctypes.POINTER(vp)]
        L.nghttp2_amd_hd_inflate_del.argtypes = [vp]
        L.nghttp2_amd_hd_inflate_del.restype = None
        L.nghttp2_amd_hd_inflate_change_table_size.argtypes = [vp, sz]
        L.nghttp2_amd_hd_inflate_get_num_table_entries.argtypes = [vp]
        L.nghttp2_amd_hd_inflate_get_num_table_entries.restype = sz
        L.nghttp2_amd_hd_inflate_get_table_entry.argtypes = [
            vp, sz, ctypes.POINTER(vp), ctypes.POINTER(sz), ctypes.POINTER(vp), ctypes.POINTER(sz)]
        L.nghttp2_amd_hd_inflate_get_dynamic_table_size.argtypes = [vp]
        L.nghttp2_amd_hd_inflate_get_dynamic_table_size.restype = sz
        L.nghttp2_amd_hd_inflate_get_max_dynamic_table_size.argtypes = [vp]
        L.nghttp2_amd_hd_inflate_get_max_dynamic_table_size.restype = sz
        L.nghttp2_amd_hd_inflate_blocks.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, sz,
                                                    ctypes.POINTER(sz), vp, sz,
                                                    ctypes.POINTER(sz), vp, vp]
        L._inflate_bound = True
    return L


class HpackInflater:
    """One connection's HPACK decoding context (nghttp2_hd_inflater)."""

    def __init__(self):
        self.L = _inflate_lib()
        p = ctypes.c_void_p()
        _check(self.L.nghttp2_amd_hd_inflate_new(ctypes.byref(p)), "inflate_new")
        self.p = p

    def __del__(self):
        if getattr(self, "p", None):
            self.L.nghttp2_amd_hd_inflate_del(self.p)
            self.p = None

    def change_table_size(self, settings_max):
        _check(self.L.nghttp2_amd_hd_inflate_change_table_size(self.p, settings_max),
               "inflate_change_table_size")

    def dynamic_table(self):
        """[(name, value)] of the dynamic table, most recent first."""
        out = []
        n = self.L.nghttp2_amd_hd_inflate_get_num_table_entries(self.p)
        for idx in range(62, n + 1):
            a, b = ctypes.c_void_p(), ctypes.c_void_p()
            la, lb = ctypes.c_size_t(), ctypes.c_size_t()
            _check(self.L.nghttp2_amd_hd_inflate_get_table_entry(
                self.p, idx, ctypes.byref(a), ctypes.byref(la), ctypes.byref(b),
                ctypes.byref(lb)), "inflate_get_table_entry")
            out.append((ctypes.string_at(a, la.value) if la.value else b"",
                        ctypes.string_at(b, lb.value) if lb.value else b""))
        return out

    def dynamic_table_size(self):
        return self.L.nghttp2_amd_hd_inflate_get_dynamic_table_size(self.p)

    def max_dynamic_table_size(self):
        """nghttp2_hd_inflate_get_max_dynamic_table_size: the table limit in
        force (the reference's ctx.hd_table_bufsize_max)."""
        return self.L.nghttp2_amd_hd_inflate_get_max_dynamic_table_size(self.p)

    def num_table_entries(self):
        """nghttp2_hd_inflate_get_num_table_entries: static (61) + dynamic."""
        return self.L.nghttp2_amd_hd_inflate_get_num_table_entries(self.p)


_NV_DTYPE = np.dtype([("block", "<u4"), ("name_off", "<u4"), ("name_len", "<u4"),
                      ("value_off", "<u4"), ("value_len", "<u4"), ("flags", "u1")], align=True)
assert _NV_DTYPE.itemsize == ctypes.sizeof(_Nv)


def inflate_blocks(inflaters, blocks, stream=None, nva_cap=None, arena_cap=None, retry=True):
    """Inflate complete header blocks, block i against inflaters[i], with
    every Huffman literal decoded in one GPU batch.  Returns
    (status[i], fields[i] = [(name, value, flags)]).  A batch that outgrows
    the field/arena buffers is cut at the first block that does not fit
    (status NGHTTP2_ERR_BUFFER_ERROR from there on, those blocks not
    applied); with retry the rest is resubmitted with buffers twice the size.
    The blocks go in as one joined buffer and the fields come out of
    uninitialised numpy buffers (no per-block ctypes objects, no zero fill)."""
    L = _inflate_lib()
    nb = len(blocks)
    joined = b"".join(bytes(b) for b in blocks)
    total = len(joined)
    lens_all = np.fromiter((len(b) for b in blocks), dtype=np.uint64, count=nb)
    starts = np.zeros(nb, dtype=np.uint64)
    if nb > 1:
        np.cumsum(lens_all[:-1], out=starts[1:])
    pool = np.frombuffer(joined, dtype=np.uint8) if total else np.zeros(1, dtype=np.uint8)
    ptrs_all = starts + np.uint64(pool.ctypes.data)
    infs_all = np.fromiter((i.p.value for i in inflaters), dtype=np.uint64, count=nb)
    nva_cap = total + 16 if nva_cap is None else nva_cap
    arena_cap = 8 * total + 64 * (total + 16) + 4096 if arena_cap is None else arena_cap
    s = None
    if stream is not None:
        s = ctypes.c_void_p(stream.cuda_stream)
    else:
        try:
            import torch
            if torch.cuda.is_available():
                s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        except Exception:  # pragma: no cover - torch is part of the image
            s = None
    status = [NGHTTP2_ERR_BUFFER_ERROR] * nb
    fields = [[] for _ in range(nb)]
    first = 0
    vp = ctypes.c_void_p
    while first < nb:
        m = nb - first
        ptrs = np.ascontiguousarray(ptrs_all[first:])
        lens = np.ascontiguousarray(lens_all[first:])
        infs = np.ascontiguousarray(infs_all[first:])
        nva = np.empty(max(1, nva_cap), dtype=_NV_DTYPE)
        arena = np.empty(max(1, arena_cap), dtype=np.uint8)
        st = np.empty(m, dtype=np.int32)
        nv_used, ar_used = ctypes.c_size_t(), ctypes.c_size_t()
        rv = L.nghttp2_amd_hd_inflate_blocks(vp(infs.ctypes.data), m, vp(ptrs.ctypes.data),
                                             vp(lens.ctypes.data), vp(nva.ctypes.data), nva_cap,
                                             ctypes.byref(nv_used), vp(arena.ctypes.data), arena_cap,
                                             ctypes.byref(ar_used), vp(st.ctypes.data), s)
        if rv != NGHTTP2_ERR_BUFFER_ERROR:
            _check(rv, "inflate_blocks")
        raw = arena[:ar_used.value].tobytes()
        nv = nva[:nv_used.value]
        for b, no, nl, vo, vl, fl in zip((nv["block"] + first).tolist(), nv["name_off"].tolist(),
                                         nv["name_len"].tolist(), nv["value_off"].tolist(),
                                         nv["value_len"].tolist(), nv["flags"].tolist()):
            fields[b].append((raw[no:no + nl], raw[vo:vo + vl], fl))
        stl = st.tolist()
        done = 0
        while done < m and stl[done] != NGHTTP2_ERR_BUFFER_ERROR:
            status[first + done] = stl[done]
            done += 1
        first += done
        if done < m:
            if not retry:
                break
            if done == 0:
                nva_cap, arena_cap = 2 * nva_cap + 16, 2 * arena_cap + 4096
    return status, fields


# ---------------------------------------------------------------------------
# Batched HPACK deflate front-end (nghttp2_amd_hd_deflate_*)
# ---------------------------------------------------------------------------
class _NvIn(ctypes.Structure):
    _fields_ = [("name", ctypes.c_void_p), ("value", ctypes.c_void_p),
                ("namelen", ctypes.c_size_t), ("valuelen", ctypes.c_size_t),
                ("flags", ctypes.c_uint8)]


_NVIN_DTYPE = np.dtype([("name", "<u8"), ("value", "<u8"), ("namelen", "<u8"),
                        ("valuelen", "<u8"), ("flags", "u1")], align=True)
assert _NVIN_DTYPE.itemsize == ctypes.sizeof(_NvIn)


def _deflate_lib():
    L = _inflate_lib()
    if not getattr(L, "_deflate_bound", False):
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.nghttp2_amd_hd_deflate_new.argtypes = [ctypes.POINTER(vp), sz]
        L.nghttp2_amd_hd_deflate_del.argtypes = [vp]
        L.nghttp2_amd_hd_deflate_del.restype = None
        L.nghttp2_amd_hd_deflate_change_table_size.argtypes = [vp, sz]
        L.nghttp2_amd_hd_deflate_get_num_table_entries.argtypes = [vp]
        L.nghttp2_amd_hd_deflate_get_num_table_entries.restype = sz
        L.nghttp2_amd_hd_deflate_get_table_entry.argtypes = [
            vp, sz, ctypes.POINTER(vp), ctypes.POINTER(sz), ctypes.POINTER(vp), ctypes.POINTER(sz)]
        L.nghttp2_amd_hd_deflate_get_dynamic_table_size.argtypes = [vp]
        L.nghttp2_amd_hd_deflate_get_dynamic_table_size.restype = sz
        L.nghttp2_amd_hd_deflate_blocks.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, sz, vp, vp, vp]
        L.nghttp2_amd_hd_deflate_get_max_dynamic_table_size.argtypes = [vp]
        L.nghttp2_amd_hd_deflate_get_max_dynamic_table_size.restype = sz
        L.nghttp2_amd_hd_deflate_bound.argtypes = [vp, vp, sz]
        L.nghttp2_amd_hd_deflate_bound.restype = sz
        L.nghttp2_amd_hd_deflate_hd2.argtypes = [vp, vp, sz, vp, sz, vp]
        L.nghttp2_amd_hd_deflate_hd2.restype = ctypes.c_ssize_t
        L.nghttp2_amd_hd_deflate_hd_vec2.argtypes = [vp, vp, sz, vp, sz, vp]
        L.nghttp2_amd_hd_deflate_hd_vec2.restype = ctypes.c_ssize_t
        L.nghttp2_amd_hd_decode_length.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(sz),
                                                   ctypes.POINTER(ctypes.c_int), ctypes.c_uint32, sz,
                                                   vp, vp, sz]
        L.nghttp2_amd_hd_decode_length.restype = ctypes.c_ssize_t
        L._deflate_bound = True
    return L


class HpackDeflater:
    """One connection's HPACK encoding context (nghttp2_hd_deflater)."""

    def __init__(self, max_deflate_table_size=4096):
        self.L = _deflate_lib()
        p = ctypes.c_void_p()
        _check(self.L.nghttp2_amd_hd_deflate_new(ctypes.byref(p), max_deflate_table_size),
               "deflate_new")
        self.p = p

    def __del__(self):
        if getattr(self, "p", None):
            self.L.nghttp2_amd_hd_deflate_del(self.p)
            self.p = None

    def change_table_size(self, settings_max):
        _check(self.L.nghttp2_amd_hd_deflate_change_table_size(self.p, settings_max),
               "deflate_change_table_size")

    def dynamic_table(self):
        out = []
        n = self.L.nghttp2_amd_hd_deflate_get_num_table_entries(self.p)
        for idx in range(62, n + 1):
            a, b = ctypes.c_void_p(), ctypes.c_void_p()
            la, lb = ctypes.c_size_t(), ctypes.c_size_t()
            _check(self.L.nghttp2_amd_hd_deflate_get_table_entry(
                self.p, idx, ctypes.byref(a), ctypes.byref(la), ctypes.byref(b),
                ctypes.byref(lb)), "deflate_get_table_entry")
            out.append((ctypes.string_at(a, la.value) if la.value else b"",
                        ctypes.string_at(b, lb.value) if lb.value else b""))
        return out

    def dynamic_table_size(self):
        return self.L.nghttp2_amd_hd_deflate_get_dynamic_table_size(self.p)

    def max_dynamic_table_size(self):
        """nghttp2_hd_deflate_get_max_dynamic_table_size (the reference's
        ctx.hd_table_bufsize_max)."""
        return self.L.nghttp2_amd_hd_deflate_get_max_dynamic_table_size(self.p)

    def num_table_entries(self):
        return self.L.nghttp2_amd_hd_deflate_get_num_table_entries(self.p)

    def bound(self, header_list):
        """nghttp2_hd_deflate_bound of one list."""
        nva, keep = _nv_array(header_list)
        return self.L.nghttp2_amd_hd_deflate_bound(self.p, nva.ctypes.data, len(header_list))

    def deflate_hd2(self, header_list, buflen, stream=None):
        """nghttp2_hd_deflate_hd2 into a buffer of buflen bytes: (rv, wire);
        rv is the length or NGHTTP2_ERR_INSUFF_BUFSIZE / HEADER_COMP."""
        nva, keep = _nv_array(header_list)
        buf = np.zeros(max(1, buflen), dtype=np.uint8)
        rv = self.L.nghttp2_amd_hd_deflate_hd2(self.p, buf.ctypes.data, buflen, nva.ctypes.data,
                                               len(header_list), _cur_stream(stream))
        return rv, (buf[:rv].tobytes() if rv >= 0 else b"")

    def deflate_hd_vec2(self, header_list, chunk_lens, stream=None):
        """nghttp2_hd_deflate_hd_vec2 over chunks of the given lengths (None:
        a NULL vector of length 0): (rv, [chunk bytes])."""
        nva, keep = _nv_array(header_list)
        if chunk_lens is None:
            rv = self.L.nghttp2_amd_hd_deflate_hd_vec2(self.p, None, 0, nva.ctypes.data,
                                                       len(header_list), _cur_stream(stream))
            return rv, []
        bufs = [np.zeros(max(1, n), dtype=np.uint8) for n in chunk_lens]
        vec = (_Vec * max(1, len(chunk_lens)))()
        for k, (b, n) in enumerate(zip(bufs, chunk_lens)):
            vec[k].base = b.ctypes.data if n else None
            vec[k].len = n
        rv = self.L.nghttp2_amd_hd_deflate_hd_vec2(self.p, vec, len(chunk_lens), nva.ctypes.data,
                                                   len(header_list), _cur_stream(stream))
        return rv, [b[:n].tobytes() for b, n in zip(bufs, chunk_lens)]


class _Vec(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("len", ctypes.c_size_t)]


def _cur_stream(stream):
    if stream is not None:
        return ctypes.c_void_p(stream.cuda_stream)
    import torch
    if torch.cuda.is_available():
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    return None


def _nv_array(header_list):
    """An nghttp2_nv-layout array over one list's (name, value[, flags]);
    returns (array, buffers kept alive)."""
    nva = np.zeros(max(1, len(header_list)), dtype=_NVIN_DTYPE)
    keep = []
    for k, h in enumerate(header_list):
        n, v = np.frombuffer(bytes(h[0]) + b"\0", np.uint8), np.frombuffer(bytes(h[1]) + b"\0", np.uint8)
        keep += [n, v]
        nva[k] = (n.ctypes.data, v.ctypes.data, len(h[0]), len(h[1]), h[2] if len(h) > 2 else 0)
    return nva, keep


def decode_length(data, prefix, initial=0, shift=0):
    """nghttp2_hd_decode_length over bytes `data`: (rv, value, shift, fin)."""
    L = _deflate_lib()
    buf = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)
    res, sh, fin = ctypes.c_uint32(), ctypes.c_size_t(), ctypes.c_int()
    base = buf.ctypes.data
    rv = L.nghttp2_amd_hd_decode_length(ctypes.byref(res), ctypes.byref(sh), ctypes.byref(fin),
                                        initial, shift, base, base + len(data), prefix)
    return rv, res.value, sh.value, fin.value


def deflate_blocks(deflaters, header_lists, stream=None, out_cap=None):
    """Encode header lists (each [(name, value[, flags])]), list i with
    deflaters[i]; every literal framed in one GPU batch.  Returns
    (status[i], wire[i]).  out_cap (default: room for every list) limits the
    output: a list that does not fit gets NGHTTP2_ERR_BUFFER_ERROR and its
    deflater turns bad."""
    L = _deflate_lib()
    nb = len(header_lists)
    flat = [(bytes(h[0]), bytes(h[1]), (h[2] if len(h) > 2 else 0))
            for hl in header_lists for h in hl]
    nf = len(flat)
    # every name and value in one joined buffer; the nv array (nghttp2_nv
    # layout) points into it -- no ctypes object per field
    parts = [x for n_, v_, _ in flat for x in (n_, v_)]
    joined = b"".join(parts)
    plen = np.fromiter((len(x) for x in parts), dtype=np.uint64, count=2 * nf)
    pstart = np.zeros(2 * nf, dtype=np.uint64)
    if nf:
        np.cumsum(plen[:-1], out=pstart[1:])
    pool = np.frombuffer(joined, dtype=np.uint8) if joined else np.zeros(1, dtype=np.uint8)
    nva = np.zeros(max(1, nf), dtype=_NVIN_DTYPE)
    if nf:
        base = np.uint64(pool.ctypes.data)
        nva["name"][:nf] = pstart[0::2] + base
        nva["value"][:nf] = pstart[1::2] + base
        nva["namelen"][:nf] = plen[0::2]
        nva["valuelen"][:nf] = plen[1::2]
        nva["flags"][:nf] = np.fromiter((f for _, _, f in flat), dtype=np.uint8, count=nf)
    offs = np.zeros(nb + 1, dtype=np.uint32)
    if nb:
        np.cumsum(np.fromiter((len(hl) for hl in header_lists), dtype=np.uint32, count=nb),
                  out=offs[1:])
    cap = int(plen.sum()) + 16 * nf + 16 * nb + 64 if out_cap is None else out_cap
    out = np.empty(max(1, cap), dtype=np.uint8)
    out_off = np.zeros(nb + 1, dtype=np.uint32)
    st = np.zeros(max(1, nb), dtype=np.int32)
    defl = np.fromiter((d.p.value for d in deflaters), dtype=np.uint64, count=nb) if nb \
        else np.zeros(1, dtype=np.uint64)
    s = None
    if stream is not None:
        s = ctypes.c_void_p(stream.cuda_stream)
    else:
        import torch
        if torch.cuda.is_available():
            s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    vp = ctypes.c_void_p
    rv = L.nghttp2_amd_hd_deflate_blocks(vp(defl.ctypes.data), nb, vp(nva.ctypes.data),
                                         vp(offs.ctypes.data), vp(out.ctypes.data), cap,
                                         vp(out_off.ctypes.data), vp(st.ctypes.data), s)
    if rv not in (0, NGHTTP2_ERR_BUFFER_ERROR):
        _check(rv, "deflate_blocks")
    oo = out_off.tolist()
    raw = out[:oo[nb]].tobytes()
    return st[:nb].tolist(), [raw[oo[i]:oo[i + 1]] for i in range(nb)]
