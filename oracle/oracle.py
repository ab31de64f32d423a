"""ctypes wrapper for the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / CPU baseline.  The product
package (nghttp2_amd) never imports it.

Every function mirrors a reference function (see oracle/huff_oracle.c for the
file:line citations into /root/reference/lib/nghttp2_hd_huffman.c).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libhuff_oracle.so")

NGHTTP2_ERR_BUFFER_ERROR = -502
NGHTTP2_ERR_HEADER_COMP = -523
ACCEPTED = 0x01
SYM = 0x02

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.orc_init.restype = ctypes.c_int
        L.orc_sym_table.restype = ctypes.c_void_p
        L.orc_dec_table.restype = ctypes.c_void_p
        L.orc_encode_count.restype = ctypes.c_size_t
        L.orc_encode_count.argtypes = [u8p, ctypes.c_size_t]
        L.orc_encode.restype = ctypes.c_int
        L.orc_encode.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t,
                                 ctypes.POINTER(ctypes.c_size_t)]
        L.orc_decode.restype = ctypes.c_long
        L.orc_decode.argtypes = [ctypes.c_void_p, u8p,
                                 ctypes.POINTER(ctypes.c_size_t), u8p,
                                 ctypes.c_size_t, ctypes.c_int]
        L.orc_decode_failure_state.restype = ctypes.c_int
        L.orc_decode_failure_state.argtypes = [ctypes.c_void_p]
        vp = ctypes.c_void_p
        L.orc_encode_count_batch.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_int]
        L.orc_encode_batch.argtypes = [vp, vp, ctypes.c_uint32, vp, vp, vp, ctypes.c_int]
        L.orc_decode_batch.argtypes = [vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp,
                                       ctypes.c_int]
        L.orc_roundtrip_timed.argtypes = [vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp,
                                          ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_double)]
        L.orc_count_encoded_length.restype = ctypes.c_size_t
        L.orc_count_encoded_length.argtypes = [ctypes.c_size_t, ctypes.c_size_t]
        L.orc_encode_length.restype = ctypes.c_size_t
        L.orc_encode_length.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t]
        L.orc_emit_string.restype = ctypes.c_size_t
        L.orc_emit_string.argtypes = [u8p, u8p, ctypes.c_size_t]
        L.orc_emit_strings_batch.argtypes = [vp, vp, ctypes.c_uint32, vp, vp]
        if L.orc_init() != 0:
            raise RuntimeError("oracle table construction failed")
        _lib = L
    return _lib


class Ctx(ctypes.Structure):
    """nghttp2_hd_huff_decode_context (lib/nghttp2_hd_huffman.h:56-60)."""
    _fields_ = [("fstate", ctypes.c_uint16), ("flags", ctypes.c_uint8)]


def _buf(b):
    b = bytes(b)
    return (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b + b"\0"), len(b)


def tables_ref_layout():
    """(sym_bytes, dec_bytes) in the reference's struct layouts."""
    L = lib()
    sym = ctypes.string_at(L.orc_sym_table(), 257 * 8)
    dec = ctypes.string_at(L.orc_dec_table(), 257 * 16 * 4)
    return sym, dec


def encode_count(data):
    p, n = _buf(data)
    return lib().orc_encode_count(p, n)


def encode(data, cap=None):
    """Returns (rv, bytes written).  cap=None: unbounded buffer."""
    p, n = _buf(data)
    if cap is None:
        cap = (n * 30 + 7) // 8 + 8
    out = (ctypes.c_uint8 * max(1, cap))()
    w = ctypes.c_size_t(0)
    rv = lib().orc_encode(out, cap, p, n, ctypes.byref(w))
    return rv, bytes(out[:w.value])


def decode(data, final=1, ctx=None):
    """nghttp2_hd_huff_decode.  Returns (rv, output bytes, ctx)."""
    if ctx is None:
        ctx = Ctx(0, ACCEPTED)
    p, n = _buf(data)
    out = (ctypes.c_uint8 * (n * 8 // 5 + 1))()
    w = ctypes.c_size_t(0)
    rv = lib().orc_decode(ctypes.byref(ctx), out, ctypes.byref(w), p, n, final)
    return rv, bytes(out[:w.value]), ctx


def failure_state(ctx):
    return bool(lib().orc_decode_failure_state(ctypes.byref(ctx)))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def encode_batch(pool, off, nthreads=1):
    """Batch count+encode. Returns (enc_pool u8, enc_off u32[n+1])."""
    pool = np.ascontiguousarray(pool, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    n = len(off) - 1
    enc_len = np.zeros(n, dtype=np.uint32)
    lib().orc_encode_count_batch(_ptr(pool), _ptr(off), n, _ptr(enc_len), nthreads)
    enc_off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(enc_len, out=enc_off[1:])
    assert enc_off[-1] < 2**32
    enc_off = enc_off.astype(np.uint32)
    enc = np.zeros(max(1, int(enc_off[-1])), dtype=np.uint8)
    status = np.zeros(n, dtype=np.int32)
    lib().orc_encode_batch(_ptr(pool), _ptr(off), n, _ptr(enc_off), _ptr(enc),
                           _ptr(status), nthreads)
    assert not status.any()
    return enc[:int(enc_off[-1])], enc_off


def decode_bound_offsets(enc_off):
    """Output slots of floor(8E/5)+1 bytes (the reference's allocation,
    lib/nghttp2_hd.c:2080-2082 via nghttp2_huff_estimate_decode_length)."""
    enc_off = np.asarray(enc_off, dtype=np.int64)
    cap = (np.diff(enc_off) * 8) // 5 + 1
    out = np.zeros(len(enc_off), dtype=np.uint64)
    np.cumsum(cap, out=out[1:])
    return out.astype(np.uint32)


def decode_batch(enc, enc_off, dst_off=None, nthreads=1):
    """Batch decode with final=1.  Returns (dst, dst_off, status, fstate, flags);
    status[i] = decoded length or NGHTTP2_ERR_HEADER_COMP."""
    enc = np.ascontiguousarray(enc, dtype=np.uint8)
    if enc.size == 0:
        enc = np.zeros(1, dtype=np.uint8)
    enc_off = np.ascontiguousarray(enc_off, dtype=np.uint32)
    n = len(enc_off) - 1
    if dst_off is None:
        dst_off = decode_bound_offsets(enc_off)
    dst_off = np.ascontiguousarray(dst_off, dtype=np.uint32)
    dst = np.zeros(max(1, int(dst_off[-1])), dtype=np.uint8)
    status = np.zeros(n, dtype=np.int32)
    fstate = np.zeros(n, dtype=np.uint16)
    flags = np.zeros(n, dtype=np.uint8)
    lib().orc_decode_batch(_ptr(enc), _ptr(enc_off), n, _ptr(dst_off), _ptr(dst),
                           _ptr(status), _ptr(fstate), _ptr(flags), nthreads)
    return dst, dst_off, status, fstate, flags


def encode_length(n, prefix, first=0):
    """encode_length (lib/nghttp2_hd.c:840-863): the RFC 7541 5.1 prefix
    integer, keeping the bits of `first` above the prefix."""
    buf = (ctypes.c_uint8 * 16)(first)
    k = lib().orc_encode_length(buf, n, prefix)
    return bytes(buf[:k])


def emit_string(data):
    """emit_string (lib/nghttp2_hd.c:1001-1044): one HPACK string literal."""
    p, n = _buf(data)
    out = (ctypes.c_uint8 * (n + 16))()
    k = lib().orc_emit_string(out, p, n)
    return bytes(out[:k])


def emit_strings_batch(pool, off):
    """Batch of string literals back to back.  Returns (dst u8, dst_off u32[n+1])."""
    pool = np.ascontiguousarray(pool, dtype=np.uint8)
    if pool.size == 0:
        pool = np.zeros(1, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    n = len(off) - 1
    raw = int(off[-1]) - int(off[0]) if n else 0
    dst = np.zeros(raw + 6 * n + 16, dtype=np.uint8)
    dst_off = np.zeros(n + 1, dtype=np.uint32)
    lib().orc_emit_strings_batch(_ptr(pool), _ptr(off), n, _ptr(dst), _ptr(dst_off))
    return dst[:int(dst_off[-1])], dst_off


def roundtrip_timed(pool, off, nthreads=1):
    """Times count+encode and decode (final=1) over the batch; returns
    (t_enc, t_dec, enc_total_bytes, status)."""
    pool = np.ascontiguousarray(pool, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    n = len(off) - 1
    raw = np.diff(off.astype(np.int64))
    enc_off = np.zeros(n + 1, dtype=np.uint32)
    enc = np.zeros(int((raw * 30 + 7).sum() // 8) + 16, dtype=np.uint8)
    dec_off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(raw + 1, out=dec_off[1:])
    dec_off = dec_off.astype(np.uint32)
    dec = np.zeros(int(dec_off[-1]) + 1, dtype=np.uint8)
    status = np.zeros(n, dtype=np.int32)
    te, td = ctypes.c_double(0), ctypes.c_double(0)
    lib().orc_roundtrip_timed(_ptr(pool), _ptr(off), n, _ptr(enc_off), _ptr(enc),
                              _ptr(dec_off), _ptr(dec), _ptr(status), nthreads,
                              ctypes.byref(te), ctypes.byref(td))
    return te.value, td.value, int(enc_off[-1]), status
