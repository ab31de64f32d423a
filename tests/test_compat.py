"""Link-level drop-in (nghttp2_hd_huff_* exported by libnghttp2_amd_hd.so).

CPU: the C test program links against the library.  GPU: it runs (the
reference's Huffman unit tests, chain spill, wrap overflow, chunked decode),
and a bulk ctypes comparison against the oracle: encode_count, encode into a
single wrap buffer, and whole / chunked decode with the carried context.
"""
import ctypes
import os
import subprocess
import tempfile

import numpy as np
import pytest

from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "nghttp2_amd", "lib")


def build_c_test(outdir):
    exe = os.path.join(outdir, "test_compat")
    subprocess.run(["gcc", "-O1", "-rdynamic", "-Wall", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "c", "test_compat.c"), "-L" + LIBDIR,
                    "-lnghttp2_amd_hd", "-Wl,-rpath," + LIBDIR, "-o", exe], check=True)
    return exe


def test_c_compat_program_links():
    with tempfile.TemporaryDirectory() as d:
        assert os.path.exists(build_c_test(d))


@pytest.mark.gpu
def test_c_compat_program_runs(dev):
    with tempfile.TemporaryDirectory() as d:
        exe = build_c_test(d)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert "compat OK" in r.stdout


class Buf(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("begin", "end", "pos", "last", "mark")]


class Chain(ctypes.Structure):
    pass


Chain._fields_ = [("next", ctypes.POINTER(Chain)), ("buf", Buf)]


class Bufs(ctypes.Structure):
    _fields_ = [("head", ctypes.POINTER(Chain)), ("cur", ctypes.POINTER(Chain)),
                ("mem", ctypes.c_void_p), ("chunk_length", ctypes.c_size_t),
                ("max_chunk", ctypes.c_size_t), ("chunk_used", ctypes.c_size_t),
                ("chunk_keep", ctypes.c_size_t), ("offset", ctypes.c_size_t)]


class Ctx(ctypes.Structure):
    _fields_ = [("fstate", ctypes.c_uint16), ("flags", ctypes.c_uint8)]


@pytest.mark.gpu
def test_compat_bulk_vs_oracle(dev):
    import nghttp2_amd
    from nghttp2_amd import workloads as W
    L = nghttp2_amd.lib()
    u8p = ctypes.c_char_p
    L.nghttp2_hd_huff_encode_count.restype = ctypes.c_size_t
    L.nghttp2_hd_huff_encode_count.argtypes = [u8p, ctypes.c_size_t]
    L.nghttp2_hd_huff_encode.argtypes = [ctypes.POINTER(Bufs), u8p, ctypes.c_size_t]
    L.nghttp2_hd_huff_decode.restype = ctypes.c_ssize_t
    L.nghttp2_hd_huff_decode.argtypes = [ctypes.POINTER(Ctx), ctypes.POINTER(Buf), u8p,
                                         ctypes.c_size_t, ctypes.c_int]
    L.nghttp2_hd_huff_decode_failure_state.argtypes = [ctypes.POINTER(Ctx)]
    pool, off = W.gen_all_bytes(300, seed=71, lo=0, hi=80)
    adv, aoff, _ = W.gen_adversarial(300, seed=72)
    rng = np.random.default_rng(5)
    for i in range(300):
        raw = bytes(pool[off[i]:off[i + 1]])
        assert L.nghttp2_hd_huff_encode_count(raw, len(raw)) == O.encode_count(raw)
        mem = ctypes.create_string_buffer(len(raw) * 4 + 8)
        ch = Chain()
        base = ctypes.addressof(mem)
        ch.buf = Buf(base, base + len(mem), base, base, base)
        bufs = Bufs(ctypes.pointer(ch), ctypes.pointer(ch), None, len(mem), 1, 1, 1, 0)
        assert L.nghttp2_hd_huff_encode(ctypes.byref(bufs), raw, len(raw)) == 0
        n = ch.buf.last - base
        rv, ref = O.encode(raw)
        assert mem.raw[:n] == ref
        # decode: whole, then in two chunks with the carried context
        src = bytes(adv[aoff[i]:aoff[i + 1]]) if i % 2 else ref
        rrv, rout, rctx = O.decode(src, 1)
        cut = int(rng.integers(0, len(src) + 1))
        ctx = Ctx(0, 1)
        ob = ctypes.create_string_buffer(len(src) * 8 // 5 + 16)
        ob_base = ctypes.addressof(ob)
        buf = Buf(ob_base, ob_base + len(ob), ob_base, ob_base, ob_base)
        r1 = L.nghttp2_hd_huff_decode(ctypes.byref(ctx), ctypes.byref(buf), src[:cut], cut, 0)
        r2 = L.nghttp2_hd_huff_decode(ctypes.byref(ctx), ctypes.byref(buf), src[cut:],
                                      len(src) - cut, 1)
        assert r1 == cut
        assert r2 == (rrv if rrv < 0 else len(src) - cut)
        assert (ctx.fstate, ctx.flags) == (rctx.fstate, rctx.flags)
        assert ob.raw[:buf.last - ob_base] == rout
        assert bool(L.nghttp2_hd_huff_decode_failure_state(ctypes.byref(ctx))) == \
            O.failure_state(rctx)


@pytest.mark.gpu
def test_compat_long_strings_vs_oracle(dev):
    """Strings on both sides of the drop-in's copy threshold (64 KiB: the
    mapped block below it, a device copy from it on), whole and chunked,
    bit-exact against the oracle."""
    import nghttp2_amd
    L = nghttp2_amd.lib()
    u8p = ctypes.c_char_p
    L.nghttp2_hd_huff_encode_count.restype = ctypes.c_size_t
    L.nghttp2_hd_huff_encode_count.argtypes = [u8p, ctypes.c_size_t]
    L.nghttp2_hd_huff_encode.argtypes = [ctypes.POINTER(Bufs), u8p, ctypes.c_size_t]
    L.nghttp2_hd_huff_decode.restype = ctypes.c_ssize_t
    L.nghttp2_hd_huff_decode.argtypes = [ctypes.POINTER(Ctx), ctypes.POINTER(Buf), u8p,
                                         ctypes.c_size_t, ctypes.c_int]
    rng = np.random.default_rng(0x10C)
    for size in (65535, 65536, 65537, 300001, (1 << 20) + 7):
        # mostly printable, some bytes of every value (long codes included)
        raw = rng.choice(np.arange(32, 127, dtype=np.uint8), size=size)
        raw[rng.integers(0, size, size=size // 50)] = rng.integers(0, 256, size=size // 50)
        raw = raw.tobytes()
        rv, ref = O.encode(raw)
        assert L.nghttp2_hd_huff_encode_count(raw, len(raw)) == len(ref) == O.encode_count(raw)
        mem = ctypes.create_string_buffer(len(ref) + 64)
        ch = Chain()
        base = ctypes.addressof(mem)
        ch.buf = Buf(base, base + len(mem), base, base, base)
        bufs = Bufs(ctypes.pointer(ch), ctypes.pointer(ch), None, len(mem), 1, 1, 1, 0)
        assert L.nghttp2_hd_huff_encode(ctypes.byref(bufs), raw, len(raw)) == 0
        assert mem.raw[:ch.buf.last - base] == ref, size
        for cut in (len(ref), len(ref) // 3):  # whole, then two chunks
            ctx = Ctx(0, 1)
            ob = ctypes.create_string_buffer(len(ref) * 8 // 5 + 16)
            ob_base = ctypes.addressof(ob)
            buf = Buf(ob_base, ob_base + len(ob), ob_base, ob_base, ob_base)
            r1 = L.nghttp2_hd_huff_decode(ctypes.byref(ctx), ctypes.byref(buf), ref[:cut], cut,
                                          1 if cut == len(ref) else 0)
            assert r1 == cut
            if cut < len(ref):
                r2 = L.nghttp2_hd_huff_decode(ctypes.byref(ctx), ctypes.byref(buf), ref[cut:],
                                              len(ref) - cut, 1)
                assert r2 == len(ref) - cut
            assert ob.raw[:buf.last - ob_base] == raw, (size, cut)
