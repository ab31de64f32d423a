"""The bounds-checked debug build (nghttp2_amd/lib/libnghttp2_amd_hd_bounds.so,
the library compiled with HD_BOUNDS=1): every LDS staging, region and image
index and every per-string global index the hot-path kernels compute is
checked against its buffer (csrc/hd_huff.hip HD_CHECK sites).
A child process loads that build through NGHTTP2_AMD_LIB, runs the parity
cases of tests/test_parity_gpu.py through it -- encode, both decode_batch_auto
instances, the slot decoder, emit_strings, adversarial and window-edge
inputs, NGHTTP2_HD_MAX_NV-sized and empty strings, one-tile batches -- and
after each asks nghttp2_amd_hd__bounds_check for the first recorded
violation, which must be none.  The report path itself is checked by the
build's self-test kernel (site 0x1FF)."""
import ctypes
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOUNDS_LIB = os.path.join(REPO, "nghttp2_amd", "lib", "libnghttp2_amd_hd_bounds.so")

CHILD = r"""
import ctypes, sys
sys.path.insert(0, %r)
import numpy as np
import torch
import nghttp2_amd
from nghttp2_amd import workloads as W
from oracle import oracle as O
from tests import test_parity_gpu as T

L = nghttp2_amd.lib()
L.nghttp2_amd_hd__bounds_check.argtypes = [ctypes.POINTER(ctypes.c_uint32)]


def take():
    s = ctypes.c_uint32(0)
    rc = L.nghttp2_amd_hd__bounds_check(ctypes.byref(s))
    assert rc == 0, "not the bounds-checked build (rc %%d)" %% rc
    return s.value


s = ctypes.c_uint32(0x5E1F7E57)
assert L.nghttp2_amd_hd__bounds_check(ctypes.byref(s)) == 0 and s.value == 0x1FF, hex(s.value)
assert take() == 0, "the record is not cleared"
dev = torch.device("cuda:0")
codec = nghttp2_amd.HuffmanBatchCodec(dev)


def done(tag):
    v = take()
    assert v == 0, "%%s: out-of-bounds index at site 0x%%x" %% (tag, v)
    print("ok", tag, flush=True)


def ragged():
    rng = np.random.default_rng(9)
    lens = rng.choice([0, 0, 1, 2, 3, 15, 16, 17, 31, 33, 300], size=9000)
    return W._pool_from_lengths(lens, rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8))


def max_len():
    rng = np.random.default_rng(12)
    lens = np.array([65536, 1, 65536, 70000, 0, 65535], dtype=np.int64)
    return W._pool_from_lengths(lens, rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8))


cases = [("pseudo", W.gen_pseudo_headers(60000)), ("mixed", W.gen_mixed_values(20000)),
         ("allbytes", W.gen_all_bytes(20000, seed=5)), ("ragged", ragged()), ("max-len", max_len()),
         ("one-tile", W.gen_mixed_values(200)),
         ("all-empty", W._pool_from_lengths(np.zeros(3000, np.int64), np.zeros(0, np.uint8)))]
for tag, (pool, off) in cases:
    T.check_roundtrip(codec, dev, pool, off, tag)
    enc, eoff = O.encode_batch(pool, off)
    for pick in ("items64", "pieces40"):
        T.auto_decode_check(codec, dev, enc, eoff, tag + " " + pick, pick=pick)
    T.check_emit(codec, dev, pool, off, tag)
    done(tag)
pool, off, cats = W.gen_adversarial(50000, seed=77)
enc_w, eoff_w = T.window_edge_batch()
for tag, (enc, eoff) in (("adversarial", (pool, off)), ("window edges", (enc_w, eoff_w)),
                         ("garbage", W.gen_all_bytes(40000, seed=21, lo=0, hi=48))):
    T.check_decode(codec, dev, enc, eoff, tag)
    for pick in ("items64", "pieces40"):
        T.auto_decode_check(codec, dev, enc, eoff, tag + " " + pick, pick=pick)
    done(tag)
print("BOUNDS-OK")
""" % REPO


def test_bounds_lib_built_and_exports():
    """(CPU) the debug build exists beside the product and exports the
    report; the product's report says it compiled no checks (1), without a
    GPU call."""
    assert os.path.exists(BOUNDS_LIB), "build() makes " + BOUNDS_LIB
    for path, want in ((BOUNDS_LIB, None), (os.path.join(REPO, "nghttp2_amd", "lib",
                                                         "libnghttp2_amd_hd.so"), 1)):
        L = ctypes.CDLL(path)
        fn = L.nghttp2_amd_hd__bounds_check
        fn.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
        if want is not None:
            s = ctypes.c_uint32(7)
            assert fn(ctypes.byref(s)) == want and s.value == 7


@pytest.mark.gpu
def test_bounds_checked_build_vs_oracle():
    env = dict(os.environ, NGHTTP2_AMD_LIB=BOUNDS_LIB)
    r = subprocess.run([sys.executable, "-u", "-c", CHILD], env=env, cwd=REPO,
                       capture_output=True, text=True, timeout=115)
    assert r.returncode == 0 and "BOUNDS-OK" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
