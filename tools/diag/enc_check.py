#!/usr/bin/env python3
"""encode_batch and emit_strings_batch of each tools/diag/lib_*.so against
the oracle over several workloads and sizes (multi-tile batches); prints
the first differing string per case.  Usage: enc_check.py"""
import ctypes, glob, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
from oracle import oracle as O

vp, u32, u64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
dev = torch.device("cuda:0")
libs = {}
for p in sorted(glob.glob(os.path.join(HERE, "lib_*.so"))):
    L = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
    L.nghttp2_amd_hd_huff_encode_batch.argtypes = [vp, vp, u32, vp, sz, vp, vp, sz, vp]
    L.nghttp2_amd_hd_huff_encode_workspace_size.restype = sz
    L.nghttp2_amd_hd_huff_encode_workspace_size.argtypes = [u64, u32]
    L.nghttp2_amd_hd_huff_encode_bound.restype = sz
    L.nghttp2_amd_hd_huff_encode_bound.argtypes = [u64, u32]
    L.nghttp2_amd_hd_emit_strings_batch.argtypes = [vp, vp, u32, u64, vp, sz, vp, vp, sz, vp]
    L.nghttp2_amd_hd_emit_strings_workspace_size.restype = sz
    L.nghttp2_amd_hd_emit_strings_workspace_size.argtypes = [u64, u32]
    L.nghttp2_amd_hd_emit_strings_bound.restype = sz
    L.nghttp2_amd_hd_emit_strings_bound.argtypes = [u64, u32]
    libs[os.path.basename(p)[4:-3]] = L
s = torch.cuda.current_stream()
P = lambda t: ctypes.c_void_p(t.data_ptr())


def first_diff(got, goff, ref, roff):
    n = len(roff) - 1
    if not np.array_equal(goff, roff):
        i = int(np.nonzero(goff != roff)[0][0])
        return "offset %d (tile %d): %d vs %d" % (i, i // 256, goff[i], roff[i])
    for i in range(n):
        a, b = int(roff[i]), int(roff[i + 1])
        if not np.array_equal(got[a:b], ref[a:b]):
            return "bytes of string %d (tile %d)" % (i, i // 256)
    return None


cases = []
for n in (100, 300, 1000, 5000, 40000, 200000):
    cases.append(("mixed", n) + W.gen_mixed_values(n, seed=n))
    cases.append(("pseudo", n) + W.gen_pseudo_headers(n, seed=n + 1))
    cases.append(("allbytes", n) + W.gen_all_bytes(n, seed=n + 2))
# header names and values of the config-1 cases (the deflater's literals)
_src = json.load(open(os.path.join(HERE, "..", "..", "tests", "golden", "config1_cases.json")))["cases"]
_strs = [x.encode() for c in _src for h in c["headers"] for kv in h.items() for x in kv]
for lo, hi in ((0, 2000), (3000, 4500), (0, len(_strs))):
    ss = _strs[lo:hi]
    o = np.zeros(len(ss) + 1, dtype=np.uint32)
    o[1:] = np.cumsum([len(x) for x in ss])
    cases.append(("config1_hdr%d" % lo, len(ss), np.frombuffer(b"".join(ss), np.uint8).copy(), o))
bad = 0
for name, n, pool, off in cases:
    R = int(off[-1])
    src = torch.from_numpy(np.concatenate([pool, np.zeros(16, np.uint8)])).to(dev)
    so = torch.from_numpy(off.astype(np.uint32).view(np.int32)).to(dev)
    ref, roff = O.encode_batch(pool, off)
    fref, froff = O.emit_strings_batch(pool, off)
    for k, L in libs.items():
        cap = L.nghttp2_amd_hd_huff_encode_bound(R, n)
        d = torch.zeros(cap, dtype=torch.uint8, device=dev)
        do = torch.zeros(n + 1, dtype=torch.int32, device=dev)
        wsz = L.nghttp2_amd_hd_huff_encode_workspace_size(R, n)
        ws = torch.full((wsz,), 0x5A, dtype=torch.uint8, device=dev)
        rc = L.nghttp2_amd_hd_huff_encode_batch(P(src), P(so), n, P(d), cap, P(do), P(ws), wsz, ctypes.c_void_p(s.cuda_stream))
        torch.cuda.synchronize()
        e1 = "rc %d" % rc if rc else first_diff(d.cpu().numpy(), do.cpu().numpy().view(np.uint32), ref, roff)
        fcap = L.nghttp2_amd_hd_emit_strings_bound(R, n)
        fd = torch.zeros(fcap, dtype=torch.uint8, device=dev)
        fo = torch.zeros(n + 1, dtype=torch.int32, device=dev)
        fwsz = L.nghttp2_amd_hd_emit_strings_workspace_size(R, n)
        fws = torch.full((fwsz,), 0x5A, dtype=torch.uint8, device=dev)
        rc = L.nghttp2_amd_hd_emit_strings_batch(P(src), P(so), n, R, P(fd), fcap, P(fo), P(fws), fwsz, ctypes.c_void_p(s.cuda_stream))
        torch.cuda.synchronize()
        e2 = "rc %d" % rc if rc else first_diff(fd.cpu().numpy(), fo.cpu().numpy().view(np.uint32), fref, froff)
        bad += bool(e1) + bool(e2)
        print(json.dumps({"case": name, "n": n, "lib": k, "encode": e1 or "ok", "emit": e2 or "ok"}), flush=True)
print("mismatching cases:", bad)
