#!/usr/bin/env python3
"""Many small encode_batch / emit_strings_batch calls (1..2000 strings of
header-like text) per tools/diag/lib_*.so against the oracle: a race shows
as an occasional mismatch.  Usage: enc_small.py [calls]"""
import ctypes, glob, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
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
src_all = json.load(open(os.path.join(HERE, "..", "..", "tests", "golden", "config1_cases.json")))["cases"]
strs = [x.encode() for c in src_all for h in c["headers"] for kv in h.items() for x in kv]
rng = np.random.default_rng(7)
calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
src = torch.zeros(1 << 22, dtype=torch.uint8, device=dev)
so = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
d = torch.zeros(1 << 23, dtype=torch.uint8, device=dev)
do = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
bad = {k: [0, 0] for k in libs}
for c in range(calls):
    n = int(rng.choice([1, 3, 7, 20, 64, 65, 200, 300, 1000, 2000]))
    pick = rng.integers(0, len(strs), size=n)
    ss = [strs[i] for i in pick]
    off = np.zeros(n + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(x) for x in ss])
    pool = np.frombuffer(b"".join(ss) + bytes(16), np.uint8)
    R = int(off[-1])
    src[:len(pool)].copy_(torch.from_numpy(pool.copy()))
    so[:n + 1].copy_(torch.from_numpy(off.view(np.int32)))
    ref, roff = O.encode_batch(pool[:R], off)
    fref, froff = O.emit_strings_batch(pool[:R], off)
    for k, L in libs.items():
        for mode in (0, 1):
            if mode == 0:
                rc = L.nghttp2_amd_hd_huff_encode_batch(P(src), P(so), n, P(d), d.numel(), P(do), P(ws), ws.numel(),
                                                        ctypes.c_void_p(s.cuda_stream))
                rr, ro = ref, roff
            else:
                rc = L.nghttp2_amd_hd_emit_strings_batch(P(src), P(so), n, R, P(d), d.numel(), P(do), P(ws),
                                                         ws.numel(), ctypes.c_void_p(s.cuda_stream))
                rr, ro = fref, froff
            torch.cuda.synchronize()
            go = do[:n + 1].cpu().numpy().view(np.uint32)
            E = int(ro[-1])
            ok = rc == 0 and np.array_equal(go, ro) and np.array_equal(d[:E].cpu().numpy(), rr[:E])
            if not ok:
                bad[k][mode] += 1
                if bad[k][mode] <= 3:
                    print(json.dumps({"call": c, "n": n, "lib": k, "mode": ["encode", "emit"][mode],
                                      "offsets_equal": bool(np.array_equal(go, ro))}), flush=True)
print("bad (encode, emit) per lib:", bad)
