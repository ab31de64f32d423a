#!/usr/bin/env python3
"""Decode-only driver for PMC passes of the lane decoder: config <cfg>,
<reps> launches of nghttp2_amd_hd__decode_batch_lanes (mode 0 = auto slots,
sorted).  Usage: dec_lanes.py <cfg> <reps> [mode]"""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import numpy as np
import torch
import nghttp2_amd
from nghttp2_amd import hd, workloads as W

cfg, reps = int(sys.argv[1]), int(sys.argv[2])
mode = int(sys.argv[3]) if len(sys.argv) > 3 else int(os.environ.get("DL_MODE", "0"))
dev = torch.device("cuda:0")
vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
L = hd.lib()
L.nghttp2_amd_hd__decode_batch_lanes.argtypes = [vp, vp, u32, vp, sz, vp, vp, vp, vp, vp, ctypes.c_int]
codec = nghttp2_amd.HuffmanBatchCodec(dev)
if cfg == 5:
    pool, off, _ = W.gen_adversarial(1 << 20)
    enc = torch.from_numpy(pool).to(dev)
    eo = torch.from_numpy(off.view(np.int32)).to(dev)
else:
    pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
    src = torch.from_numpy(pool).to(dev)
    so = torch.from_numpy(off.view(np.int32)).to(dev)
    enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
torch.cuda.synchronize()
n = eo.numel() - 1
E = int(eo[-1].item())
cap = 64 * ((((E * 8) // 5) + 63) // 64 + n) + 64
d = torch.empty(cap, dtype=torch.uint8, device=dev)
do = torch.empty(n + 1, dtype=torch.int32, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
P = lambda t: ctypes.c_void_p(t.data_ptr())
s = torch.cuda.current_stream()
for _ in range(reps):
    rv = L.nghttp2_amd_hd__decode_batch_lanes(P(enc), P(eo), n, P(d), cap, P(do), P(st), None, None,
                                              ctypes.c_void_p(s.cuda_stream), mode)
    assert rv == 0
torch.cuda.synchronize()
print("ok", cfg, n, E)
