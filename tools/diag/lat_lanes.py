#!/usr/bin/env python3
"""Latency of one group alone: N strings of L raw bytes (mixed-value text),
decoded by the cooperative lane decoder (mode 4) and by decode_batch_auto;
with N = 64 one wave decodes everything, so the time is one lane's chain.
Usage: lat_lanes.py [N L ...]"""
import ctypes, json, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import numpy as np
import torch
import nghttp2_amd
from nghttp2_amd import hd, workloads as W
dev = torch.device("cuda:0")
vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
P = lambda t: ctypes.c_void_p(t.data_ptr())
L = hd.lib()
L.nghttp2_amd_hd__decode_batch_lanes.argtypes = [vp, vp, u32, vp, sz, vp, vp, vp, vp, vp, ctypes.c_int]
codec = nghttp2_amd.HuffmanBatchCodec(dev)
args = [int(x) for x in sys.argv[1:]] or [64, 1000, 640, 1000, 64, 100]
rng = np.random.default_rng(7)
alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_./=;, ABCDEFGHIJKLMNOP", dtype=np.uint8)
for N, Lr in zip(args[0::2], args[1::2]):
    pool = alpha[rng.integers(0, len(alpha), N * Lr)].copy()
    off = (np.arange(N + 1, dtype=np.uint32) * Lr).astype(np.uint32)
    src = torch.from_numpy(np.concatenate([pool, np.zeros(64, np.uint8)])).to(dev)
    so = torch.from_numpy(off.view(np.int32)).to(dev)
    enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
    torch.cuda.synchronize()
    E = int(eo[-1].item())
    cap = 64 * ((((E * 8) // 5) + 63) // 64 + N) + 64
    d = torch.empty(cap, dtype=torch.uint8, device=dev)
    do = torch.empty(N + 1, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    res = {"N": N, "raw": Lr, "E": E}
    for name in ("lanes2", "items"):
        ts = []
        for it in range(12):
            a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
            a.record(s)
            if name == "lanes2":
                rv = L.nghttp2_amd_hd__decode_batch_lanes(P(enc), P(eo), N, P(d), cap, P(do), P(st), None, None,
                                                          ctypes.c_void_p(s.cuda_stream), 4)
            else:
                rv = L.nghttp2_amd_hd_huff_decode_batch_auto(P(enc), P(eo), N, P(d), codec.decode_bound(E, N), P(do),
                                                             P(st), None, None, ctypes.c_void_p(s.cuda_stream))
            b.record(s); torch.cuda.synchronize()
            assert rv == 0
            if it >= 2: ts.append(a.elapsed_time(b) * 1000)
        res[name + "_us"] = round(float(np.median(ts)), 1)
        assert int(st[0].item()) == Lr, (name, int(st[0].item()))
    print(json.dumps(res), flush=True)
