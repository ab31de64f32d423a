#!/usr/bin/env python3
"""Encode pass times against batch size (config-3 strings): k_enc_count
alone and the whole encode_batch (count + pack), each call after a 512 MiB
read that leaves none of its inputs in the Infinity Cache (the bench's state
after a decode).  A time that steps with the count of workgroup passes
(tiles / resident workgroups) rather than with the bytes is a tail effect.
Usage: enc_scale.py [n ...]   (default 0.75M .. 2M strings)"""
import ctypes, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd

dev = torch.device("cuda:0")
codec = nghttp2_amd.HuffmanBatchCodec(dev)
L = codec.L
s = torch.cuda.current_stream()
P = lambda t: ctypes.c_void_p(t.data_ptr())
ROUNDS = int(os.environ.get("ROUNDS", "10"))
FLUSH = torch.ones(512 << 20, dtype=torch.uint8, device=dev)


def timed(fn):
    v = []
    for _ in range(ROUNDS):
        FLUSH.view(torch.int32).max()
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record(s); fn(); b.record(s); torch.cuda.synchronize()
        v.append(a.elapsed_time(b) * 1000)
    return round(float(np.median(v)), 1)


ns = [int(x) for x in sys.argv[1:]] or [3 << 18, 1 << 20, 5 << 18, 3 << 19, 1 << 21]
for n in ns:
    pool, off = W.gen_mixed_values(n)
    R = int(off[-1])
    src = torch.from_numpy(pool).to(dev)
    so = torch.from_numpy(off.view(np.int32)).to(dev)
    clen = torch.empty(n, dtype=torch.int32, device=dev)
    ecap = codec.encode_bound(R, n)
    edst = torch.empty(ecap, dtype=torch.uint8, device=dev)
    eoff = torch.empty(n + 1, dtype=torch.int32, device=dev)
    wsz = L.nghttp2_amd_hd_huff_encode_workspace_size(R, n)
    ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
    cnt = lambda: L.nghttp2_amd_hd_huff_encode_count_batch(P(src), P(so), n, P(clen), ctypes.c_void_p(s.cuda_stream))
    enc = lambda: L.nghttp2_amd_hd_huff_encode_batch(P(src), P(so), n, P(edst), ecap, P(eoff), P(ws), wsz,
                                                     ctypes.c_void_p(s.cuda_stream))
    cnt(); enc(); torch.cuda.synchronize()
    tc, te = timed(cnt), timed(enc)
    print(json.dumps({"n": n, "tiles": (n + 255) // 256, "raw_MB": round(R / 1e6, 1),
                      "count_us": tc, "count_GBps": round(R / tc / 1e3, 1),
                      "encode_us": te, "pack_us_est": round(te - tc, 1)}), flush=True)
    del src, edst, ws
