#!/usr/bin/env python3
"""Decode time against batch size (config-3 strings): per-1M-string time of
decode_batch_auto for 1M..8M strings, event-timed, median of 7.  A per-string
cost that falls with the batch size is the kernel's fixed and tail cost."""
import os, sys, json
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd
dev = torch.device("cuda:0")
codec = nghttp2_amd.HuffmanBatchCodec(dev)
s = torch.cuda.current_stream()
for m in [int(x) for x in (sys.argv[1:] or ["1", "2", "4", "8"])]:
    n = m << 20
    pool, off = W.gen_mixed_values(n, seed=3 + m)
    src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
    enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
    del src, so
    torch.cuda.synchronize()
    E = int(eo[-1].item()) & 0xFFFFFFFF
    dst = torch.empty(codec.decode_bound(E, n), dtype=torch.uint8, device=dev)
    doff = torch.empty(n + 1, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    ts = []
    for _ in range(9):
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        codec.decode_auto(enc, eo, enc_bytes=E, dst=dst, dst_off=doff, status=st, stream=s)
        b.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1000)
    t = float(np.median(ts[2:]))
    print(json.dumps({"strings_M": m, "enc_MB": round(E / 1e6, 1), "decode_us": round(t, 1),
                      "us_per_1M": round(t / m, 1), "GBps_alg": round((int(off[-1]) + E + 12 * n) / t / 1e3, 1)}),
          flush=True)
    del enc, eo, dst, doff, st
    torch.cuda.empty_cache()
