#!/usr/bin/env python3
"""Decode-only driver for PMC runs: config 2, 3 or 5, the in-tree library."""
import os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda:0")
codec = nghttp2_amd.HuffmanBatchCodec(dev)
if cfg == 5:
    pool, off = W.gen_adversarial(1 << 20)[:2]
    enc = torch.from_numpy(pool).to(dev); eo = torch.from_numpy(off.view(np.int32)).to(dev)
else:
    pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
    src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
    enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
torch.cuda.synchronize()
E = int(eo[-1].item()) & 0xFFFFFFFF
for _ in range(reps):
    codec.decode_auto(enc, eo, enc_bytes=E)
torch.cuda.synchronize()
print("ok")
