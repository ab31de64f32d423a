#!/usr/bin/env python3
"""Huffman self-synchronisation distance on configs 2/3 (CPU, oracle-encoded):
bits decoded from a random start until the path hits a true codeword
boundary.  Sizes the speculative warm-up of the piece decoder."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from nghttp2_amd import workloads as W
from oracle import oracle as O
L = W.CODE_LEN
codes = {(int(W.CODE_VAL[s]), int(L[s])): s for s in range(257)}
for cfg, gen in ((2, W.gen_pseudo_headers), (3, W.gen_mixed_values)):
    pool, off = gen(3000)
    enc, eoff = O.encode_batch(pool, off)
    bits = np.unpackbits(enc[:eoff[-1]])
    res = []
    rng = np.random.default_rng(1)
    for i in range(len(off) - 1):
        a, b = int(eoff[i]) * 8, int(eoff[i + 1]) * 8
        if b - a < 200:
            continue
        tb = set(); p = a
        for c in pool[off[i]:off[i + 1]]:
            tb.add(p); p += int(L[c])
        tb.add(p)
        for _ in range(3):
            s = int(rng.integers(a, b - 100)); p = s
            while p not in tb and p < b:
                v = 0
                for l in range(1, 31):
                    v = (v << 1) | (int(bits[p + l - 1]) if p + l - 1 < len(bits) else 0)
                    if (v, l) in codes:
                        break
                p += l
            res.append(p - s)
    r = np.array(res)
    print("cfg", cfg, "samples", len(r), "sync bits p50/90/99/99.9:", np.percentile(r, [50, 90, 99, 99.9]), "max", r.max())
