#!/usr/bin/env python3
"""Offline warm-up statistics for the item decoder (CPU only): for sampled
config-3 strings cut into 40-byte pieces, start a speculative decode OV bytes
before each later piece and report how often its first codeword boundary at
or after the piece start misses the true one, and how far (bits) the
speculative path runs before it rejoins the true boundaries."""
import os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "nghttp2_amd", "tools")); sys.path.insert(0, os.path.join(HERE, "..", ".."))
import gen_tables as G
from nghttp2_amd import workloads as W
codes = G.canonical_codes()[0]
# decode trie via dict of (len, code) -> sym
lut = {}
for sym,(c,l) in enumerate(codes): lut[(l,c)] = sym
pool, off = W.gen_mixed_values(1<<16)
L = np.array([c[1] for c in codes[:256]]); C = np.array([c[0] for c in codes[:256]])
rng = np.random.default_rng(1)
def bits_of(i):
    s = pool[off[i]:off[i+1]]
    return ''.join(format(int(C[b]), '0%db' % L[b]) for b in s)
def boundaries(bits, start):
    # decode from bit 'start', return list of boundary positions (after each symbol)
    out=[]; p=start; n=len(bits)
    while True:
        l=5; 
        while l<=30 and p+l<=n and (l, int(bits[p:p+l],2)) not in lut: l+=1
        if l>30 or p+l>n: break
        sym = lut[(l,int(bits[p:p+l],2))]
        if sym==256: break
        p+=l; out.append(p)
    return out
P=40
res={ov:[0,0,[]] for ov in (8,12,16,20,24)}
idx = rng.choice(len(off)-1, 3000, replace=False)
for i in idx:
    bits = bits_of(i); E=(len(bits)+7)//8
    if E <= P: continue
    true = set([0]+boundaries(bits,0))
    tl = sorted(true)
    for k in range(1, (E+P-1)//P):
        s=8*P*k
        te = next((b for b in tl if b>=s), None)
        if te is None: continue
        for ov in res:
            st = max(0, s-8*ov)
            sb = boundaries(bits, st)
            se = next((b for b in sb if b>=s), None)
            res[ov][0]+=1
            if se != te:
                res[ov][1]+=1
                # resync: first boundary of spec path (after se) that is a true boundary
                rs = next((b for b in sb if b>=s and b in true), None)
                res[ov][2].append((rs - s) if rs is not None else -1)
for ov,(n,m,d) in res.items():
    print(ov, n, m, m/n, "resync dist bits (median, max):", (np.median(d), max(d)) if d else None)
