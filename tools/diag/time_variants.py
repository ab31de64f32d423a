#!/usr/bin/env python3
"""Time ablation variants of the decode kernel (and encode) in ONE process,
interleaved rounds (cdna_hip_programming.md 5.4 rule 24)."""
import ctypes, glob, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
dev = torch.device("cuda:0")
pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
codec = nghttp2_amd.HuffmanBatchCodec(dev)
src = torch.from_numpy(pool).to(dev)
so = torch.from_numpy(off.view(np.int32)).to(dev)
enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
torch.cuda.synchronize()
E = int(eo[-1].item())
n = len(off) - 1
dcap = codec.decode_bound(E, n)
dst = torch.empty(dcap, dtype=torch.uint8, device=dev)
doff = torch.empty(n + 1, dtype=torch.int32, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
libs = {}
for p in sorted(glob.glob(os.path.join(HERE, "lib_*.so"))):
    L = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
    vp = ctypes.c_void_p
    L.nghttp2_amd_hd_huff_decode_batch_auto.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_size_t, vp, vp, vp, vp, vp]
    L.nghttp2_amd_hd_huff_encode_batch.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp]
    libs[os.path.basename(p)[4:-3]] = L
s = torch.cuda.current_stream()
def run(L):
    L.nghttp2_amd_hd_huff_decode_batch_auto(ctypes.c_void_p(enc.data_ptr()), ctypes.c_void_p(eo.data_ptr()), n,
        ctypes.c_void_p(dst.data_ptr()), dcap, ctypes.c_void_p(doff.data_ptr()), ctypes.c_void_p(st.data_ptr()),
        None, None, ctypes.c_void_p(s.cuda_stream))
ecap = codec.encode_bound(int(off[-1]), n)
edst = torch.empty(ecap, dtype=torch.uint8, device=dev)
eoff = torch.empty(n + 1, dtype=torch.int32, device=dev)
wsz = codec.L.nghttp2_amd_hd_huff_encode_workspace_size(int(off[-1]), n)
wss = {}
def run_enc(L):
    L.nghttp2_amd_hd_huff_encode_batch(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(so.data_ptr()), n,
        ctypes.c_void_p(edst.data_ptr()), ecap, ctypes.c_void_p(eoff.data_ptr()),
        ctypes.c_void_p(wss.setdefault(id(L), torch.zeros(wsz, dtype=torch.uint8, device=dev)).data_ptr()),
        wsz, ctypes.c_void_p(s.cuda_stream))
eres = {k: [] for k in libs}
ref_enc = enc[:E].clone()
for k, L in libs.items():
    for _ in range(3): run_enc(L)
    torch.cuda.synchronize()
    assert torch.equal(edst[:E], ref_enc), k + ": encode differs"
for rnd in range(10):
    for k, L in libs.items():
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record(s); run_enc(L); b.record(s); torch.cuda.synchronize()
        eres[k].append(a.elapsed_time(b) * 1000)
res = {k: [] for k in libs}
ref_dec = None
for k, L in libs.items():
    dst.zero_(); st.zero_()
    for _ in range(3): run(L)
    torch.cuda.synchronize()
    if ref_dec is None:
        ref_dec = (dst.clone(), st.clone(), doff.clone())
    else:
        assert torch.equal(dst, ref_dec[0]) and torch.equal(st, ref_dec[1]) and torch.equal(doff, ref_dec[2]), k + ": decode differs"
torch.cuda.synchronize()
for rnd in range(10):
    for k, L in libs.items():
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record(s); run(L); b.record(s); torch.cuda.synchronize()
        res[k].append(a.elapsed_time(b) * 1000)
out = {k: {"median_us": round(float(np.median(v)), 1), "min_us": round(float(np.min(v)), 1)} for k, v in res.items()}
eout = {k: {"median_us": round(float(np.median(v)), 1), "min_us": round(float(np.min(v)), 1)} for k, v in eres.items()}
print(json.dumps({"config": cfg, "decode_variants": out, "encode_variants": eout}, indent=1))
