#!/usr/bin/env python3
"""Interleaved timing of decode_batch_lanes (mode 0) across library builds
(the product library and tools/diag/lib_<name>.so variants).
Usage: ab_dl_libs.py <cfg,cfg> name1 name2 ..."""
import ctypes, json, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import numpy as np
import torch
import nghttp2_amd
from nghttp2_amd import hd, workloads as W
dev = torch.device("cuda:0")
MODE = int(os.environ.get("DL_MODE", "0"))  # 4: the cooperative-transfer decoder
vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
P = lambda t: ctypes.c_void_p(t.data_ptr())
libs = {"base": hd.lib()}
for name in sys.argv[2:]:
    libs[name] = ctypes.CDLL(os.path.join(HERE, "lib_%s.so" % name), mode=ctypes.RTLD_LOCAL)
for L in libs.values():
    L.nghttp2_amd_hd__decode_batch_lanes.argtypes = [vp, vp, u32, vp, sz, vp, vp, vp, vp, vp, ctypes.c_int]
codec = nghttp2_amd.HuffmanBatchCodec(dev)
for cfg in [int(x) for x in sys.argv[1].split(",")]:
    if cfg == 5:
        pool, off, _ = W.gen_adversarial(1 << 20)
        enc = torch.from_numpy(pool).to(dev); eo = torch.from_numpy(off.view(np.int32)).to(dev)
    else:
        pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
        src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
        enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
    torch.cuda.synchronize()
    n = eo.numel() - 1; E = int(eo[-1].item()); cap = 64 * ((((E * 8) // 5) + 63) // 64 + n) + 64
    d = torch.empty(cap, dtype=torch.uint8, device=dev)
    do = torch.empty(n + 1, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    res = {k: [] for k in libs}
    for it in range(12):
        for k, L in libs.items():
            a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
            a.record(s)
            rv = L.nghttp2_amd_hd__decode_batch_lanes(P(enc), P(eo), n, P(d), cap, P(do), P(st), None, None,
                                                      ctypes.c_void_p(s.cuda_stream), MODE)
            b.record(s); torch.cuda.synchronize()
            assert rv == 0
            if it >= 2: res[k].append(a.elapsed_time(b) * 1000)
    print(json.dumps({"config": cfg, **{k: round(float(np.median(v)), 1) for k, v in res.items()}}), flush=True)
