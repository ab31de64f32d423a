#!/usr/bin/env python3
"""Per-wave phase cycles of the lane decoder (DL_STAMPS=1 build,
tools/diag/lib_dlstamps.so, loaded through NGHTTP2_AMD_LIB).  Slots:
0 sort, 1 group setup, 2 period service, 3 pairs, 4 careful steps,
5 group end, 9 groups, 10 periods, 11 lifetime.  Usage: dl_stamps.py [cfg..]"""
import ctypes, json, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
os.environ["NGHTTP2_AMD_LIB"] = os.path.join(HERE, "lib_dlstamps.so")
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
L.nghttp2_amd_hd__dl_stamps.argtypes = [vp, ctypes.c_int]
codec = nghttp2_amd.HuffmanBatchCodec(dev)
for cfg in [int(x) for x in sys.argv[1:]] or [3, 2]:
    for mode in [int(x) for x in os.environ.get("DL_MODES", "0,2").split(",")]:
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
        s = torch.cuda.current_stream()
        for rep in range(3):
            L.nghttp2_amd_hd__dl_stamps(None, 1)
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
            a.record(s)
            rv = L.nghttp2_amd_hd__decode_batch_lanes(P(enc), P(eo), n, P(d), cap, P(do), P(st), None, None,
                                                      ctypes.c_void_p(s.cuda_stream), mode)
            b.record(s)
            torch.cuda.synchronize()
            assert rv == 0
        us = a.elapsed_time(b) * 1000
        buf = np.zeros((2048, 12), dtype=np.uint64)
        L.nghttp2_amd_hd__dl_stamps(buf.ctypes.data_as(ctypes.c_void_p), 0)
        live = buf[:, 11] > 0
        m = buf[live].astype(np.float64)
        names = ["sort", "gsetup", "service", "pairs", "careful", "gend", "", "", "", "groups", "periods", "life"]
        out = {"config": cfg, "mode": mode, "us": round(us, 1), "waves": int(live.sum())}
        for k in (0, 1, 2, 3, 4, 5, 9, 10, 11):
            out[names[k] + "_mean"] = round(float(m[:, k].mean()), 1)
            out[names[k] + "_max"] = round(float(m[:, k].max()), 1)
        print(json.dumps(out), flush=True)
