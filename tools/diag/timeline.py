#!/usr/bin/env python3
"""Per-wave timeline of the item decoder (a DD_TIMELINE build,
tools/diag/lib_tl.so from
`PATCH=tools/diag/patches/r4_diag_hooks.patch build_variants.sh tl:-DDD_TIMELINE`): s_memrealtime (100 MHz) at entry, after the range
search + table staging, after each task, at exit.  Prints the launch span,
the startup share and how far apart waves and workgroups finish."""
import ctypes, os, sys, json
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd
L = ctypes.CDLL(os.path.join(HERE, "lib_tl.so"), mode=ctypes.RTLD_LOCAL)
vp = ctypes.c_void_p
L.nghttp2_amd_hd_huff_decode_batch_auto.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint64, vp, ctypes.c_size_t, vp, vp, vp, vp, vp]
L.nghttp2_amd_hd__timeline.argtypes = [vp]
dev = torch.device("cuda:0")
codec = nghttp2_amd.HuffmanBatchCodec(dev)
s = torch.cuda.current_stream()
P = lambda t: vp(t.data_ptr())
for m in [int(x) for x in (sys.argv[1:] or ["1"])]:
    n = m << 20
    pool, off = W.gen_mixed_values(n, seed=3 + m)
    src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
    enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
    torch.cuda.synchronize()
    E = int(eo[-1].item()) & 0xFFFFFFFF
    cap = codec.decode_bound(E, n)
    dst = torch.empty(cap, dtype=torch.uint8, device=dev)
    doff = torch.empty(n + 1, dtype=torch.int32, device=dev); st = torch.empty(n, dtype=torch.int32, device=dev)
    buf = np.zeros(8192 * 4, dtype=np.uint64)
    res = []
    for r in range(5):
        rc = L.nghttp2_amd_hd_huff_decode_batch_auto(P(enc), P(eo), n, E, P(dst), cap, P(doff), P(st), None, None, vp(s.cuda_stream))
        assert rc == 0
        torch.cuda.synchronize()
        L.nghttp2_amd_hd__timeline(vp(buf.ctypes.data))
        t = buf.reshape(-1, 4).astype(np.int64)
        used = t[:, 3] > 0
        t = t[used]
        t0 = t[:, 0].min()
        ts = (t - t0) * 10 / 1000.0  # us
        nw = len(ts)
        wg = np.arange(nw) // 16
        end = ts[:, 3]
        wg_end = np.array([end[wg == g].max() for g in range(wg.max() + 1)])
        wg_first_end = np.array([end[wg == g].min() for g in range(wg.max() + 1)])
        res.append({"waves": int(nw), "span_us": round(float(end.max()), 1),
                    "entry_spread_us": round(float(ts[:, 0].max()), 1),
                    "staged_med_us": round(float(np.median(ts[:, 1] - ts[:, 0])), 2),
                    "first_task_end_med_us": round(float(np.median(ts[:, 2] - ts[:, 1])), 1),
                    "wave_end_med_us": round(float(np.median(end)), 1),
                    "wave_end_min_us": round(float(end.min()), 1),
                    "idle_frac": round(float(np.mean(end.max() - end) / end.max()), 4),
                    "wg_end_min_med_max": [round(float(x), 1) for x in (wg_end.min(), np.median(wg_end), wg_end.max())],
                    "in_wg_spread_med_us": round(float(np.median(wg_end - wg_first_end)), 1)})
    print(json.dumps({"strings_M": m, "runs": res[1:]}), flush=True)
    # the last run's per-workgroup end times and its waves' first-task ends
    # (for correlating with the workgroup's work, computed on the host)
    print(json.dumps({"strings_M": m, "wg_end_us": [round(float(x), 2) for x in wg_end],
                      "wg_start_us": [round(float(ts[wg == g, 0].min()), 2) for g in range(wg.max() + 1)]}),
          flush=True)
    np.save(os.path.join(os.environ.get("TL_OUT", "."), "eoff_%dM.npy" % m), eo.cpu().numpy())
