#!/usr/bin/env python3
"""Per-phase cycles of k_decode_dense from an HD_DIAG_STAMPS build
(tools/diag/lib_stamps.so): one row of s_memtime sums per wave, plus the
wave-summed lane step counts of decode_item (fast iterations, checked steps,
warm-up steps).  Usage: stamps_dense.py [config 2|3|5 ...]"""
import ctypes, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd

dev = torch.device("cuda:0")
vp = ctypes.c_void_p
L = ctypes.CDLL(os.path.join(HERE, os.environ.get("STAMPS_LIB", "lib_stamps.so")), mode=ctypes.RTLD_LOCAL)
L.nghttp2_amd_hd_huff_decode_batch_auto.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_size_t, vp, vp, vp, vp, vp]
codec = nghttp2_amd.HuffmanBatchCodec(dev)
names = ["setup", "stage", "warm_rest", "decode_rest", "verify", "scan", "store"]
sub = {10: "bb_pairs", 11: "single_fast", 12: "checked"}
for cfg in [int(x) for x in sys.argv[1:]] or [2, 3]:
    if cfg == 5:
        pool, off, _ = W.gen_adversarial(1 << 20)
        enc = torch.from_numpy(pool).to(dev); eo = torch.from_numpy(off.view(np.int32)).to(dev)
    else:
        pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
        src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
        enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
    torch.cuda.synchronize()
    E = int(eo[-1].item()); n = eo.numel() - 1
    cap = codec.decode_bound(E, n)
    dst = torch.empty(cap, dtype=torch.uint8, device=dev); doff = torch.empty(n + 1, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()

    def run():
        L.nghttp2_amd_hd_huff_decode_batch_auto(vp(enc.data_ptr()), vp(eo.data_ptr()), n, vp(dst.data_ptr()), cap,
                                                vp(doff.data_ptr()), vp(st.data_ptr()), None, None, vp(s.cuda_stream))
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    L.nghttp2_amd_hd__diag_stamps(None, 1)
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(s); run(); b.record(s); torch.cuda.synchronize()
    buf = np.zeros((4096, 20), dtype=np.uint64)
    L.nghttp2_amd_hd__diag_stamps(vp(buf.ctypes.data), 0)
    used = buf[:, 7] > 0
    B = buf[used].astype(float)
    life = B[:, 7]
    rounds = B[:, 9].sum()
    print(json.dumps({
        "config": cfg, "kernel_us": round(a.elapsed_time(b) * 1000, 1), "waves": int(used.sum()),
        "enc_bytes": E, "lifetime_cycles_median": float(np.median(life)), "lifetime_cycles_max": float(life.max()),
        "share_of_lifetime": {k: round(float(B[:, i].sum() / life.sum()), 4) for i, k in enumerate(names)},
        "cycles_per_round": {k: round(float(B[:, i].sum() / rounds), 1) for i, k in enumerate(names)},
        "loop_cycles_per_round": {v: round(float(B[:, k].sum() / rounds), 1) for k, v in sub.items()},
        "wave_iters_per_round": {
                                 "pairs": round(B[:, 13].sum() / rounds, 2),
                                 "single_fast": round(B[:, 14].sum() / rounds, 2),
                                 "checked": round(B[:, 15].sum() / rounds, 2),
                                 "redo": round(B[:, 16].sum() / rounds, 3)},
        "tasks_per_wave": float(B[:, 8].mean()), "rounds_per_wave": float(B[:, 9].mean())}), flush=True)
