#!/usr/bin/env python3
"""Per-phase cycle shares of k_decode from the HD_DIAG_STAMPS build."""
import ctypes, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
WPG = 8  # waves per decode workgroup (DEC_NT / 64)
dev = torch.device("cuda:0")
pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
codec = nghttp2_amd.HuffmanBatchCodec(dev)
src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
enc, eo = codec.encode(src, so, raw_bytes=int(off[-1])); torch.cuda.synchronize()
E = int(eo[-1].item()); n = len(off) - 1
L = ctypes.CDLL(os.path.join(HERE, "lib_stamps.so"), mode=ctypes.RTLD_LOCAL)
vp = ctypes.c_void_p
L.nghttp2_amd_hd_huff_decode_batch_auto.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_size_t, vp, vp, vp, vp, vp]
cap = codec.decode_bound(E, n)
dst = torch.empty(cap, dtype=torch.uint8, device=dev); doff = torch.empty(n + 1, dtype=torch.int32, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
def run():
    L.nghttp2_amd_hd_huff_decode_batch_auto(vp(enc.data_ptr()), vp(eo.data_ptr()), n, vp(dst.data_ptr()), cap,
        vp(doff.data_ptr()), vp(st.data_ptr()), None, None, vp(s.cuda_stream))
run(); torch.cuda.synchronize()
L.nghttp2_amd_hd__diag_stamps(None, 1)
run(); torch.cuda.synchronize()
buf = np.zeros((4096, 16), dtype=np.uint64)
L.nghttp2_amd_hd__diag_stamps(vp(buf.ctypes.data), 0)
names = ["tile", "stage+sort", "pass1", "verify", "scan", "pass2", "copyout", "unused"]
tot = buf[:, :8].sum(axis=0).astype(float)
used = buf[:, 11] > 0
print(json.dumps({"config": cfg, "wgs": int(used.sum()),
                  "share": {k: round(float(v / tot.sum()), 4) for k, v in zip(names, tot)},
                  "cycles_per_wg_median": {k: float(np.median(buf[used, i])) for i, k in enumerate(names)},
                  "verify_iters_per_round": float(buf[:, 8].sum() / max(1, buf[:, 10].sum())),
                  "mismatches_per_round": float(buf[:, 9].sum() / max(1, buf[:, 10].sum())),
                  "rounds": int(buf[:, 10].sum()), "tiles": int(buf[:, 11].sum()),
                  "wave_trips_per_round": {"fast": float(buf[:, 12].sum() / max(1, buf[:, 10].sum()) / WPG),
                                           "checked": float(buf[:, 13].sum() / max(1, buf[:, 10].sum()) / WPG),
                                           "warm": float(buf[:, 14].sum() / max(1, buf[:, 10].sum()) / WPG)},
                  "wave_pass1_cycles_per_round": float(buf[:, 15].sum() / max(1, buf[:, 10].sum()) / WPG)}, indent=1))
