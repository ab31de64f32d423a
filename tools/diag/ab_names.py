#!/usr/bin/env python3
"""A/B of the name-token kernel in one process: the in-tree library against
tools/diag/lib_names_r1.so (hd_names.hip built alone with the other
NAMES_BAL setting), on 1M mixed names (2 % long) and 1M short names; outputs
checked equal."""
import ctypes, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
from nghttp2_amd import hd
dev = torch.device("cuda:0")
vp, u32 = ctypes.c_void_p, ctypes.c_uint32
ARGS = [vp, vp, u32, vp, vp, vp]
L0 = hd.lib()
L0.nghttp2_amd_hd_name_tokens_batch.argtypes = ARGS
L1 = ctypes.CDLL(os.path.join(HERE, "lib_names_r1.so"), mode=ctypes.RTLD_LOCAL)
L1.nghttp2_amd_hd_name_tokens_batch.argtypes = ARGS
kern = {"product": L0.nghttp2_amd_hd_name_tokens_batch, "other": L1.nghttp2_amd_hd_name_tokens_batch}
for tag, lf in (("mixed", 0.02), ("short", 0.0)):
    pool, off = W.gen_names(1 << 20, long_frac=lf)
    n = len(off) - 1
    src = torch.zeros(int(off[-1]) + 64, dtype=torch.uint8, device=dev)
    src[:int(off[-1])] = torch.from_numpy(pool[:int(off[-1])]).to(dev)
    so = torch.from_numpy(off.astype(np.uint32).view(np.int32)).to(dev)
    out = {k: (torch.zeros(n, dtype=torch.int32, device=dev), torch.zeros(n, dtype=torch.int32, device=dev)) for k in kern}
    s = torch.cuda.current_stream()
    def run(k):
        t, h = out[k]
        assert kern[k](vp(src.data_ptr()), vp(so.data_ptr()), n, vp(t.data_ptr()), vp(h.data_ptr()), vp(s.cuda_stream)) == 0
    for k in kern:
        run(k)
    torch.cuda.synchronize()
    assert torch.equal(out["product"][0], out["other"][0]) and torch.equal(out["product"][1], out["other"][1])
    res = {k: [] for k in kern}
    for _ in range(20):
        for k in kern:
            a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
            a.record(s); run(k); b.record(s); torch.cuda.synchronize()
            res[k].append(a.elapsed_time(b) * 1000)
    print(json.dumps({tag: {k: round(float(np.median(v)), 1) for k, v in res.items()}, "bytes": int(off[-1])}), flush=True)
