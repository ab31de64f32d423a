#!/usr/bin/env python3
"""A/B timing of the encode pair (k_enc_count + k_encode) in ONE process,
interleaved: the product's nghttp2_amd_hd_huff_encode_batch against the
round-1 kernels (nghttp2_amd_hd__encode_batch_r1).  Outputs are checked
equal.  Usage: ab_encode.py [config 2|3|9 ...]  (9 = all byte values)"""
import ctypes, glob, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
from nghttp2_amd import hd

dev = torch.device("cuda:0")
vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
ARGS = [vp, vp, u32, vp, sz, vp, vp, sz, vp]


def main():
    cfgs = [int(x) for x in sys.argv[1:]] or [3, 2]
    L = hd.lib()
    L.nghttp2_amd_hd__encode_batch_r1.argtypes = ARGS
    kern = {"product": L.nghttp2_amd_hd_huff_encode_batch, "r1": L.nghttp2_amd_hd__encode_batch_r1}
    for p in sorted(glob.glob(os.path.join(HERE, "lib_*.so"))):  # tools/diag variant builds
        Lv = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
        Lv.nghttp2_amd_hd_huff_encode_batch.argtypes = ARGS
        kern[os.path.basename(p)[4:-3]] = Lv.nghttp2_amd_hd_huff_encode_batch
    for cfg in cfgs:
        if cfg == 9:
            pool, off = W.gen_all_bytes(1 << 18)
        else:
            pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
        n = len(off) - 1
        R = int(off[-1])
        src = torch.zeros((R + 32 + 15) // 16 * 16, dtype=torch.uint8, device=dev)
        src[:R] = torch.from_numpy(pool[:R]).to(dev)
        so = torch.from_numpy(off.view(np.int32)).to(dev)
        cap = L.nghttp2_amd_hd_huff_encode_bound(R, n)
        wsz = L.nghttp2_amd_hd_huff_workspace_size(n)
        bufs = {k: (torch.zeros(cap, dtype=torch.uint8, device=dev),
                    torch.zeros(n + 1, dtype=torch.int32, device=dev),
                    torch.zeros(wsz, dtype=torch.uint8, device=dev)) for k in kern}
        s = torch.cuda.current_stream()

        def run(k):
            d, do, ws = bufs[k]
            rv = kern[k](vp(src.data_ptr()), vp(so.data_ptr()), n, vp(d.data_ptr()), cap,
                         vp(do.data_ptr()), vp(ws.data_ptr()), wsz, vp(s.cuda_stream))
            assert rv == 0, (k, rv)
        for k in kern:
            for _ in range(3):
                run(k)
        torch.cuda.synchronize()
        a = bufs["product"]
        E = int(a[1][-1].item())
        for k in kern:
            b = bufs[k]
            assert torch.equal(a[1], b[1]), k + ": offsets differ"
            assert torch.equal(a[0][:E], b[0][:E]), k + ": bytes differ"
        res = {k: [] for k in kern}
        for _ in range(10):
            for k in kern:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                run(k)
                e1.record(s)
                torch.cuda.synchronize()
                res[k].append(e0.elapsed_time(e1) * 1000)
        print(json.dumps({"config%d" % cfg: {k: {"median_us": round(float(np.median(v)), 1),
                                                 "min_us": round(float(np.min(v)), 1)}
                                             for k, v in res.items()}, "raw": R, "enc": E}),
              flush=True)


if __name__ == "__main__":
    main()
