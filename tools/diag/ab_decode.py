#!/usr/bin/env python3
"""A/B timing of decode kernels in ONE process, interleaved rounds
(cdna_hip_programming.md 5.4 rule 24): the product's decode_batch_auto
(dense), the round-1 engine-slot kernel (nghttp2_amd_hd__decode_batch_slots)
and decode_batch_auto of every tools/diag/lib_*.so variant.  Statuses are
checked equal across kernels; the dense variants' outputs equal the
product's.  Usage: ab_decode.py [config 2|3|5 ...]"""
import ctypes, glob, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd
from nghttp2_amd import hd

dev = torch.device("cuda:0")
vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
ARGS = [vp, vp, u32, vp, sz, vp, vp, vp, vp, vp]


def load(path):
    L = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    L.nghttp2_amd_hd_huff_decode_batch_auto.argtypes = ARGS
    return L


def main():
    cfgs = [int(x) for x in sys.argv[1:]] or [3, 2, 5]
    codec = nghttp2_amd.HuffmanBatchCodec(dev)
    L0 = hd.lib()
    L0.nghttp2_amd_hd__decode_batch_slots.argtypes = ARGS
    L0.nghttp2_amd_hd__decode_batch_pieces.argtypes = ARGS
    L0.nghttp2_amd_hd__decode_batch_items.argtypes = ARGS + [ctypes.c_int]
    kern = {"dense": L0.nghttp2_amd_hd_huff_decode_batch_auto,
            "slots_r1": L0.nghttp2_amd_hd__decode_batch_slots,
            "pieces": L0.nghttp2_amd_hd__decode_batch_pieces}
    for pc in (64, 67, 68, 70, 71, 40, 32):
        kern["items%d" % pc] = (lambda pc: lambda *a: L0.nghttp2_amd_hd__decode_batch_items(*a, pc))(pc)
    for p in sorted(glob.glob(os.path.join(HERE, "lib_x*.so"))):  # extra instances (DD_XINST builds)
        Lx = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
        Lx.nghttp2_amd_hd__decode_batch_items.argtypes = ARGS + [ctypes.c_int]
        for pc in (41, 44, 33, 36, 30):
            kern["%s_%d" % (os.path.basename(p)[4:-3], pc)] = (
                lambda L_, pc: lambda *a: L_.nghttp2_amd_hd__decode_batch_items(*a, pc))(Lx, pc)
    for p in sorted(glob.glob(os.path.join(HERE, "lib_*.so"))):
        if not os.path.basename(p).startswith("lib_x"):
            kern[os.path.basename(p)[4:-3]] = load(p).nghttp2_amd_hd_huff_decode_batch_auto
    out = {}
    for cfg in cfgs:
        if cfg == 5:
            pool, off, _ = W.gen_adversarial(1 << 20)
            enc = torch.from_numpy(pool).to(dev)
            eo = torch.from_numpy(off.view(np.int32)).to(dev)
        else:
            pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
            src = torch.from_numpy(pool).to(dev)
            so = torch.from_numpy(off.view(np.int32)).to(dev)
            enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
        torch.cuda.synchronize()
        E = int(eo[-1].item())
        n = eo.numel() - 1
        cap = codec.decode_bound(E, n)
        bufs = {k: (torch.zeros(cap, dtype=torch.uint8, device=dev),
                    torch.zeros(n + 1, dtype=torch.int32, device=dev),
                    torch.zeros(n, dtype=torch.int32, device=dev)) for k in kern}
        s = torch.cuda.current_stream()

        def run(k):
            d, do, st = bufs[k]
            rv = kern[k](ctypes.c_void_p(enc.data_ptr()), ctypes.c_void_p(eo.data_ptr()), n,
                         ctypes.c_void_p(d.data_ptr()), cap, ctypes.c_void_p(do.data_ptr()),
                         ctypes.c_void_p(st.data_ptr()), None, None, ctypes.c_void_p(s.cuda_stream))
            assert rv == 0, (k, rv)
        for k in list(kern):
            d, do, st = bufs[k]
            rv = kern[k](ctypes.c_void_p(enc.data_ptr()), ctypes.c_void_p(eo.data_ptr()), n,
                         ctypes.c_void_p(d.data_ptr()), cap, ctypes.c_void_p(do.data_ptr()),
                         ctypes.c_void_p(st.data_ptr()), None, None, ctypes.c_void_p(s.cuda_stream))
            if rv != 0:  # (an instance this build does not have)
                del kern[k]
                continue
            for _ in range(3):
                run(k)
        torch.cuda.synchronize()
        ref = bufs["dense"]
        for k in list(kern):
            if k.startswith("abl"):
                continue  # ablation builds give wrong output on purpose
            bad = not torch.equal(bufs[k][2], ref[2])
            if not bad and k not in ("slots_r1", "pieces"):
                bad = not (torch.equal(bufs[k][1], ref[1]) and torch.equal(bufs[k][0], ref[0]))
            if bad:  # report (first differing strings) and leave the variant out
                d = (bufs[k][2] != ref[2]).nonzero().flatten()[:8].tolist()
                print(json.dumps({"config": cfg, "variant": k, "MISMATCH": True, "status_idx": d,
                                  "ref": [int(ref[2][i]) for i in d],
                                  "got": [int(bufs[k][2][i]) for i in d]}), flush=True)
                del kern[k]
        res = {k: [] for k in kern}
        for _ in range(10):
            for k in kern:
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record(s)
                run(k)
                b.record(s)
                torch.cuda.synchronize()
                res[k].append(a.elapsed_time(b) * 1000)
        out["config%d" % cfg] = {k: {"median_us": round(float(np.median(v)), 1),
                                     "min_us": round(float(np.min(v)), 1)} for k, v in res.items()}
        print(json.dumps({"config%d" % cfg: out["config%d" % cfg]}), flush=True)


if __name__ == "__main__":
    main()
