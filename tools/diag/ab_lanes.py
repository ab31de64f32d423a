#!/usr/bin/env python3
"""Lane decoder (nghttp2_amd_hd__decode_batch_lanes) vs the oracle and vs the
item decoder (decode_batch_auto), one process, interleaved timing.

Parity: caller-slot mode (the oracle's floor(8E/5)+1 slots, zero-initialised
pool) must equal the oracle's whole pool, status, fstate and flags; auto-slot
mode must give the same status / context and, for every string that decodes,
the same bytes.  Usage: ab_lanes.py [config 2|3|5 ...]"""
import ctypes, json, os, sys, time
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd
from nghttp2_amd import hd
from oracle import oracle as O

dev = torch.device("cuda:0")
vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None


def main():
    cfgs = [int(x) for x in sys.argv[1:]] or [3, 2, 5]
    codec = nghttp2_amd.HuffmanBatchCodec(dev)
    L = hd.lib()
    L.nghttp2_amd_hd__decode_batch_lanes.argtypes = [vp, vp, u32, vp, sz, vp, vp, vp, vp, vp,
                                                     ctypes.c_int]
    s = torch.cuda.current_stream()
    for cfg in cfgs:
        t0 = time.time()
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
        n = eo.numel() - 1
        E = int(eo[-1].item())
        enc_h = enc.cpu().numpy()[:E]
        eo_h = eo.cpu().numpy().view(np.uint32).copy()
        rd, rdo, rst, rfs, rfl = O.decode_batch(enc_h, eo_h, nthreads=16)
        print(json.dumps({"config": cfg, "n": n, "E": E, "oracle_s": round(time.time() - t0, 1)}),
              flush=True)
        capA = codec.decode_bound(E, n)
        # lane decoder's auto slots need 16 n more than the item decoder's bound
        capL = (E * 8) // 5 + 16 * n + 32
        exact_off = torch.from_numpy(rdo.view(np.int32)).to(dev)
        bufs = {}

        def mk(cap):
            return (torch.zeros(cap, dtype=torch.uint8, device=dev),
                    torch.zeros(n + 1, dtype=torch.int32, device=dev),
                    torch.zeros(n, dtype=torch.int32, device=dev),
                    torch.zeros(n, dtype=torch.int16, device=dev),
                    torch.zeros(n, dtype=torch.uint8, device=dev))
        bufs["items"] = mk(capA)
        bufs["lanes"] = mk(capL)
        bufs["lanes_nosort"] = mk(capL)
        bufs["lanes2"] = mk(64 * ((((E * 8) // 5) + 63) // 64 + n))
        bufs["lanes_exact"] = mk(int(rdo[-1]) + 16)
        bufs["lanes_exact"][1].copy_(exact_off)

        def run(k, ctx=True):
            d, do, st, fs, fl = bufs[k]
            f1, f2 = (P(fs), P(fl)) if ctx else (None, None)
            if k == "items":
                rv = L.nghttp2_amd_hd_huff_decode_batch_auto(P(enc), P(eo), n, P(d), d.numel(), P(do),
                                                             P(st), f1, f2, ctypes.c_void_p(s.cuda_stream))
            else:
                mode = {"lanes": 0, "lanes_nosort": 2, "lanes_exact": 1, "lanes2": 4}[k]
                rv = L.nghttp2_amd_hd__decode_batch_lanes(P(enc), P(eo), n, P(d), d.numel(), P(do),
                                                          P(st), f1, f2,
                                                          ctypes.c_void_p(s.cuda_stream), mode)
            assert rv == 0, (k, rv)
        for k in bufs:
            run(k)
        torch.cuda.synchronize()
        # parity
        d, do, st, fs, fl = [x.cpu().numpy() for x in bufs["lanes_exact"]]
        res = {"config": cfg}
        res["exact_status"] = bool(np.array_equal(st, rst))
        res["exact_fstate"] = bool(np.array_equal(fs.view(np.uint16), rfs))
        res["exact_flags"] = bool(np.array_equal(fl, rfl))
        res["exact_bytes"] = bool(np.array_equal(d[:int(rdo[-1])], rd[:int(rdo[-1])]))
        if not res["exact_status"]:
            bad = np.nonzero(st != rst)[0][:6]
            res["exact_bad"] = [(int(i), int(st[i]), int(rst[i]), int(eo_h[i + 1] - eo_h[i])) for i in bad]
        if not res["exact_bytes"]:
            i = int(np.nonzero(d[:int(rdo[-1])] != rd[:int(rdo[-1])])[0][0])
            res["exact_first_bad_byte"] = i
            res["exact_first_bad_str"] = int(np.searchsorted(rdo, i, side="right") - 1)
        for k in ("lanes", "lanes_nosort", "lanes2"):
            d2, do2, st2, fs2, fl2 = [x.cpu().numpy() for x in bufs[k]]
            ok = np.array_equal(st2, rst) and np.array_equal(fs2.view(np.uint16), rfs) and \
                np.array_equal(fl2, rfl)
            do2 = do2.view(np.uint32)
            good = np.nonzero(rst > 0)[0]
            lens = rst[good].astype(np.int64)
            # gather every decoded string of both layouts
            idx_a = np.repeat(do2[good].astype(np.int64), lens) + (np.arange(lens.sum()) - np.repeat(np.cumsum(lens) - lens, lens))
            idx_r = np.repeat(rdo[good].astype(np.int64), lens) + (np.arange(lens.sum()) - np.repeat(np.cumsum(lens) - lens, lens))
            okb = bool(np.array_equal(d2[idx_a], rd[idx_r]))
            res[k + "_ctx"] = bool(ok)
            res[k + "_bytes"] = okb
        it = bufs["items"][2].cpu().numpy()
        res["items_status"] = bool(np.array_equal(it, rst))
        print(json.dumps(res), flush=True)
        # timing, interleaved
        tm = {k: [] for k in bufs}
        for _ in range(10):
            for k in bufs:
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record(s)
                run(k, ctx=False)
                b.record(s)
                torch.cuda.synchronize()
                tm[k].append(a.elapsed_time(b) * 1000)
        print(json.dumps({"config%d" % cfg: {k: {"median_us": round(float(np.median(v)), 1),
                                                  "min_us": round(float(np.min(v)), 1)}
                                              for k, v in tm.items()}}), flush=True)


if __name__ == "__main__":
    main()
