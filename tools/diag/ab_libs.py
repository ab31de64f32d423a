#!/usr/bin/env python3
"""One-process A/B of library builds (tools/diag/lib_*.so, built by
build_variants.sh): decode_batch_auto and encode_batch on configs 3 / 2 / 5,
outputs checked equal across the variants (decode: bytes, offsets, status,
fstate, flags; encode: bytes and offsets), then interleaved event-timed
rounds (cdna_hip_programming.md 5.4 rule 24).  Usage: ab_libs.py [cfg ...]"""
import ctypes, glob, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd

vp, u32, u64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
dev = torch.device("cuda:0")
libs = {}
for p in sorted(glob.glob(os.path.join(HERE, "lib_*.so"))):
    L = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
    L.nghttp2_amd_hd_huff_decode_batch_auto.argtypes = [vp, vp, u32, u64, vp, sz, vp, vp, vp, vp, vp]
    L.nghttp2_amd_hd_huff_encode_batch.argtypes = [vp, vp, u32, vp, sz, vp, vp, sz, vp]
    L.nghttp2_amd_hd_huff_encode_count_batch.argtypes = [vp, vp, u32, vp, vp]
    L.nghttp2_amd_hd_emit_strings_batch.argtypes = [vp, vp, u32, u64, vp, sz, vp, vp, sz, vp]
    L.nghttp2_amd_hd_emit_strings_workspace_size.restype = sz
    L.nghttp2_amd_hd_emit_strings_workspace_size.argtypes = [u64, u32]
    L.nghttp2_amd_hd_emit_strings_bound.restype = sz
    L.nghttp2_amd_hd_emit_strings_bound.argtypes = [u64, u32]
    libs[os.path.basename(p)[4:-3]] = L
codec = nghttp2_amd.HuffmanBatchCodec(dev)
s = torch.cuda.current_stream()
P = lambda t: ctypes.c_void_p(t.data_ptr())
ROUNDS = int(os.environ.get("ROUNDS", "10"))


# FLUSH=write: write 512 MiB (twice the Infinity Cache) before every timed
# call, so the call reads its inputs from HBM behind dirty lines' write-backs
# (the pipelined bench's state after a decode); FLUSH=read: read them, so
# the call starts on a clean cache that holds none of its inputs
FLUSH_MODE = os.environ.get("FLUSH", "")
FLUSH = torch.ones(512 << 20, dtype=torch.uint8, device=dev) if FLUSH_MODE else None


def timed(fn, keys):
    res = {k: [] for k in keys}
    for _ in range(ROUNDS):
        for k in keys:
            if FLUSH is not None:
                if FLUSH_MODE == "read":
                    FLUSH.view(torch.int32).max()
                else:
                    FLUSH.fill_(1)
            a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
            a.record(s); fn(k); b.record(s); torch.cuda.synchronize()
            res[k].append(a.elapsed_time(b) * 1000)
    return {k: {"median_us": round(float(np.median(v)), 1), "min_us": round(float(np.min(v)), 1)}
            for k, v in res.items()}


for cfg in [int(c) for c in sys.argv[1:]] or [3, 2, 5]:
    print("config", cfg, "libs", sorted(libs), file=sys.stderr, flush=True)
    if cfg == 5:
        pool, off = W.gen_adversarial(1 << 20)[:2]
        enc = torch.from_numpy(pool).to(dev)
        eo = torch.from_numpy(off.view(np.int32)).to(dev)
        src = None
    else:
        pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
        src = torch.from_numpy(pool).to(dev)
        so = torch.from_numpy(off.view(np.int32)).to(dev)
        enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
    torch.cuda.synchronize()
    n = len(off) - 1
    E = int(eo[-1].item()) & 0xFFFFFFFF
    dcap = codec.decode_bound(E, n)
    dst = torch.empty(dcap, dtype=torch.uint8, device=dev)
    doff = torch.empty(n + 1, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    fs = torch.empty(n, dtype=torch.int16, device=dev)
    fl = torch.empty(n, dtype=torch.uint8, device=dev)

    def dec(k):
        rc = libs[k].nghttp2_amd_hd_huff_decode_batch_auto(P(enc), P(eo), n, E, P(dst), dcap, P(doff),
                                                           P(st), P(fs), P(fl), ctypes.c_void_p(s.cuda_stream))
        assert rc == 0, (k, rc)
    ref = None
    same = {}
    for k in ([] if os.environ.get("SKIP_DECODE") else libs):
        dst.fill_(0xA5); st.zero_()
        for _ in range(2):
            dec(k)
        torch.cuda.synchronize()
        used = int(doff[-1].item()) & 0xFFFFFFFF
        # each string's bytes gathered through the library's own offsets (the
        # offsets and the gaps between tasks' outputs move with the task
        # decomposition; status, state and bytes may not)
        w = torch.clamp(st, min=0).long()
        starts = torch.repeat_interleave(doff[:n].long() & 0xFFFFFFFF, w)
        rel = torch.arange(int(w.sum().item()), device=dev) - torch.repeat_interleave(torch.cumsum(w, 0) - w, w)
        cur = (dst[starts + rel].clone(), st.clone(), fs.clone(), fl.clone())
        if ref is None:
            ref = cur
        same[k] = all(torch.equal(x, y) for x, y in zip(ref, cur))
    out = {"config": cfg, "n": n, "E": E, "decode_same": same,
           "decode": {} if os.environ.get("SKIP_DECODE") else timed(dec, list(libs))}
    if src is not None and not os.environ.get("SKIP_ENCODE"):
        ecap = codec.encode_bound(int(off[-1]), n)
        edst = torch.empty(ecap, dtype=torch.uint8, device=dev)
        eoff = torch.empty(n + 1, dtype=torch.int32, device=dev)
        # (the largest workspace any library asks for: their layouts may differ)
        for L_ in libs.values():
            L_.nghttp2_amd_hd_huff_encode_workspace_size.restype = sz
            L_.nghttp2_amd_hd_huff_encode_workspace_size.argtypes = [u64, u32]
        wsz = max(L_.nghttp2_amd_hd_huff_encode_workspace_size(int(off[-1]), n) for L_ in libs.values())
        ws = torch.empty(wsz, dtype=torch.uint8, device=dev)

        def encf(k):
            rc = libs[k].nghttp2_amd_hd_huff_encode_batch(P(src), P(so), n, P(edst), ecap, P(eoff), P(ws),
                                                          wsz, ctypes.c_void_p(s.cuda_stream))
            assert rc == 0, (k, rc)
        esame = {}
        count_only = bool(os.environ.get("COUNT_ONLY"))  # ablation builds whose counts are wrong
        for k in ([] if count_only else libs):
            edst.zero_()
            encf(k)
            torch.cuda.synchronize()
            esame[k] = bool(torch.equal(edst[:E], enc[:E]) and torch.equal(eoff, eo))
        out["encode_same"] = esame
        out["encode"] = {} if count_only else timed(encf, list(libs))
        clen = torch.empty(n, dtype=torch.int32, device=dev)

        def cntf(k):
            rc = libs[k].nghttp2_amd_hd_huff_encode_count_batch(P(src), P(so), n, P(clen),
                                                                ctypes.c_void_p(s.cuda_stream))
            assert rc == 0, (k, rc)
        out["count"] = timed(cntf, list(libs))
        if count_only:
            # counts (bits per string) of each library against the first one
            ref_c, csame = None, {}
            for k in libs:
                cntf(k)
                torch.cuda.synchronize()
                c = clen.clone()
                ref_c = c if ref_c is None else ref_c
                csame[k] = bool(torch.equal(c, ref_c))
            out["count_same"] = csame
            print(json.dumps(out), flush=True)
            continue
        # emit_strings (string literals): each library with its own workspace
        R = int(off[-1])
        fcap = max(L.nghttp2_amd_hd_emit_strings_bound(R, n) for L in libs.values())
        fdst = torch.empty(fcap, dtype=torch.uint8, device=dev)
        foff = torch.empty(n + 1, dtype=torch.int32, device=dev)
        fws = {k: torch.empty(L.nghttp2_amd_hd_emit_strings_workspace_size(R, n) + 256,
                              dtype=torch.uint8, device=dev) for k, L in libs.items()}

        def emitf(k):
            w = fws[k]
            wp = ctypes.c_void_p(w.data_ptr() + (256 - w.data_ptr() % 256) % 256)
            rc = libs[k].nghttp2_amd_hd_emit_strings_batch(P(src), P(so), n, R, P(fdst), fcap, P(foff), wp,
                                                           libs[k].nghttp2_amd_hd_emit_strings_workspace_size(R, n),
                                                           ctypes.c_void_p(s.cuda_stream))
            assert rc == 0, (k, rc)
        fref, fsame = None, {}
        for k in libs:
            fdst.zero_()
            emitf(k)
            torch.cuda.synchronize()
            used = int(foff[-1].item()) & 0xFFFFFFFF
            cur = (fdst[:used].clone(), foff.clone())
            fref = fref or cur
            fsame[k] = all(torch.equal(x, y) for x, y in zip(fref, cur))
        out["emit_same"] = fsame
        out["emit"] = timed(emitf, list(libs))
    print(json.dumps(out), flush=True)
