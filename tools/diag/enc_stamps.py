#!/usr/bin/env python3
"""Per-phase shader-clock breakdown of k_encode (a DE_STAMPS build,
tools/diag/lib_estamps.so from `PATCH=tools/diag/patches/r5_enc_stamps.patch
build_variants.sh estamps:-DDE_STAMPS`): prologue, pads, chunk wait +
lookups, scan + ORs, pads/prefixes, stores, zeroing/carry.  Cycles per
wave-round and shares per config, after a 512 MiB read (clean cache)."""
import ctypes, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
vp, u32, u64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
L = ctypes.CDLL(os.path.join(HERE, "lib_estamps.so"), mode=ctypes.RTLD_LOCAL)
L.nghttp2_amd_hd__enc_stamps.argtypes = [vp, ctypes.c_int]
L.nghttp2_amd_hd_huff_encode_batch.argtypes = [vp, vp, u32, vp, sz, vp, vp, sz, vp]
L.nghttp2_amd_hd_huff_encode_workspace_size.restype = sz
L.nghttp2_amd_hd_huff_encode_workspace_size.argtypes = [u64, u32]
L.nghttp2_amd_hd_huff_encode_bound.restype = sz
L.nghttp2_amd_hd_huff_encode_bound.argtypes = [u64, u32]
P = lambda t: ctypes.c_void_p(t.data_ptr())
NAMES = ["prologue_scans", "pads", "wait_lookup_quads", "scan_or", "pads_prefix_barrier", "stores", "zero_carry",
         "pro_staging", "pro_bits_offsets", None, "pro_tile_prefix"]
KS = [0, 7, 8, 10, 1, 2, 3, 4, 5, 6]
dev = torch.device("cuda:0")
FL = torch.ones(512 << 20, dtype=torch.uint8, device=dev)
buf = np.zeros(16, dtype=np.uint64)
for cfg in [int(c) for c in sys.argv[1:]] or [3, 2]:
    pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
    n, R = len(off) - 1, int(off[-1])
    src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
    cap = L.nghttp2_amd_hd_huff_encode_bound(R, n)
    d = torch.empty(cap, dtype=torch.uint8, device=dev); do = torch.empty(n + 1, dtype=torch.int32, device=dev)
    wsz = L.nghttp2_amd_hd_huff_encode_workspace_size(R, n); ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    run = lambda: L.nghttp2_amd_hd_huff_encode_batch(P(src), P(so), n, P(d), cap, P(do), P(ws), wsz, s)
    run(); torch.cuda.synchronize()
    L.nghttp2_amd_hd__enc_stamps(buf.ctypes.data, 1)
    K = 5
    for _ in range(K):
        FL.view(torch.int32).max(); run()
    torch.cuda.synchronize()
    L.nghttp2_amd_hd__enc_stamps(buf.ctypes.data, 1)
    rounds = buf[9] / K
    tot = float(sum(buf[k] for k in KS))
    print(json.dumps({"config": cfg, "wave_rounds": int(rounds),
                      "cycles_per_wave_round": {NAMES[k]: round(float(buf[k]) / K / rounds, 1) for k in KS},
                      "share": {NAMES[k]: round(float(buf[k]) / tot, 3) for k in KS}}), flush=True)
