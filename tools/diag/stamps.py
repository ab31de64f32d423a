#!/usr/bin/env python3
"""Per-phase shader-clock breakdown of the item decoder (a DD_STAMPS build of
the engine, tools/diag/lib_stamps.so from
`PATCH=tools/diag/patches/r4_diag_hooks.patch build_variants.sh stamps:-DDD_STAMPS`):
task setup, item map, staging,
warm-up, decode + verify, scans + finish, store, round tails.  Cycles per
wave-round and shares, per config.  The stamps themselves cost ~10 %."""
import ctypes, json, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import nghttp2_amd
from nghttp2_amd import workloads as W
vp, u32, u64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
L = ctypes.CDLL(os.path.join(HERE, "lib_stamps.so"), mode=ctypes.RTLD_LOCAL)
L.nghttp2_amd_hd__stamps.argtypes = [vp, ctypes.c_int]
L.nghttp2_amd_hd_huff_decode_batch_auto.argtypes = [vp, vp, u32, u64, vp, sz, vp, vp, vp, vp, vp]
P = lambda t: ctypes.c_void_p(t.data_ptr())
NAMES = ["task_setup", "item_map", "prefetch_issue", "warmup", "decode_verify", "scans_finish", "store", "tails",
         None, "stage_wait_write"]
dev = torch.device("cuda:0")
codec = nghttp2_amd.HuffmanBatchCodec(dev)
buf = np.zeros(16, dtype=np.uint64)
for cfg in [int(c) for c in sys.argv[1:]] or [3, 2, 5]:
    if cfg == 5:
        pool, off = W.gen_adversarial(1 << 20)[:2]
        enc = torch.from_numpy(pool).to(dev); eo = torch.from_numpy(off.view(np.int32)).to(dev)
    else:
        pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
        src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
        enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
    torch.cuda.synchronize()
    E = int(eo[-1].item()) & 0xFFFFFFFF
    n = eo.numel() - 1
    dcap = codec.decode_bound(E, n)
    dst = torch.empty(dcap, dtype=torch.uint8, device=dev)
    doff = torch.empty(n + 1, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def dec():
        rc = L.nghttp2_amd_hd_huff_decode_batch_auto(P(enc), P(eo), n, E, P(dst), dcap, P(doff), P(st),
                                                     None, None, s)
        assert rc == 0, rc
    for _ in range(3):
        dec()
    torch.cuda.synchronize()
    L.nghttp2_amd_hd__stamps(ctypes.c_void_p(buf.ctypes.data), 1)
    reps = 10
    for _ in range(reps):
        dec()
    torch.cuda.synchronize()
    L.nghttp2_amd_hd__stamps(ctypes.c_void_p(buf.ctypes.data), 1)
    rounds = float(buf[8])
    tot = float(sum(buf[i] for i, k in enumerate(NAMES) if k))
    out = {"config": cfg, "wave_rounds_per_launch": rounds / reps,
           "cycles_per_round": {k: round(float(buf[i]) / rounds, 1) for i, k in enumerate(NAMES) if k},
           "share": {k: round(float(buf[i]) / tot, 3) for i, k in enumerate(NAMES) if k}}
    print(json.dumps(out), flush=True)
