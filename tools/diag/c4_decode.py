#!/usr/bin/env python3
"""Config-4 (16M strings) decode with one decoder instance, timed, with
progress lines (diagnosis).  Usage: c4_decode.py PIECE [STRINGS]"""
import os, sys, time
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from nghttp2_amd import workloads as W
import nghttp2_amd
t0 = time.perf_counter()
def p(m): print("[%6.1fs] %s" % (time.perf_counter() - t0, m), flush=True)
piece = int(sys.argv[1]); n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 24
dev = torch.device("cuda:0")
lengths = W.mixed_lengths(n)
pool, off = W.gen_mixed_range(lengths, 0, n)
p("generated %d strings %d bytes" % (n, int(off[-1])))
codec = nghttp2_amd.HuffmanBatchCodec(dev)
src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
enc, eo = codec.encode(src, so, raw_bytes=int(off[-1])); torch.cuda.synchronize()
E = int(eo[-1].item()) & 0xFFFFFFFF
p("encoded %d" % E)
dst, do, st = codec.decode_auto(enc, eo, enc_bytes=E, piece=piece); torch.cuda.synchronize()
p("decoded once")
a = time.perf_counter()
for _ in range(3):
    codec.decode_auto(enc, eo, enc_bytes=E, dst=dst, dst_off=do, status=st, piece=piece)
torch.cuda.synchronize()
p("3 decodes: %.2f ms each" % ((time.perf_counter() - a) / 3 * 1e3))
ln = torch.from_numpy(np.diff(off.astype(np.int64)).astype(np.int32)).to(dev)
p("status == length: %s" % bool(torch.equal(st, ln)))
if len(sys.argv) > 3 and sys.argv[3] == "streams":
    # two streams, each its own buffers: encode + decode concurrently (bench.py's pipes)
    s1 = torch.cuda.Stream(device=dev)
    enc_cap = E + 4096
    bufs = []
    for k in range(2):
        c = nghttp2_amd.HuffmanBatchCodec(dev)
        bufs.append((c, torch.empty(enc_cap, dtype=torch.uint8, device=dev),
                     torch.empty(n + 1, dtype=torch.int32, device=dev),
                     torch.empty(codec.decode_bound(E, n), dtype=torch.uint8, device=dev),
                     torch.empty(n + 1, dtype=torch.int32, device=dev),
                     torch.empty(n, dtype=torch.int32, device=dev)))
    torch.cuda.synchronize()
    p("stream buffers ready")
    for k, sm in enumerate((torch.cuda.current_stream(), s1)):
        c, e_, eo_, d_, do_, st_ = bufs[k]
        c.encode(src, so, raw_bytes=int(off[-1]), dst=e_, dst_off=eo_, stream=sm)
        p("encode %d launched" % k)
        c.decode_auto(e_, eo_, enc_bytes=E, dst=d_, dst_off=do_, status=st_, stream=sm, piece=piece)
        p("decode %d launched" % k)
    torch.cuda.synchronize()
    p("both streams done; status equal: %s" % bool(torch.equal(bufs[0][5], bufs[1][5])))
