import sys, numpy as np, torch
sys.path.insert(0, '.')
from nghttp2_amd import workloads as W
import nghttp2_amd
from oracle import oracle as O
pool, off = W.gen_pseudo_headers(63)
dev = torch.device('cuda:0')
codec = nghttp2_amd.HuffmanBatchCodec(dev)
src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
enc, eo = codec.encode(src, so, raw_bytes=int(off[-1])); torch.cuda.synchronize()
enc = enc.cpu().numpy(); eo = eo.cpu().numpy().astype(np.int64)
renc, reo = O.encode_batch(pool, off)
print("offsets equal", np.array_equal(eo, reo.astype(np.int64)))
L = np.diff(off.astype(np.int64))
m = np.maximum(1, -(-L // 32)); P = np.cumsum(m)
for s in range(len(off) - 1):
    a, b = int(reo[s]), int(reo[s + 1])
    if not np.array_equal(enc[a:b], renc[a:b]):
        print("string", s, "raw", L[s], "pieces", m[s], "first piece idx", P[s] - m[s], "enc", a, b)
        d = np.nonzero(enc[a:b] != renc[a:b])[0]
        print("  diff at", d[:10], "got", enc[a:b][d[:5]], "want", renc[a:b][d[:5]])
        break
