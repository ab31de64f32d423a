import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np, torch
import nghttp2_amd
from oracle import oracle as O
dev = torch.device("cuda:0")
codec = nghttp2_amd.HuffmanBatchCodec(dev)
for strs in ([b"a"], [b"abc"], [b"\xff"], [b"hello world this is a test of it"], [b"ab", b"cd", b"ef"], [b"x" * 40]):
    off = np.zeros(len(strs) + 1, np.uint32); off[1:] = np.cumsum([len(s) for s in strs])
    pool = np.frombuffer(b"".join(strs) + b"\0" * 64, np.uint8)
    src = torch.from_numpy(pool.copy()).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
    enc, eo = codec.encode(src, so, raw_bytes=int(off[-1]))
    torch.cuda.synchronize()
    e = enc.cpu().numpy(); o = eo.cpu().numpy().view(np.uint32)
    re, ro = O.encode_batch(pool[:int(off[-1])], off)
    print(strs[0][:8], "gpu", o.tolist(), bytes(e[:o[-1]]).hex(), "ref", ro.tolist(), bytes(re[:ro[-1]]).hex())
