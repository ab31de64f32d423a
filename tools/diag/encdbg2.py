"""Debug helper: encode a workload on the GPU and report mismatching strings vs the oracle."""
import sys, os
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import nghttp2_amd
from nghttp2_amd import workloads as W
from oracle import oracle as O
dev = torch.device("cuda:0")
codec = nghttp2_amd.HuffmanBatchCodec(dev)
for name, (pool, off) in [("pseudo_1k", W.gen_pseudo_headers(1000)), ("mixed_200", W.gen_mixed_values(200)),
                          ("pseudo_4096", W.gen_pseudo_headers(4096))]:
    src = torch.from_numpy(pool).to(dev); so = torch.from_numpy(off.view(np.int32)).to(dev)
    enc, eo = codec.encode(src, so, raw_bytes=int(off[-1])); torch.cuda.synchronize()
    eo = eo.cpu().numpy().view(np.uint32); enc = enc.cpu().numpy()
    renc, roff = O.encode_batch(pool, off)
    print(name, "offsets equal:", np.array_equal(eo, roff), "E", int(roff[-1]))
    bad = np.nonzero(enc[:int(roff[-1])] != renc)[0]
    print("  bad bytes:", len(bad), bad[:10])
    if len(bad):
        s = np.searchsorted(roff, bad, side="right") - 1
        us = np.unique(s)
        print("  bad strings:", len(us), us[:20], "waves", np.unique(us // 64)[:20])
        for i in us[:3]:
            a, b = roff[i], roff[i + 1]
            print("   str", i, "raw", off[i], off[i+1], "enc", a, b, "gpu", enc[a:b][:16].tolist(), "ref", renc[a:b][:16].tolist())
