#!/usr/bin/env python3
"""Decode write traffic vs output layout (DESIGN.md 2.3 sector hypothesis).

Encodes the config-2 batch once, then decodes it K times into
  auto   engine slots (nghttp2_amd_hd_huff_decode_batch_auto, k_decode<true>)
  slots  caller slots of floor(8E/5)+1 bytes (k_decode<false>, launches 1..K)
  tight  caller slots (launches K+1..2K) at the exact decoded offsets (the raw offsets;
         nghttp2_amd_hd_huff_decode_batch, k_decode<false>)
and checks both outputs.  Run under
  rocprofv3 --kernel-trace --pmc WRITE_SIZE -- python3 tools/diag/write_layout.py
and compare WRITE_SIZE per launch of the two k_decode instantiations."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main(k=5):
    import torch
    import nghttp2_amd
    from nghttp2_amd import workloads as W
    dev = torch.device("cuda:0")
    pool, off = W.gen_pseudo_headers(1 << 20)
    n, raw = len(off) - 1, int(off[-1])
    codec = nghttp2_amd.HuffmanBatchCodec(dev)
    src = torch.from_numpy(pool).to(dev)
    so = torch.from_numpy(off.view(np.int32)).to(dev)
    enc, eo = codec.encode(src, so, raw_bytes=raw)
    torch.cuda.synchronize()
    # auto slots (k_decode<true>), then the reference's floor(8E/5)+1 caller
    # slots (k_decode<false>, the first k launches of it)
    for _ in range(k):
        dst, do, st = codec.decode_auto(enc, eo)[:3]
    for _ in range(k):
        codec.decode(enc, eo)
    torch.cuda.synchronize()
    d = dst.cpu().numpy()
    dof = do.cpu().numpy().view(np.uint32)
    assert (st.cpu().numpy() >= 0).all()
    for i in range(0, n, 4099):
        assert np.array_equal(d[dof[i]:dof[i] + off[i + 1] - off[i]], pool[off[i]:off[i + 1]])
    # tight caller slots: exactly the decoded bytes, back to back
    tdst = torch.zeros(raw + 64, dtype=torch.uint8, device=dev)
    tst = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(k):
        rv = codec.L.nghttp2_amd_hd_huff_decode_batch(
            nghttp2_amd.hd._p(enc), nghttp2_amd.hd._p(eo), n, nghttp2_amd.hd._p(tdst),
            nghttp2_amd.hd._p(so), nghttp2_amd.hd._p(tst), None, None,
            nghttp2_amd.hd._stream(None))
        assert rv == 0
    torch.cuda.synchronize()
    assert (tst.cpu().numpy() >= 0).all()
    assert np.array_equal(tdst[:raw].cpu().numpy(), pool[:raw])
    print("ok: %d strings, raw %d B, enc %d B, auto pool %d B, tight pool %d B"
          % (n, raw, int(eo[-1].item()), int(dof[-1]), raw))


if __name__ == "__main__":
    main()
