#!/usr/bin/env python3
"""emit_strings_batch probe: small batches of chosen shapes against the
oracle; prints each failing case with the first differing literal."""
import itertools, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import nghttp2_amd
from oracle import oracle as O

dev = torch.device("cuda:0")
codec = nghttp2_amd.HuffmanBatchCodec(dev)
rng = np.random.Generator(np.random.PCG64(7))


def run(strs, tag):
    off = np.zeros(len(strs) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(s) for s in strs])
    pool = np.frombuffer(b"".join(strs) + b"\0" * 32, dtype=np.uint8).copy()
    src = torch.from_numpy(pool).to(dev)
    so = torch.from_numpy(off.view(np.int32)).to(dev)
    d, do = codec.emit_strings(src, so, raw_bytes=int(off[-1]))
    torch.cuda.synchronize()
    do = do.cpu().numpy().view(np.uint32)
    d = d.cpu().numpy()[:int(do[-1])]
    rd, rdo = O.emit_strings_batch(pool[:int(off[-1])], off)
    if not np.array_equal(do, rdo):
        i = int(np.nonzero(do != rdo)[0][0])
        print("FAIL %s: offsets differ at %d (%d vs %d)" % (tag, i, do[i], rdo[i]))
        return False
    if not np.array_equal(d, rd):
        i = int(np.nonzero(d != rd)[0][0])
        s = int(np.searchsorted(do, i, side="right") - 1)
        lit = bytes(rd[rdo[s]:rdo[s + 1]])
        print("FAIL %s: byte %d (string %d of %d, R=%d, literal %d bytes, pos %d in it, first %02x): "
              "got %s want %s" % (tag, i, s, len(strs), len(strs[s]), len(lit), i - int(rdo[s]),
                                  lit[0], bytes(d[i:i + 6]).hex(), bytes(rd[i:i + 6]).hex()))
        return False
    return True


def text(k):
    return bytes(rng.choice(np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-/=", np.uint8), k))


def raw(k):
    return bytes(rng.integers(128, 256, size=k, dtype=np.uint8))


L = [0, 1, 2, 3, 5, 10, 16, 17, 50, 126, 127, 128, 200, 300]
bad = 0
for k in L:
    bad += not run([text(k)], "text%d" % k)
    bad += not run([raw(k)], "raw%d" % k)
for k1, k2 in itertools.product([0, 1, 5, 20, 130], repeat=2):
    for f1, f2 in itertools.product([text, raw], repeat=2):
        bad += not run([f1(k1), f2(k2)], "%s%d+%s%d" % (f1.__name__, k1, f2.__name__, k2))
for trip in [[b"", b"", text(5)], [text(5), b"", b""], [text(5), b"", text(7)], [raw(3), b"", raw(4)],
             [b"", raw(5), b""], [text(150), b"", text(3)]]:
    bad += not run(trip, "trip%s" % [len(x) for x in trip])
for seed in range(40):
    r = np.random.Generator(np.random.PCG64(seed))
    n = int(r.integers(1, 300))
    strs = []
    for _ in range(n):
        c = int(r.integers(0, 4))
        k = int(r.integers(0, 200))
        strs.append(b"" if c == 0 else text(k) if c < 3 else raw(k))
    if not run(strs, "rand%d" % seed):
        bad += 1
        if bad > 12:
            break
print("bad", bad)
