#!/usr/bin/env python3
"""Generate the committed golden vectors tests/golden/*.npz.

Inputs come from the deterministic generators in nghttp2_amd/workloads.py
(small-N samples of the BASELINE.json config distributions, every byte value,
the decode-only adversarial mix, and edge cases); expected outputs come from
the oracle (oracle/huff_oracle.c), which tests/test_oracle.py pins to the
reference (table sha256 from mkhufftbl.py + the reference's Huffman
unit-test vectors).  Files are plain .npz (no pickles).

Usage: python3 tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

CASES = ["pseudo_1k", "mixed_200", "allbytes_1k", "adversarial_3k", "edge"]


def decoded_bytes(dst, doff, status):
    """The whole (zero-initialised) slot pool: written bytes + untouched."""
    return np.ascontiguousarray(dst[:int(doff[-1])]).tobytes()


def _edge():
    from nghttp2_amd import workloads as W
    rng = np.random.Generator(np.random.PCG64(0xED6E))
    strs = [b"", b"", b"a", b"", bytes([0]), bytes([255]), bytes([10]), bytes([13]),
            bytes([22]), bytes(range(256)), bytes(range(255, -1, -1))]
    strs += [bytes([b]) for b in range(256)]
    strs += [bytes(rng.integers(0, 256, size=65536, dtype=np.uint8))]   # NGHTTP2_HD_MAX_NV
    strs += [b"\xff" * 4096, b"0" * 4097, b""]
    lens = np.array([len(s) for s in strs], dtype=np.int64)
    return W._pool_from_lengths(lens, np.frombuffer(b"".join(strs), dtype=np.uint8))


def inputs(name):
    from nghttp2_amd import workloads as W
    if name == "pseudo_1k":
        return "roundtrip", W.gen_pseudo_headers(1000, seed=W.SEED[2] + 1)
    if name == "mixed_200":
        return "roundtrip", W.gen_mixed_values(200, seed=W.SEED[3] + 1)
    if name == "allbytes_1k":
        return "roundtrip", W.gen_all_bytes(1000, seed=0xA11)
    if name == "adversarial_3k":
        pool, off, _ = W.gen_adversarial(3000, seed=W.SEED[5] + 1)
        return "decode", (pool, off)
    if name == "edge":
        return "roundtrip", _edge()
    raise KeyError(name)


def make(name):
    from oracle import oracle as O
    kind, (pool, off) = inputs(name)
    rec = {"kind": np.array(kind)}
    if kind == "roundtrip":
        enc, eoff = O.encode_batch(pool, off)
        rec.update(raw=pool[:int(off[-1])], raw_off=off, enc=enc, enc_off=eoff)
        src, soff = enc, eoff
    else:
        rec.update(enc=pool[:int(off[-1])], enc_off=off)
        src, soff = pool, off
    dst, doff, st, fs, fl = O.decode_batch(src, soff)
    rec.update(status=st, fstate=fs, flags=fl,
               dec_sha256=np.array(hashlib.sha256(decoded_bytes(dst, doff, st)).hexdigest()))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **rec)


def load(name):
    with np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    g["kind"] = str(g["kind"])
    g["dec_sha256"] = str(g["dec_sha256"])
    return g


if __name__ == "__main__":
    for c in CASES:
        make(c)
        print("wrote", c)
