"""In-process multi-device sharding: ShardedCodec cuts a
batch into byte-balanced shards, runs each on its own host thread and HIP
stream, and rebases the outputs into one batch.  On the one-GPU box the
device list repeats cuda:0 (two / three shards, threads and streams on one
GPU); the merged result must equal the oracle's result for the unsharded
batch bit for bit."""
import numpy as np
import pytest

from nghttp2_amd import workloads as W
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nshards", [2, 3])
def test_sharded_encode_equals_unsharded_oracle(dev, nshards):
    from nghttp2_amd.shard import ShardedCodec
    pool, off = W.gen_mixed_values(40000, seed=77 + nshards)
    sc = ShardedCodec([dev.index or 0] * nshards)
    enc, eoff = sc.encode(pool, off)
    ref, roff = O.encode_batch(pool, off)
    assert np.array_equal(eoff, roff.astype(np.uint64)), "merged offsets"
    assert np.array_equal(enc, ref), "merged encoded bytes"



@pytest.mark.parametrize("kind", ["mixed", "adversarial"])
def test_sharded_decode_equals_unsharded_oracle(dev, kind):
    from nghttp2_amd.shard import ShardedCodec
    if kind == "mixed":
        pool, off = W.gen_mixed_values(30000, seed=91)
        enc, eoff = O.encode_batch(pool, off)
    else:
        enc, eoff = W.gen_adversarial(20000, seed=93)[:2]
        eoff = np.asarray(eoff, dtype=np.uint32)
    sc = ShardedCodec([dev.index or 0, dev.index or 0])
    d, do, st = sc.decode_auto(enc, eoff)
    rd, rdo, rst, _, _ = O.decode_batch(enc[:int(eoff[-1])], eoff)
    assert np.array_equal(st, rst), "merged status"
    n = len(eoff) - 1
    assert len(do) == n + 1 and int(do[-1]) == len(d)
    for i in range(n):
        if st[i] > 0:
            a, b = int(do[i]), int(rdo[i])
            assert np.array_equal(d[a:a + st[i]], rd[b:b + st[i]]), "string %d" % i
    if kind == "mixed":
        assert np.array_equal(st, np.diff(off.astype(np.int64)))


def test_sharded_codec_more_shards_than_strings(dev):
    from nghttp2_amd.shard import ShardedCodec
    pool, off = W.gen_pseudo_headers(3, seed=5)
    sc = ShardedCodec([dev.index or 0] * 4)  # some shards are empty
    enc, eoff = sc.encode(pool, off)
    ref, roff = O.encode_batch(pool, off)
    assert np.array_equal(enc, ref) and np.array_equal(eoff, roff.astype(np.uint64))
