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


@pytest.mark.timeout(900)
def test_sharded_8way_config4_full_16m(dev):
    """The C ABI's sharded engine cut 8 ways (8 worker threads and streams,
    all on device 0) over the whole config-4 set, 16,777,216 strings of the
    config-4 generator (2.5 GB raw): merged encode equal to the oracle's
    encode of the unsharded set, byte for byte; merged decode with status ==
    length and every decoded byte equal to the input."""
    from nghttp2_amd.shard import ShardedCodec
    n = 1 << 24
    lengths = W.mixed_lengths(n)
    pool, off = W.gen_mixed_range(lengths, 0, n, threads=16)
    raw = int(off[-1])
    print("generated %d strings, %d bytes" % (n, raw), flush=True)
    sc = ShardedCodec([dev.index or 0] * 8)
    enc, eoff = sc.encode(pool, off)
    print("sharded encode done", flush=True)
    ref, roff = O.encode_batch(pool, off, nthreads=16)
    assert np.array_equal(eoff, roff.astype(np.uint64)), "merged offsets"
    assert np.array_equal(enc, ref[:int(roff[-1])]), "merged encoded bytes"
    del ref
    d, do, st = sc.decode_auto(enc, roff)
    print("sharded decode done", flush=True)
    assert np.array_equal(st, lengths.astype(np.int32)), "merged status"
    assert int(do[-1]) == len(d) >= raw  # (dense per task; tasks start at their bound)
    do = do.astype(np.int64)
    for a in range(0, n, 1 << 20):
        b = min(n, a + (1 << 20))
        lc = lengths[a:b]
        rel = np.arange(int(lc.sum())) - np.repeat(np.cumsum(lc) - lc, lc)
        got = d[np.repeat(do[a:b], lc) + rel]
        want = pool[np.repeat(off[a:b].astype(np.int64), lc) + rel]
        assert np.array_equal(got, want), "decoded bytes of strings [%d, %d)" % (a, b)
