"""The inflate front-end's host logic (nghttp2_amd_hd_inflate_blocks: pass-1
parse, connection grouping, the output bound and the cut-and-replay when a
batch outgrows the caller's buffers, pass-2 replay against each connection's
dynamic table) on blocks whose literals are all raw: such a batch has no
Huffman literal, so no GPU call is made and it runs here.  Checked against
the oracle's inflater (lib/nghttp2_hd.c:1919-2288 restated), block by block,
connection by connection."""
import random

import pytest

import nghttp2_amd
from oracle import hpack_oracle as HO


def _int(v, prefix, first):
    k = (1 << prefix) - 1
    if v < k:
        return bytes([first | v])
    out = [first | k]
    v -= k
    while v >= 128:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _lit(s):
    return _int(len(s), 7, 0) + s


def _block(rng, ndyn):
    """Indexed static and dynamic references, literals with incremental
    indexing (new and indexed names), literals without indexing, size updates
    at the block start; raw strings only."""
    b = b""
    if rng.random() < 0.1:
        b += _int(rng.choice([0, 100, 4096]), 5, 0x20)
        ndyn[0] = 0 if b[-1] == 0x20 else ndyn[0]
    for _ in range(rng.randint(0, 12)):
        r = rng.random()
        if r < 0.25:
            b += _int(rng.randint(1, 61), 7, 0x80)
        elif r < 0.4 and ndyn[0]:
            b += _int(62 + rng.randint(0, ndyn[0] - 1), 7, 0x80)
        elif r < 0.7:
            b += b"\x40" + _lit(bytes(rng.choice(b"abcdef") for _ in range(rng.randint(1, 30)))) + \
                _lit(bytes(rng.randint(32, 126) for _ in range(rng.randint(0, 200))))
            ndyn[0] = min(ndyn[0] + 1, 8)
        elif r < 0.85:
            b += _int(rng.randint(1, 61), 6, 0x40) + _lit(bytes(rng.randint(32, 126) for _ in range(rng.randint(0, 90))))
            ndyn[0] = min(ndyn[0] + 1, 8)
        else:
            b += _int(rng.randint(1, 61), 4, 0x00) + _lit(b"x" * rng.randint(0, 50))
    return b


@pytest.mark.parametrize("cap", [None, 5, 20, 60])
def test_raw_literal_batches_match_oracle(cap):
    rng = random.Random(1234 + (cap or 0))
    for _ in range(12):
        nconn = rng.randint(1, 9)
        infs = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
        refs = [HO.Inflater() for _ in range(nconn)]
        ndyn = [[0] for _ in range(nconn)]
        conns = [rng.randrange(nconn) for _ in range(rng.randint(1, 40))]
        blocks = [_block(rng, ndyn[c]) for c in conns]
        kw = {} if cap is None else {"nva_cap": cap, "arena_cap": cap * 40}
        st, f = nghttp2_amd.inflate_blocks([infs[c] for c in conns], blocks, **kw)
        for k, (c, b) in enumerate(zip(conns, blocks)):
            assert (st[k], f[k]) == refs[c].inflate_block(b), (k, c)
        for c in range(nconn):
            assert infs[c].dynamic_table_size() == refs[c].size
            assert [tuple(map(bytes, e)) for e in infs[c].dynamic_table()] == \
                [tuple(map(bytes, e)) for e in refs[c].table]


def test_same_inflater_twice_in_separate_batches():
    """The grouping stamp: an inflater's connection number from one call must
    not leak into the next (different batch, different connection order)."""
    rng = random.Random(7)
    infs = [nghttp2_amd.HpackInflater() for _ in range(3)]
    refs = [HO.Inflater() for _ in range(3)]
    ndyn = [[0] for _ in range(3)]
    for order in ([0, 1, 2, 0], [2, 2, 1], [1, 0, 2, 1, 0]):
        blocks = [_block(rng, ndyn[c]) for c in order]
        st, f = nghttp2_amd.inflate_blocks([infs[c] for c in order], blocks)
        for k, (c, b) in enumerate(zip(order, blocks)):
            assert (st[k], f[k]) == refs[c].inflate_block(b)
