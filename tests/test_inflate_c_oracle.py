"""The C inflater of the oracle (oracle/hpack_inflate_oracle.c, the inflate
front-end's CPU baseline) against the Python Inflater: every status, field
and final table on the RFC 7541 examples, the reference's own inflate cases
(tests/golden/ref_hd_tests.json) and random batches with Huffman literals,
corruptions and table size updates (CPU only)."""
import json
import os

import numpy as np
import pytest

from oracle import hpack_oracle as HO
from tests.test_inflate import EXAMPLES, _encode_block, _random_fields

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _same(blocks, nconn=1, conns=None, sizes=None, settings=()):
    conns = conns or [0] * len(blocks)
    py = [HO.Inflater() for _ in range(nconn)]
    c = [HO.CInflater() for _ in range(nconn)]
    for v in settings:
        for x in py + c:
            x.change_table_size(v)
    for k, (ci, b) in enumerate(zip(conns, blocks)):
        if sizes and sizes[k] is not None:
            py[ci].change_table_size(sizes[k])
            c[ci].change_table_size(sizes[k])
        assert c[ci].inflate_block(b) == py[ci].inflate_block(b), k
    for ci in range(nconn):
        assert c[ci].table == py[ci].table
        assert c[ci].table_size() == sum(len(a) + len(b) + 32 for a, b in py[ci].table)


@pytest.mark.parametrize("ex", EXAMPLES, ids=lambda e: e["section"])
def test_c_inflater_rfc7541(ex):
    blocks = [bytes.fromhex(b["wire"]) for b in ex["blocks"]]
    settings = ()
    if ex["table_size"] != 4096:
        settings = (ex["table_size"],)
        blocks[0] = bytes.fromhex("3fe101") + blocks[0]  # table size update to 256
    _same(blocks, settings=settings)


def test_c_inflater_random_connections():
    rng = np.random.Generator(np.random.PCG64(0xC1F))
    nconn, order, blocks, sizes = 7, [], [], []
    tables = [[] for _ in range(nconn)]
    tmax = [4096] * nconn
    for _ in range(40):
        for c in rng.permutation(nconn):
            size = None
            pre = b""
            if rng.random() < 0.15:
                tmax[c] = int(rng.choice([0, 64, 300, 1500, 4096]))
                pre = bytes(HO.O.encode_length(tmax[c], 5, 0x20))
                t, sz = tables[c], sum(len(a) + len(b) + 32 for a, b in tables[c])
                while sz > tmax[c] and t:
                    a, b = t.pop()
                    sz -= len(a) + len(b) + 32
            blk = pre + _encode_block(rng, tables[c], _random_fields(rng, int(rng.integers(1, 10))),
                                      tmax[c], huff_p=0.6)
            if rng.random() < 0.06:  # corruption: truncate or flip the last byte
                blk = blk[:max(1, len(blk) - 2)] if rng.random() < 0.5 else blk[:-1] + bytes([blk[-1] ^ 0xA5])
            order.append(int(c))
            blocks.append(blk)
            sizes.append(size)
    _same(blocks, nconn, order, sizes)


def test_c_inflater_reference_cases():
    """tests/nghttp2_hd_test.c's inflate cases, extracted as data."""
    cases = json.load(open(os.path.join(GOLDEN, "ref_hd_tests.json")))["inflate_cases"]
    assert cases
    for case in cases:
        _same([bytes.fromhex(case["block"])], settings=case["settings"])


def test_c_inflater_batch_timed_counts_fields():
    rng = np.random.Generator(np.random.PCG64(5))
    tables = [[] for _ in range(3)]
    blocks, conns = [], []
    for _ in range(10):
        for c in range(3):
            blocks.append(_encode_block(rng, tables[c], _random_fields(rng, 5), 4096, huff_p=0.5))
            conns.append(c)
    ref = [HO.Inflater() for _ in range(3)]
    want = sum(max(0, ref[c].inflate_block(b)[0]) for c, b in zip(conns, blocks))
    for t in (1, 2):
        dt, nf = HO.c_inflate_batch_timed(blocks, conns, 3, t)
        assert nf == want and dt >= 0
