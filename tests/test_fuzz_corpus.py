"""The reference's fuzz corpus through the batched inflate front-end.

`tests/golden/fuzz_corpus_blocks.json` holds the HPACK header blocks of the
136 HTTP/2 client connections in the reference's `fuzz/corpus/{h2spec,nghttp}`
(the inputs `fuzz/fuzz_target.cc` feeds a server session, whose inflater
decodes each block in order), extracted by frame parsing only
(`tests/golden/make_fuzz_corpus_blocks.py`).  The corpus holds no expected
outputs, so parity here is against the oracle (`oracle/hpack_oracle.py`, the
restatement of `lib/nghttp2_hd.c`'s inflater, pinned by RFC 7541 Appendix C and
the reference's own hd tests): per block the status (field count or the
reference's error), the fields with their flags, and each connection's
dynamic table after its last block, malformed blocks and sticky failures
included."""
import json
import os

import pytest

from oracle import hpack_oracle as HO

CORPUS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "fuzz_corpus_blocks.json")))
CONNS = CORPUS["connections"]


def _oracle(conn):
    ref = HO.Inflater()
    res = [ref.inflate_block(bytes.fromhex(b)) for b in conn["blocks"]]
    return res, [tuple(e) for e in ref.table]


def test_fuzz_corpus_fixture_cpu():
    """The fixture covers the whole corpus, and the oracle both accepts and
    rejects blocks of it (so the GPU test below sees errors as well)."""
    assert len(CONNS) == 136
    assert sorted({c["corpus"] for c in CONNS}) == ["h2spec", "nghttp"]
    nblk = sum(len(c["blocks"]) for c in CONNS)
    assert nblk == 301
    ok = bad = 0
    for c in CONNS:
        res, _ = _oracle(c)
        ok += sum(1 for s, _ in res if s >= 0)
        bad += sum(1 for s, _ in res if s < 0)
    assert ok > 250 and bad > 0


def _interleaved():
    """Every connection's blocks, round-robin across connections (block k of
    each connection before block k + 1 of any), as one batch."""
    order, blocks = [], []
    depth = max(len(c["blocks"]) for c in CONNS)
    for k in range(depth):
        for ci, c in enumerate(CONNS):
            if k < len(c["blocks"]):
                order.append(ci)
                blocks.append(bytes.fromhex(c["blocks"][k]))
    return order, blocks


@pytest.mark.gpu
def test_fuzz_corpus_one_batch_vs_oracle():
    """All 136 connections in one inflate_blocks call."""
    import nghttp2_amd
    infs = [nghttp2_amd.HpackInflater() for _ in CONNS]
    order, blocks = _interleaved()
    st, f = nghttp2_amd.inflate_blocks([infs[c] for c in order], blocks)
    want = [_oracle(c) for c in CONNS]
    seen = [0] * len(CONNS)
    for k, c in enumerate(order):
        rs, rf = want[c][0][seen[c]]
        assert (st[k], f[k]) == (rs, rf), (CONNS[c]["file"], seen[c])
        seen[c] += 1
    for c, inf in enumerate(infs):
        assert inf.dynamic_table() == want[c][1], CONNS[c]["file"]


@pytest.mark.gpu
def test_fuzz_corpus_per_connection_vs_oracle():
    """Each connection alone, one call per block (the single-connection path)."""
    import nghttp2_amd
    for c in CONNS:
        inf = nghttp2_amd.HpackInflater()
        res, table = _oracle(c)
        for k, b in enumerate(c["blocks"]):
            st, f = nghttp2_amd.inflate_blocks([inf], [bytes.fromhex(b)])
            assert (st[0], f[0]) == res[k], (c["file"], k)
        assert inf.dynamic_table() == table, c["file"]
