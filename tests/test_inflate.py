"""Batched HPACK inflate front-end (nghttp2_amd_hd_inflate_blocks, SURVEY.md
8(f) row 2) against RFC 7541 Appendix C and the pure-Python restatement of
nghttp2's inflater (oracle/hpack_oracle.py).

Blocks without Huffman literals make no GPU call, so the RFC C.3 / C.5
sequences and the error cases run on the CPU; everything with Huffman
literals is marked gpu."""
import json
import os

import numpy as np
import pytest

from oracle import hpack_oracle as HO
from oracle import oracle as O

KA = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
EXAMPLES = KA["rfc7541_header_blocks"]["examples"]
SIZE_256 = bytes.fromhex("3fe101")  # table size update to 256 (RFC 7541 6.3)


def _setup(ex, n=None):
    import nghttp2_amd
    inf = nghttp2_amd.HpackInflater()
    ref = HO.Inflater()
    blocks = [bytes.fromhex(b["wire"]) for b in ex["blocks"]]
    if ex["table_size"] != 4096:
        inf.change_table_size(ex["table_size"])
        ref.change_table_size(ex["table_size"])
        blocks[0] = SIZE_256 + blocks[0]
    return inf, ref, blocks


def _check_example(ex, per_block):
    import nghttp2_amd
    inf, ref, blocks = _setup(ex)
    if per_block:
        res = [nghttp2_amd.inflate_blocks([inf], [b]) for b in blocks]
        status = [r[0][0] for r in res]
        fields = [r[1][0] for r in res]
        tables = None
    else:
        status, fields = nghttp2_amd.inflate_blocks([inf] * len(blocks), blocks)
        tables = None
    for k, b in enumerate(ex["blocks"]):
        want = [(n.encode(), v.encode(), 0) for n, v in b["headers"]]
        assert status[k] == len(want), (ex["section"], k)
        assert fields[k] == want, (ex["section"], k)
        rs, rf = ref.inflate_block(blocks[k])
        assert (rs, rf) == (status[k], fields[k])
    want_tab = [(n.encode(), v.encode()) for n, v in ex["blocks"][-1]["table"]]
    assert inf.dynamic_table() == want_tab
    assert inf.dynamic_table_size() == ex["blocks"][-1]["table_bytes"]
    return tables


@pytest.mark.parametrize("ex", [e for e in EXAMPLES if not e["huffman"]],
                         ids=lambda e: e["section"])
def test_rfc7541_plain_blocks_cpu(ex):
    _check_example(ex, per_block=True)
    _check_example(ex, per_block=False)


@pytest.mark.parametrize("ex", EXAMPLES, ids=lambda e: e["section"])
def test_rfc7541_oracle_tables(ex):
    """The restatement reproduces every intermediate table of Appendix C."""
    _, ref, blocks = _setup(ex)
    for b, want in zip(blocks, ex["blocks"]):
        st, f = ref.inflate_block(b)
        assert st == len(want["headers"])
        assert [(n.decode(), v.decode()) for n, v in ref.table] == [tuple(x) for x in want["table"]]
        assert ref.size == want["table_bytes"]


def test_rfc7541_wire_matches_components():
    """The Huffman examples' literals are emit_string of their strings and the
    plain examples' literals the raw strings (C.4 vs C.3, C.6 vs C.5)."""
    by = {e["section"]: e for e in EXAMPLES}
    for plain, huff in (("RFC 7541 C.3", "RFC 7541 C.4"), ("RFC 7541 C.5", "RFC 7541 C.6")):
        for bp, bh in zip(by[plain]["blocks"], by[huff]["blocks"]):
            assert bp["headers"] == bh["headers"]
            # every Huffman literal of the C.4/C.6 wire is the framed literal of a header string
            wire = bytes.fromhex(bh["wire"])
            for n, v in bh["headers"]:
                for s in (n, v):
                    lit = O.emit_string(s.encode())
                    if lit[0] & 0x80 and lit in wire:
                        break


def _cpu_error_cases():
    return [
        bytes.fromhex("80"),                    # index 0
        bytes.fromhex("be"),                    # index 62: empty dynamic table
        bytes.fromhex("8286" + "3f00"),         # size update after a field
        bytes.fromhex("3fe21f"),                # size update above the 4096 setting
        bytes.fromhex("400a637573746f6d2d6b6579"),  # truncated: no value
        bytes.fromhex("0f"),                    # truncated index
        bytes.fromhex("00ff8080808080808001"),  # name length overflow
        bytes.fromhex("007f81ff03") + b"x" * 10,  # name length > NGHTTP2_HD_MAX_NV
        bytes.fromhex("828684"),                # fine
    ]


def test_inflate_errors_cpu():
    import nghttp2_amd
    for blk in _cpu_error_cases():
        inf, ref = nghttp2_amd.HpackInflater(), HO.Inflater()
        st, f = nghttp2_amd.inflate_blocks([inf], [blk])
        rs, rf = ref.inflate_block(blk)
        assert (st[0], f[0]) == (rs, rf), blk.hex()
        # sticky: the next block of a failed inflater fails too
        st2, f2 = nghttp2_amd.inflate_blocks([inf], [bytes.fromhex("82")])
        assert (st2[0], f2[0]) == ref.inflate_block(bytes.fromhex("82"))


def test_expected_table_size_update_cpu():
    import nghttp2_amd
    for blk in (bytes.fromhex("82"), b"", bytes.fromhex("3f6182"), bytes.fromhex("3fe20f82"),
                bytes.fromhex("20" + "3f61" + "82")):
        inf, ref = nghttp2_amd.HpackInflater(), HO.Inflater()
        inf.change_table_size(128)
        ref.change_table_size(128)
        st, f = nghttp2_amd.inflate_blocks([inf], [blk])
        assert (st[0], f[0]) == ref.inflate_block(blk), blk.hex()


# ---- random batches (GPU: Huffman literals) ----
def _encode_block(rng, table, fields, table_max, huff_p=0.7):
    """A small HPACK encoder for test blocks: random representation and
    Huffman choices.  `table` mirrors the decoder's dynamic table."""
    out = bytearray()

    def integer(v, prefix, first):
        out.extend(O.encode_length(v, prefix, first))

    def string(s):
        if rng.random() < huff_p:
            out.extend(O.emit_string(s))
        else:  # raw even when Huffman would be shorter
            integer(len(s), 7, 0)
            out.extend(s)

    size = sum(len(n) + len(v) + 32 for n, v in table)

    def add(n, v):
        nonlocal size
        room = len(n) + len(v) + 32
        while size + room > table_max and table:
            a, b = table.pop()
            size -= len(a) + len(b) + 32
        if room <= table_max:
            table.insert(0, (n, v))
            size += room

    for n, v in fields:
        allnv = HO.STATIC + table
        exact = [i for i, e in enumerate(allnv) if e == (n, v)]
        named = [i for i, e in enumerate(allnv) if e[0] == n]
        r = rng.random()
        if exact and r < 0.4:
            integer(exact[0] + 1, 7, 0x80)
            continue
        mode = rng.integers(0, 3)  # 0: incremental, 1: without, 2: never
        first, prefix = ((0x40, 6), (0x00, 4), (0x10, 4))[mode]
        if named and rng.random() < 0.5:
            integer(named[0] + 1, prefix, first)
        else:
            out.append(first)
            string(n)
        string(v)
        if mode == 0:
            add(n, v)
    return bytes(out)


def _random_fields(rng, k):
    from nghttp2_amd import workloads as W
    pool, off = W.gen_mixed_values(k, seed=int(rng.integers(1 << 30)), hi=200)
    names = [b":method", b":path", b":authority", b"cookie", b"user-agent", b"x-trace",
             b"accept", b"set-cookie", b"content-type", b"x-" + bytes(rng.integers(97, 123, 5))]
    out = []
    for i in range(k):
        v = bytes(pool[off[i]:off[i + 1]])
        if rng.random() < 0.3:
            v = v[:rng.integers(0, 8)]
        out.append((names[rng.integers(0, len(names))], v))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("ex", [e for e in EXAMPLES if e["huffman"]], ids=lambda e: e["section"])
def test_rfc7541_huffman_blocks(ex):
    _check_example(ex, per_block=True)
    _check_example(ex, per_block=False)


@pytest.mark.gpu
def test_inflate_random_connections_vs_oracle():
    import nghttp2_amd
    rng = np.random.Generator(np.random.PCG64(0x1F1A7E))
    nconn, nblk = 12, 6
    infs = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
    refs = [HO.Inflater() for _ in range(nconn)]
    enc_tables = [[] for _ in range(nconn)]
    order, blocks = [], []
    for r in range(nblk):
        for c in rng.permutation(nconn):
            fields = _random_fields(rng, int(rng.integers(1, 12)))
            blk = _encode_block(rng, enc_tables[c], fields, 4096)
            if rng.random() < 0.1:  # corruption: truncate, or flip a byte
                blk = blk[:max(1, len(blk) - int(rng.integers(1, 4)))] if rng.random() < 0.5 \
                    else blk[:-1] + bytes([blk[-1] ^ 0xFF])
            order.append(int(c))
            blocks.append(blk)
    st, f = nghttp2_amd.inflate_blocks([infs[c] for c in order], blocks)
    for k, (c, blk) in enumerate(zip(order, blocks)):
        rs, rf = refs[c].inflate_block(blk)
        assert (st[k], f[k]) == (rs, rf), (k, c)
    for c in range(nconn):
        assert infs[c].dynamic_table() == [tuple(e) for e in refs[c].table]


# ---- many connections without Huffman literals (no GPU call): the threaded
# replay, and the buffer cut with its table rollback ----
def _plain_batch(seed, nconn, nblk):
    rng = np.random.Generator(np.random.PCG64(seed))
    enc_tables = [[] for _ in range(nconn)]
    order, blocks = [], []
    for _ in range(nblk):
        for c in rng.permutation(nconn):
            fields = _random_fields(rng, int(rng.integers(1, 10)))
            blk = _encode_block(rng, enc_tables[c], fields, 4096, huff_p=0.0)
            if rng.random() < 0.05:
                blk = blk[:max(1, len(blk) - int(rng.integers(1, 4)))]
            order.append(int(c))
            blocks.append(blk)
    return order, blocks


def test_inflate_many_connections_plain_cpu():
    import nghttp2_amd
    nconn = 300
    order, blocks = _plain_batch(0xC0FFEE, nconn, 4)
    infs = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
    refs = [HO.Inflater() for _ in range(nconn)]
    st, f = nghttp2_amd.inflate_blocks([infs[c] for c in order], blocks)
    for k, (c, blk) in enumerate(zip(order, blocks)):
        assert (st[k], f[k]) == refs[c].inflate_block(blk), (k, c)
    for c in range(nconn):
        assert infs[c].dynamic_table() == [tuple(e) for e in refs[c].table]


@pytest.mark.parametrize("nconn,per,cap", [(40, 5, 6000), (1, 60, 800)])
def test_inflate_buffer_cut_rolls_back_cpu(nconn, per, cap):
    """Buffers too small for the batch: the blocks before the cut are applied,
    the rest are not (tables as if they never came), and resubmitting them
    gives the oracle's result.  One connection takes the direct replay into
    the caller's buffers (csrc/hd_inflate.cpp DirectSink), whose blocks near
    the caps go through a table copy and a scratch buffer."""
    import nghttp2_amd
    from nghttp2_amd import hd
    order, blocks = _plain_batch(0xB0F, nconn, per)
    infs = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
    refs = [HO.Inflater() for _ in range(nconn)]
    st, f = nghttp2_amd.inflate_blocks([infs[c] for c in order], blocks, arena_cap=cap, retry=False)
    cut = st.index(hd.NGHTTP2_ERR_BUFFER_ERROR)
    assert 0 < cut < len(blocks)
    assert all(s == hd.NGHTTP2_ERR_BUFFER_ERROR for s in st[cut:])
    for k in range(cut):
        assert (st[k], f[k]) == refs[order[k]].inflate_block(blocks[k]), k
    for c in range(nconn):
        assert infs[c].dynamic_table() == [tuple(e) for e in refs[c].table], c
    st2, f2 = nghttp2_amd.inflate_blocks([infs[c] for c in order[cut:]], blocks[cut:],
                                         arena_cap=cap)
    for k in range(cut, len(blocks)):
        assert (st2[k - cut], f2[k - cut]) == refs[order[k]].inflate_block(blocks[k]), k


@pytest.mark.parametrize("nconn,per,cap", [(40, 5, 6000), (1, 60, 800), (1, 60, 100000)])
def test_inflate_cut_with_huge_table_limit_cpu(nconn, per, cap):
    """As above with the SETTINGS table limit at 2^32 - 1 (the reference's
    change_table_size case): a dynamic reference's output is bounded by the
    longest entry and literal, not by the limit (csrc/hd_inflate.cpp
    dyn_ref_bound), so one connection's blocks take the direct replay; the
    results and the cut are the oracle's either way."""
    import nghttp2_amd
    from nghttp2_amd import hd
    order, blocks = _plain_batch(0xB1F, nconn, per)
    infs = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
    refs = [HO.Inflater() for _ in range(nconn)]
    for i, r in zip(infs, refs):
        i.change_table_size(2**32 - 1)
        r.change_table_size(2**32 - 1)
    st, f = nghttp2_amd.inflate_blocks([infs[c] for c in order], blocks, arena_cap=cap, retry=False)
    cut = st.index(hd.NGHTTP2_ERR_BUFFER_ERROR) if hd.NGHTTP2_ERR_BUFFER_ERROR in st else len(blocks)
    assert all(s == hd.NGHTTP2_ERR_BUFFER_ERROR for s in st[cut:])
    for k in range(cut):
        assert (st[k], f[k]) == refs[order[k]].inflate_block(blocks[k]), k
    for c in range(nconn):
        assert infs[c].dynamic_table() == [tuple(e) for e in refs[c].table], c
    if cut < len(blocks):
        st2, f2 = nghttp2_amd.inflate_blocks([infs[c] for c in order[cut:]], blocks[cut:],
                                             arena_cap=cap)
        for k in range(cut, len(blocks)):
            assert (st2[k - cut], f2[k - cut]) == refs[order[k]].inflate_block(blocks[k]), k


# ---- the dynamic table's byte ring (csrc/hd_inflate.cpp DynTable): long
# runs that wrap it many times, size updates that shrink and regrow it, and
# an insertion whose name comes from the entry it evicts ----
def test_inflate_table_ring_wraps_and_resizes_cpu():
    import nghttp2_amd
    rng = np.random.Generator(np.random.PCG64(0x5EED1))
    nconn = 3
    infs = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
    refs = [HO.Inflater() for _ in range(nconn)]
    enc_tables = [[] for _ in range(nconn)]
    table_max = [4096] * nconn
    for rnd in range(60):
        order, blocks = [], []
        for c in rng.permutation(nconn):
            pre = b""
            if rng.random() < 0.25:  # a table size update at the block head
                table_max[c] = int(rng.choice([0, 50, 300, 1000, 2500, 4096]))
                pre = bytes(O.encode_length(table_max[c], 5, 0x20))
                t, size = enc_tables[c], sum(len(a) + len(b) + 32 for a, b in enc_tables[c])
                while size > table_max[c] and t:
                    a, b = t.pop()
                    size -= len(a) + len(b) + 32
            fields = _random_fields(rng, int(rng.integers(1, 14)))
            blocks.append(pre + _encode_block(rng, enc_tables[c], fields, table_max[c], huff_p=0.0))
            order.append(int(c))
        st, f = nghttp2_amd.inflate_blocks([infs[c] for c in order], blocks)
        for k, (c, blk) in enumerate(zip(order, blocks)):
            assert (st[k], f[k]) == refs[c].inflate_block(blk), (rnd, k, c)
    for c in range(nconn):
        assert infs[c].dynamic_table() == [tuple(e) for e in refs[c].table], c
        assert infs[c].dynamic_table_size() == sum(len(a) + len(b) + 32 for a, b in refs[c].table)


def test_inflate_name_from_evicted_entry_cpu():
    """Literal with incremental indexing whose indexed name is the entry its
    own insertion evicts (lib/nghttp2_hd.c add_hd_table_incremental copies
    the name first)."""
    import nghttp2_amd
    inf, ref = nghttp2_amd.HpackInflater(), HO.Inflater()
    blk = bytes(O.encode_length(100, 5, 0x20))  # table of 100 bytes
    blk += b"\x40" + bytes(O.encode_length(4, 7, 0)) + b"aaaa" + bytes(O.encode_length(40, 7, 0)) + b"v" * 40
    blk += bytes(O.encode_length(62, 6, 0x40)) + bytes(O.encode_length(41, 7, 0)) + b"w" * 41
    blk += bytes(O.encode_length(62, 6, 0x40)) + bytes(O.encode_length(0, 7, 0))
    st, f = nghttp2_amd.inflate_blocks([inf], [blk])
    assert (st[0], f[0]) == ref.inflate_block(blk)
    assert inf.dynamic_table() == [(b"aaaa", b"")] == [tuple(e) for e in ref.table]
