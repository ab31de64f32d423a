"""Batched HPACK deflate front-end (nghttp2_amd_hd_deflate_blocks, SURVEY.md
8(f)) against nghttp2's own deflater output for RFC 7541 C.4 (the reference's
deflater emits exactly the RFC's Huffman request sequence), the pure-Python
restatement of nghttp2_hd_deflate_hd2 (oracle/hpack_oracle.py Deflater), and
deflate -> inflate round trips through the batched inflater.

Every literal is framed on the GPU (one emit_strings batch per call), so a
block with a literal is a GPU test; fully indexed blocks run on the CPU."""
import json
import os

import numpy as np
import pytest

from oracle import hpack_oracle as HO

KA = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
EXAMPLES = {e["section"]: e for e in KA["rfc7541_header_blocks"]["examples"]}


def _lists(ex):
    return [[(n.encode(), v.encode()) for n, v in b["headers"]] for b in ex["blocks"]]


def test_oracle_deflater_rfc7541_c4():
    """The restatement reproduces the RFC's Huffman request sequence and its
    tables (nghttp2's deflater produces exactly this wire)."""
    ex = EXAMPLES["RFC 7541 C.4"]
    d = HO.Deflater()
    for hl, b in zip(_lists(ex), ex["blocks"]):
        assert d.deflate_block(hl).hex() == b["wire"]
        assert [(n.decode(), v.decode()) for n, v in d.table] == [tuple(x) for x in b["table"]]


def test_oracle_deflater_rfc7541_c6():
    """C.6 (responses, 256-byte table): after the 256 table-size setting the
    deflater sends the 6.3 size update first.  nghttp2 never indexes
    location/set-cookie (the RFC does), so the wire is checked by decoding
    it with the restated inflater instead of byte equality."""
    ex = EXAMPLES["RFC 7541 C.6"]
    d, inf = HO.Deflater(), HO.Inflater()
    d.change_table_size(256)
    inf.change_table_size(256)
    for k, hl in enumerate(_lists(ex)):
        w = d.deflate_block(hl)
        if k == 0:
            assert w.startswith(bytes.fromhex("3fe101"))
        st, f = inf.inflate_block(w)
        assert [(n, v) for n, v, _ in f] == hl
        assert inf.table == d.table


def test_indexed_only_blocks_cpu():
    """Blocks whose fields all hit the static table make no GPU call."""
    import nghttp2_amd
    hls = [[(b":method", b"GET"), (b":scheme", b"http"), (b":path", b"/")],
           [(b":status", b"200"), (b"accept-encoding", b"gzip, deflate")],
           []]
    ds = [nghttp2_amd.HpackDeflater() for _ in hls]
    st, wire = nghttp2_amd.deflate_blocks(ds, hls)
    for d, hl, s, w in zip(ds, hls, st, wire):
        ref = HO.Deflater().deflate_block(hl)
        assert w == ref and s == len(ref)
        assert d.dynamic_table() == []


def test_table_size_update_indexed_cpu():
    import nghttp2_amd
    for mx, settings in ((4096, [256]), (4096, [0, 4096]), (1024, []), (4096, [100, 50, 2000])):
        d, r = nghttp2_amd.HpackDeflater(mx), HO.Deflater(mx)
        for v in settings:
            d.change_table_size(v)
            r.change_table_size(v)
        hl = [(b":method", b"GET")]
        st, w = nghttp2_amd.deflate_blocks([d], [hl])
        assert w[0] == r.deflate_block(hl), (mx, settings)
        st, w = nghttp2_amd.deflate_blocks([d], [hl])
        assert w[0] == r.deflate_block(hl) == bytes.fromhex("82")


# ---- GPU: literals ----
def _random_lists(rng, nlists, hi=200):
    from nghttp2_amd import workloads as W
    names = [b":method", b":path", b":authority", b":status", b"cookie", b"authorization",
             b"user-agent", b"set-cookie", b"content-type", b"cache-control", b"etag", b"te",
             b"x-trace", b"x-request-id", b"accept-encoding", b"age", b"location"]
    tot = nlists * 14
    pool, off = W.gen_mixed_values(tot, seed=int(rng.integers(1 << 30)), hi=hi)
    vals = [bytes(pool[off[i]:off[i + 1]]) for i in range(tot)]
    recent = []
    out = []
    for _ in range(nlists):
        hl = []
        for _ in range(int(rng.integers(0, 14))):
            r = rng.random()
            if recent and r < 0.35:            # repeat: dynamic-table hits
                n, v = recent[int(rng.integers(0, len(recent)))]
            else:
                n = names[int(rng.integers(0, len(names)))]
                if rng.random() < 0.1:
                    n = b"x-" + bytes(rng.integers(97, 123, int(rng.integers(1, 30))))
                v = vals[int(rng.integers(0, tot))]
                if rng.random() < 0.25:
                    v = v[:int(rng.integers(0, 24))]
                if n == b":method" and rng.random() < 0.5:
                    v = b"GET"
                recent.append((n, v))
            fl = HO.NO_INDEX if rng.random() < 0.05 else 0
            hl.append((n, v, fl))
        out.append(hl)
    return out


@pytest.mark.gpu
def test_rfc7541_c4_product():
    import nghttp2_amd
    ex = EXAMPLES["RFC 7541 C.4"]
    d = nghttp2_amd.HpackDeflater()
    for hl, b in zip(_lists(ex), ex["blocks"]):
        st, w = nghttp2_amd.deflate_blocks([d], [hl])
        assert w[0].hex() == b["wire"] and st[0] == len(w[0])
    assert d.dynamic_table() == [(n.encode(), v.encode()) for n, v in ex["blocks"][-1]["table"]]
    assert d.dynamic_table_size() == ex["blocks"][-1]["table_bytes"]
    # the three blocks in one batch give the same wire
    d2 = nghttp2_amd.HpackDeflater()
    st, w = nghttp2_amd.deflate_blocks([d2] * 3, _lists(ex))
    assert [x.hex() for x in w] == [b["wire"] for b in ex["blocks"]]


def _names_min(n):
    import ctypes
    from nghttp2_amd import hd
    L = hd._deflate_lib()
    L.nghttp2_amd_hd__set_gpu_names_min.argtypes = [ctypes.c_uint32]
    L.nghttp2_amd_hd__set_gpu_names_min.restype = None
    L.nghttp2_amd_hd__set_gpu_names_min(n)


@pytest.mark.gpu
@pytest.mark.parametrize("names", ["host", "gpu"])
@pytest.mark.parametrize("table", [4096, 256, 0])
def test_deflate_random_connections_vs_oracle_and_roundtrip(table, names):
    """names: the field names' tokens and hashes from the host lookup, or
    from one k_name_tokens launch over the batch (the large-batch path)."""
    import nghttp2_amd
    _names_min(0 if names == "gpu" else 1 << 30)
    try:
        _deflate_random(table)
    finally:
        _names_min(2048)


def _deflate_random(table):
    import nghttp2_amd
    rng = np.random.Generator(np.random.PCG64(0xDEF1 + table))
    nconn, rounds = 10, 6
    ds = [nghttp2_amd.HpackDeflater() for _ in range(nconn)]
    rs = [HO.Deflater() for _ in range(nconn)]
    infs = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
    if table != 4096:
        for x in ds + rs + infs:
            x.change_table_size(table)
    order, lists = [], []
    for _ in range(rounds):
        for c in rng.permutation(nconn):
            order.append(int(c))
        lists += _random_lists(rng, nconn)
    st, wire = nghttp2_amd.deflate_blocks([ds[c] for c in order], lists)
    for k, c in enumerate(order):
        want = rs[c].deflate_block(lists[k])
        assert wire[k] == want, (k, c)
        assert st[k] == len(want)
    for c in range(nconn):
        assert ds[c].dynamic_table() == [tuple(e) for e in rs[c].table]
        assert ds[c].dynamic_table_size() == rs[c].size
    # round trip: the batched inflater gets the fields back, flags included
    ist, fields = nghttp2_amd.inflate_blocks([infs[c] for c in order], wire)
    for k in range(len(order)):
        want = [(n, v, fl) for n, v, fl in lists[k]]
        got = fields[k]
        assert ist[k] == len(want), k
        for (n, v, fl), (gn, gv, gf) in zip(want, got):
            assert (gn, gv) == (n, v)
            if fl:
                assert gf == HO.NO_INDEX


@pytest.mark.gpu
def test_deflate_buffer_error_is_sticky():
    import nghttp2_amd
    import ctypes
    from nghttp2_amd import hd
    d = nghttp2_amd.HpackDeflater()
    big = [(b"x-big", b"a" * 5000)]
    L = hd._deflate_lib()
    nva = (hd._NvIn * 1)()
    bn, bv = ctypes.create_string_buffer(big[0][0]), ctypes.create_string_buffer(big[0][1])
    nva[0].name, nva[0].value = ctypes.cast(bn, ctypes.c_void_p), ctypes.cast(bv, ctypes.c_void_p)
    nva[0].namelen, nva[0].valuelen = 5, 5000
    off = (ctypes.c_uint32 * 3)(0, 1, 1)
    out = (ctypes.c_uint8 * 64)()
    oo = (ctypes.c_uint32 * 3)()
    st = (ctypes.c_int32 * 2)()
    dd = (ctypes.c_void_p * 2)(d.p.value, d.p.value)
    rv = L.nghttp2_amd_hd_deflate_blocks(dd, 2, nva, off, out, 64, oo, st, None)
    assert rv == hd.NGHTTP2_ERR_BUFFER_ERROR
    assert st[0] == hd.NGHTTP2_ERR_BUFFER_ERROR and st[1] == hd.NGHTTP2_ERR_HEADER_COMP
    assert oo[2] == 0
    st2, w2 = nghttp2_amd.deflate_blocks([d], [[(b":method", b"GET")]])
    assert st2[0] == hd.NGHTTP2_ERR_HEADER_COMP and w2[0] == b""


def test_deflate_gpu_stage_failure_turns_deflaters_bad_cpu():
    """A failure after pass 1 (which has already changed the tables) marks
    every deflater of the batch bad and reports the error on every block, as
    nghttp2_hd_deflate_hd_bufs sets ctx.bad on each failure path
    (lib/nghttp2_hd.c:1509-1516).  The fault hook fails the GPU stage before
    any HIP call, so this runs without a GPU."""
    import ctypes
    import nghttp2_amd
    from nghttp2_amd import hd
    L = hd._deflate_lib()
    L.nghttp2_amd_hd__test_fail_deflate_gpu.argtypes = [ctypes.c_int]
    L.nghttp2_amd_hd__test_fail_deflate_gpu.restype = None
    d1, d2 = nghttp2_amd.HpackDeflater(), nghttp2_amd.HpackDeflater()
    lists = [[(b"x-custom", b"value-one")], [(b":method", b"GET"), (b"x-other", b"two")]]
    L.nghttp2_amd_hd__test_fail_deflate_gpu(1)
    try:
        with pytest.raises(RuntimeError):
            nghttp2_amd.deflate_blocks([d1, d2], lists)
    finally:
        L.nghttp2_amd_hd__test_fail_deflate_gpu(0)
    # both deflaters are bad: even an indexed-only list (no GPU work) fails
    for d in (d1, d2):
        st, w = nghttp2_amd.deflate_blocks([d], [[(b":method", b"GET")]])
        assert st[0] == hd.NGHTTP2_ERR_HEADER_COMP and w[0] == b""


def test_deflate_names_stage_failure_leaves_deflaters_cpu():
    """The batched name lookup runs before pass 1: a failure there returns
    the error and leaves every deflater as it was (not bad)."""
    import ctypes
    import nghttp2_amd
    from nghttp2_amd import hd
    L = hd._deflate_lib()
    L.nghttp2_amd_hd__test_fail_deflate_gpu.argtypes = [ctypes.c_int]
    L.nghttp2_amd_hd__test_fail_deflate_gpu.restype = None
    d = nghttp2_amd.HpackDeflater()
    _names_min(0)
    L.nghttp2_amd_hd__test_fail_deflate_gpu(1)
    try:
        with pytest.raises(RuntimeError):
            nghttp2_amd.deflate_blocks([d], [[(b"x-custom", b"value-one")]])
    finally:
        L.nghttp2_amd_hd__test_fail_deflate_gpu(0)
        _names_min(2048)
    assert d.dynamic_table() == []
    st, w = nghttp2_amd.deflate_blocks([d], [[(b":method", b"GET")]])
    assert st[0] == 1 and w[0] == b"\x82"
