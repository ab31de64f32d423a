"""CPU tests: the oracle (and the product's tables) pinned to the reference.

The oracle is oracle/huff_oracle.c, a restatement of
lib/nghttp2_hd_huffman.c.  It is pinned by (a) the sha256 of the tables the
reference's own generator mkhufftbl.py prints (tests/golden/
reference_tables.json, produced by oracle/pin_reference.py in the build
container) and (b) the reference's Huffman unit-test expectations
(tests/nghttp2_hd_test.c:1605-1670) plus RFC 7541 App. C literals
(tests/golden/known_answers.json).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_oracle_tables_match_reference_generator():
    ref = _json("reference_tables.json")
    sym, dec = O.tables_ref_layout()
    assert hashlib.sha256(sym).hexdigest() == ref["sym_sha256"]
    assert hashlib.sha256(dec).hexdigest() == ref["dec_sha256"]


def test_product_generator_tables_match_reference():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(GOLD), "..", "nghttp2_amd", "tools"))
    from nghttp2_amd.tools import gen_tables
    ref = _json("reference_tables.json")
    sym, dec = gen_tables.packed_ref_layout(gen_tables.build())
    assert hashlib.sha256(sym).hexdigest() == ref["sym_sha256"]
    assert hashlib.sha256(dec).hexdigest() == ref["dec_sha256"]


@pytest.mark.parametrize("v", _json("known_answers.json")["ref_unit_decode"],
                         ids=lambda v: v["src"] or "empty")
def test_reference_unit_decode_vectors(v):
    rv, out, ctx = O.decode(bytes.fromhex(v["src"]), v["final"])
    assert rv == v["rv"], v["cite"]
    if "out" in v:
        assert out.hex() == v["out"]
    if "failure_state" in v:
        assert O.failure_state(ctx) == v["failure_state"]


def test_reference_unit_encode_roundtrip():
    # tests/nghttp2_hd_test.c:1605-1633: bytes 22..0 (28/30-bit codes)
    raw = bytes.fromhex(_json("known_answers.json")["ref_unit_encode_roundtrip"][0]["raw"])
    rv, enc = O.encode(raw)
    assert rv == 0
    assert len(enc) == O.encode_count(raw)
    rv, dec, ctx = O.decode(enc, 1)
    assert rv == len(enc) and dec == raw


@pytest.mark.parametrize("pair", _json("known_answers.json")["rfc7541"], ids=lambda p: p[0][:20])
def test_rfc7541_appendix_c_literals(pair):
    s, h = pair
    rv, enc = O.encode(s.encode())
    assert rv == 0 and enc.hex() == h
    rv, dec, _ = O.decode(bytes.fromhex(h), 1)
    assert rv == len(h) // 2 and dec == s.encode()


def test_encode_buffer_error_like_wrap_mode():
    # a wrap-mode bufs one byte short fails with NGHTTP2_ERR_BUFFER_ERROR
    # (lib/nghttp2_buf.c:303-305 via nghttp2_bufs_addb), as
    # test_nghttp2_hd_public_api relies on (tests/nghttp2_hd_test.c:1322-1365).
    raw = b"www.example.com"
    need = O.encode_count(raw)
    rv, enc = O.encode(raw, cap=need)
    assert rv == 0 and len(enc) == need
    rv, part = O.encode(raw, cap=need - 1)
    assert rv == O.NGHTTP2_ERR_BUFFER_ERROR


def test_streaming_decode_equals_whole():
    # chunked decode with a carried context (tests/nghttp2_test_helper.c:165-205)
    from nghttp2_amd import workloads as W
    pool, off = W.gen_all_bytes(300, seed=7)
    enc, eoff = O.encode_batch(pool, off)
    rng = np.random.default_rng(3)
    for i in range(300):
        e = bytes(enc[eoff[i]:eoff[i + 1]])
        rv, whole, wctx = O.decode(e, 1)
        ctx = O.Ctx(0, O.ACCEPTED)
        out = b""
        cuts = sorted(rng.integers(0, len(e) + 1, size=3)) if e else []
        prev = 0
        for c in list(cuts) + [len(e)]:
            fin = 1 if c == len(e) else 0
            r, o, ctx = O.decode(e[prev:c], fin, ctx)
            out += o
            prev = c
        assert out == whole and (ctx.fstate, ctx.flags) == (wctx.fstate, wctx.flags)


def test_numpy_packer_matches_oracle():
    from nghttp2_amd import workloads as W
    pool, off = W.gen_all_bytes(3000, seed=11)
    pk, po, _ = W.pack_symbols(pool[:off[-1]].astype(np.int64), off.astype(np.int64))
    enc, eoff = O.encode_batch(pool, off)
    assert np.array_equal(po, eoff)
    assert np.array_equal(pk[:po[-1]], enc)


def test_golden_vectors_regression():
    """The committed golden vectors (tests/golden/make_golden.py) still come
    out of the oracle unchanged."""
    from tests.golden import make_golden
    for name in make_golden.CASES:
        g = make_golden.load(name)
        if g["kind"] == "roundtrip":
            enc, eoff = O.encode_batch(g["raw"], g["raw_off"])
            assert np.array_equal(eoff, g["enc_off"]), name
            assert np.array_equal(enc, g["enc"][:eoff[-1]]), name
            src, soff = enc, eoff
        else:
            src, soff = g["enc"], g["enc_off"]
        dst, doff, st, fs, fl = O.decode_batch(src, soff)
        assert np.array_equal(st, g["status"]), name
        assert np.array_equal(fs, g["fstate"]), name
        assert np.array_equal(fl, g["flags"]), name
        assert hashlib.sha256(make_golden.decoded_bytes(dst, doff, st)).hexdigest() \
            == g["dec_sha256"], name


# ---- HPACK string literal framing (emit_string) ----
def test_oracle_prefix_integers_rfc7541():
    ka = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
    for v, prefix, hx, _cite in ka["rfc7541_integers"]["vectors"]:
        assert O.encode_length(v, prefix).hex() == hx


def test_oracle_string_literals_rfc7541():
    ka = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
    for s, hx, _cite in ka["rfc7541_string_literals"]["vectors"]:
        assert O.emit_string(s.encode()).hex() == hx


def test_oracle_emit_string_raw_and_long_lengths():
    # Huffman only when strictly shorter (lib/nghttp2_hd.c:1011): raw for bytes
    # whose codes are long, and multi-byte length prefixes from 127 on
    for n in (0, 1, 126, 127, 128, 254, 255, 256, 16383 + 127, 16384 + 127, 70000):
        raw = bytes(range(256)) * (n // 256 + 1)
        raw = raw[:n]
        out = O.emit_string(raw)
        enclen = O.encode_count(raw)
        huff = enclen < n
        plen = len(O.encode_length(enclen if huff else n, 7))
        assert out[0] >> 7 == (1 if huff else 0)
        assert len(out) == plen + (enclen if huff else n)
        if not huff:
            assert out[plen:] == raw
    assert O.emit_string(b"") == b"\x00"
