"""The reference's own HPACK unit tests, replayed through the product front-ends
(nghttp2_amd.inflate_blocks / deflate_blocks over the C ABI) and through the
restated oracle (oracle/hpack_oracle.py), with the reference's exact
expectations (tests/golden/ref_hd_tests.json, read out of
tests/nghttp2_hd_test.c by tests/golden/make_ref_hd_tests.py):

- test_nghttp2_hd_inflate_zero_length_huffman      :577-610
- test_nghttp2_hd_inflate_expect_table_size_update :612-701
- test_nghttp2_hd_inflate_unexpected_table_size_update :703-724
- test_nghttp2_hd_deflate_inflate                  :1080-1236
- test_nghttp2_hd_no_index                         :1238-1287
- test_nghttp2_hd_deflate_bound                    :1289-1320

Blocks without Huffman literals make no GPU call, so those cases run on the
CPU; a block with a Huffman literal, and every deflate with literals, is gpu.
"""
import ctypes
import json
import os

import pytest

from oracle import hpack_oracle as HO

REF = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_hd_tests.json")))
HEADER_COMP = -523


def _has_huffman_literal(block):
    # only the zero-length-Huffman case carries one among these blocks
    return "zero_length_huffman" in block["test"]


def _check_inflate_case(case, inflate):
    st, fields = inflate(case)
    exp = case["expect"]
    if "rv" in exp:
        assert st == exp["rv"], case["test"]
    else:
        want = [(n.encode(), v.encode(), 0) for n, v in exp["fields"]]
        assert st == len(want), case["test"]
        assert fields == want, case["test"]


def _product_inflate(case):
    import nghttp2_amd
    inf = nghttp2_amd.HpackInflater()
    for v in case["settings"]:
        inf.change_table_size(v)
    st, f = nghttp2_amd.inflate_blocks([inf], [bytes.fromhex(case["block"])])
    return st[0], f[0]


def _oracle_inflate(case):
    ref = HO.Inflater()
    for v in case["settings"]:
        ref.change_table_size(v)
    return ref.inflate_block(bytes.fromhex(case["block"]))


@pytest.mark.parametrize("case", REF["inflate_cases"], ids=lambda c: c["test"].split()[-1])
def test_reference_inflate_cases_oracle(case):
    """The restated inflater meets the reference's expectations."""
    _check_inflate_case(case, _oracle_inflate)


@pytest.mark.parametrize("case", [c for c in REF["inflate_cases"] if not _has_huffman_literal(c)],
                         ids=lambda c: c["test"].split()[-1])
def test_reference_inflate_cases_cpu(case):
    _check_inflate_case(case, _product_inflate)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in REF["inflate_cases"] if _has_huffman_literal(c)],
                         ids=lambda c: c["test"].split()[-1])
def test_reference_inflate_cases_huffman(case):
    _check_inflate_case(case, _product_inflate)


def _sets():
    return [[(n.encode(), v.encode()) for n, v in s] for s in REF["deflate_inflate"]["sets"]]


def test_reference_deflate_inflate_oracle():
    """check_deflate_inflate (:1053-1078) over the ten sets, restated
    deflater into restated inflater."""
    d, i = HO.Deflater(), HO.Inflater()
    for s in _sets():
        wire = d.deflate_block(s)
        st, fields = i.inflate_block(wire)
        assert st == len(s)
        assert [(n, v) for n, v, _ in fields] == s


@pytest.mark.gpu
def test_reference_deflate_inflate_product():
    """The ten sets, one deflate_blocks / inflate_blocks call per set as the
    reference test calls them, and again as one batch of ten lists: rv 0,
    the inflated fields equal the input, and the wire equals the restated
    deflater's."""
    import nghttp2_amd
    sets = _sets()
    d, i = nghttp2_amd.HpackDeflater(), nghttp2_amd.HpackInflater()
    rd = HO.Deflater()
    wires = []
    for s in sets:
        st, wire = nghttp2_amd.deflate_blocks([d], [s])
        assert st[0] == len(wire[0]) > 0
        assert wire[0] == rd.deflate_block(s)
        ist, fields = nghttp2_amd.inflate_blocks([i], [wire[0]])
        assert ist[0] == len(s)
        assert [(n, v) for n, v, _ in fields[0]] == s
        wires.append(wire[0])
    # the same ten lists as one batch on a fresh pair: the same wire
    d2, i2 = nghttp2_amd.HpackDeflater(), nghttp2_amd.HpackInflater()
    st, w2 = nghttp2_amd.deflate_blocks([d2] * len(sets), sets)
    assert w2 == wires
    ist, fields = nghttp2_amd.inflate_blocks([i2] * len(sets), w2)
    assert ist == [len(s) for s in sets]
    assert [[(n, v) for n, v, _ in f] for f in fields] == sets
    assert d2.dynamic_table() == d.dynamic_table() == i2.dynamic_table()


@pytest.mark.gpu
def test_reference_no_index():
    import nghttp2_amd
    nva = [(n.encode(), v.encode(), 1 if k >= REF["no_index"]["no_index_from"] else 0)
           for k, (n, v) in enumerate(REF["no_index"]["nva"])]
    d, i = nghttp2_amd.HpackDeflater(), nghttp2_amd.HpackInflater()
    st, wire = nghttp2_amd.deflate_blocks([d], [nva])
    assert st[0] > 0
    ist, fields = nghttp2_amd.inflate_blocks([i], wire)
    assert ist[0] == len(nva)
    assert fields[0] == [(n, v, fl) for n, v, fl in nva]


def test_reference_deflate_bound_cpu():
    import nghttp2_amd
    from nghttp2_amd.hd import _NvIn, _deflate_lib
    L = _deflate_lib()
    L.nghttp2_amd_hd_deflate_bound.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.nghttp2_amd_hd_deflate_bound.restype = ctypes.c_size_t
    nva = [(n.encode(), v.encode()) for n, v in REF["deflate_bound"]["nva"]]
    arr = (_NvIn * len(nva))()
    keep = []
    for k, (n, v) in enumerate(nva):
        bn, bv = ctypes.create_string_buffer(n, len(n)), ctypes.create_string_buffer(v, len(v))
        keep += [bn, bv]
        arr[k].name = ctypes.cast(bn, ctypes.c_void_p)
        arr[k].value = ctypes.cast(bv, ctypes.c_void_p)
        arr[k].namelen, arr[k].valuelen, arr[k].flags = len(n), len(v), 0
    d = nghttp2_amd.HpackDeflater()
    assert L.nghttp2_amd_hd_deflate_bound(d.p, arr, len(nva)) == REF["deflate_bound"]["bound"]
    # the restated deflater's block for the list is shorter than the bound
    assert len(HO.Deflater().deflate_block(nva)) < REF["deflate_bound"]["bound"]


@pytest.mark.gpu
def test_reference_deflate_bound_product():
    import nghttp2_amd
    nva = [(n.encode(), v.encode()) for n, v in REF["deflate_bound"]["nva"]]
    d = nghttp2_amd.HpackDeflater()
    st, wire = nghttp2_amd.deflate_blocks([d], [nva])
    assert 0 < len(wire[0]) < REF["deflate_bound"]["bound"]
