#!/usr/bin/env python3
"""Generate tests/golden/ref_hd_tests.json: the inputs and expectations of
the reference's own HPACK unit tests, read out of tests/nghttp2_hd_test.c as
data.

BUILD-CONTAINER ONLY (reads /root/reference as text; never runs on the GPU
box).  Vectors:

- deflate_inflate: the ten header sets of test_nghttp2_hd_deflate_inflate
  (:1080-1236), deflated in order by one deflater and inflated by one
  inflater; expectation (check_deflate_inflate, :1053-1078): rv 0 and the
  inflated fields equal the input, set by set.
- no_index: test_nghttp2_hd_no_index (:1238-1287): fields 1.. flagged
  NGHTTP2_NV_FLAG_NO_INDEX; they round-trip with the flag kept, field 0
  without it.
- deflate_bound: test_nghttp2_hd_deflate_bound (:1289-1320): the bound is
  12 + 6*2*nvlen + the name and value bytes, above the block's length, and
  unchanged after the deflate.
- inflate cases: test_nghttp2_hd_inflate_zero_length_huffman (:577-610),
  test_nghttp2_hd_inflate_expect_table_size_update (:612-701),
  test_nghttp2_hd_inflate_unexpected_table_size_update (:703-724): the
  settings changes before the block, the block bytes (table size updates as
  nghttp2_hd_emit_table_size writes them: 0x20 | 5-bit prefix integer), and
  the reference's expected result (HEADER_COMP or the fields).

Usage: python3 tests/golden/make_ref_hd_tests.py
"""
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REF_TEST = "/root/reference/tests/nghttp2_hd_test.c"


def c_string(s):
    return bytes(s, "ascii").decode("unicode_escape").encode("latin-1").decode("latin-1")


def nv_arrays(body):
    """{name: [(n, v), ...]} of the `static const nghttp2_nv X[] = {...}` /
    `nghttp2_nv X[] = {...}` arrays in body."""
    out = {}
    for m in re.finditer(r"nghttp2_nv\s+(\w+)\[\]\s*=\s*\{(.*?)\};", body, re.S):
        rows = re.findall(r'MAKE_NV\(\s*"((?:[^"\\]|\\.)*)"\s*,\s*"((?:[^"\\]|\\.)*)"\s*\)',
                          m.group(2))
        out[m.group(1)] = [(c_string(a), c_string(b)) for a, b in rows]
    return out


def function_body(text, name):
    start = text.index("void %s(void) {" % name)
    return text[start:text.index("\n}\n", start)]


def table_size_update(v):
    # nghttp2_hd_emit_table_size: encode_length(.., 5) with 0x20 set
    out = bytearray()
    k = (1 << 5) - 1
    if v < k:
        return bytes([0x20 | v])
    out.append(0x20 | k)
    v -= k
    while v >= 128:
        out.append(0x80 | (v & 0x7F))
        v >>= 7
    out.append(v)
    return bytes(out)


def main():
    text = open(REF_TEST).read()
    di = nv_arrays(function_body(text, "test_nghttp2_hd_deflate_inflate"))
    sets = [di["nv%d" % i] for i in range(1, 11)]
    ni = nv_arrays(function_body(text, "test_nghttp2_hd_no_index"))["nva"]
    db = nv_arrays(function_body(text, "test_nghttp2_hd_deflate_bound"))["nva"]
    assert len(sets) == 10 and all(sets) and len(ni) == 5 and len(db) == 2
    HC = -523
    inflate_cases = [
        {"test": "test_nghttp2_hd_inflate_zero_length_huffman :577-610",
         "settings": [], "block": bytes([0x40, 0x01, 0x78, 0x80]).hex(),
         "expect": {"fields": [["x", ""]]}},
        {"test": "test_nghttp2_hd_inflate_expect_table_size_update :630-636",
         "settings": [4095, 4096], "block": "82", "expect": {"rv": HC}},
        {"test": "test_nghttp2_hd_inflate_expect_table_size_update :643-647",
         "settings": [4096], "block": "82", "expect": {"fields": [[":method", "GET"]]}},
        {"test": "test_nghttp2_hd_inflate_expect_table_size_update :654-658",
         "settings": [4097], "block": "82", "expect": {"fields": [[":method", "GET"]]}},
        {"test": "test_nghttp2_hd_inflate_expect_table_size_update :664-671",
         "settings": [111, 4096], "block": table_size_update(112).hex(), "expect": {"rv": HC}},
        {"test": "test_nghttp2_hd_inflate_expect_table_size_update :677-685",
         "settings": [111, 4096], "block": (table_size_update(111) + table_size_update(4096)).hex(),
         "expect": {"fields": []}},
        {"test": "test_nghttp2_hd_inflate_expect_table_size_update :691-699",
         "settings": [111, 4095], "block": (table_size_update(111) + table_size_update(4096)).hex(),
         "expect": {"rv": HC}},
        {"test": "test_nghttp2_hd_inflate_unexpected_table_size_update :703-724",
         "settings": [], "block": "8220", "expect": {"rv": HC}},
    ]
    out = {
        "source": "tests/nghttp2_hd_test.c of the reference (nghttp2 1.70.90), read as data",
        "deflate_inflate": {"test": "test_nghttp2_hd_deflate_inflate :1080-1236", "sets": sets},
        "no_index": {"test": "test_nghttp2_hd_no_index :1238-1287", "nva": ni,
                     "no_index_from": 1},
        "deflate_bound": {"test": "test_nghttp2_hd_deflate_bound :1289-1320", "nva": db,
                          "bound": 12 + 6 * 2 * len(db) + sum(len(a) + len(b) for a, b in db)},
        "inflate_cases": inflate_cases,
    }
    with open(os.path.join(HERE, "ref_hd_tests.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote ref_hd_tests.json: %d sets, %d inflate cases" % (len(sets), len(inflate_cases)))


if __name__ == "__main__":
    main()
