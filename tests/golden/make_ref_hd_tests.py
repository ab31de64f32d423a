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

- round 5, the rest of the suite (the remaining hd tests of
  tests/nghttp2_hd_test.c; block wire computed as the reference's
  nghttp2_hd_emit_indname_block / emit_newname_block / emit_table_size
  write it, lib/nghttp2_hd.c:1046-1128, :947-973, with the string literals
  from the restated emit_string, oracle/huff_oracle.c, pinned by RFC 7541):
  deflate sequences (test_nghttp2_hd_deflate :68-181,
  deflate_same_indexed_repr :183-240, ringbuf_reserve :726-777), inflate
  sequences with the table checks (inflate_indexed :242-281,
  indname_noinc :283-324, indname_inc :326-362, indname_inc_eviction
  :364-419, newname_noinc :421-464, newname_inc :466-500, clearall_inc
  :502-575), the change_table_size script (:779-1051), public_api
  (:1322-1365), deflate_hd_vec (:1367-1512) and decode_length (:1514-1603).
  Scenario steps that only the reference's internals can observe
  (settings_hd_table_bufsize_max, min_hd_table_bufsize_max) are kept as
  oracle-only expectations.

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


def encode_int(n, prefix, first=0):
    """The RFC 7541 5.1 prefix integer (the test's encode_length helper,
    :1514-1540, and the library's): first byte's high bits kept."""
    k = (1 << prefix) - 1
    if n < k:
        return bytes([first | n])
    out = bytearray([first | k])
    n -= k
    while n >= 128:
        out.append(0x80 | (n & 0x7F))
        n >>= 7
    out.append(n)
    return bytes(out)


WITH, WITHOUT, NEVER = 0x40, 0x00, 0x10


def emit_string(b):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import oracle as O
    return O.emit_string(b)


def indname(idx, value, mode):
    """nghttp2_hd_emit_indname_block(bufs, idx, nv, mode): index idx + 1."""
    return encode_int(idx + 1, 6 if mode == WITH else 4, mode) + emit_string(value)


def newname(name, value, mode):
    """nghttp2_hd_emit_newname_block(bufs, nv, mode)."""
    return bytes([mode]) + emit_string(name) + emit_string(value)


def hexs(b):
    return bytes(b).hex()


def more_cases(text):
    """The rest of the reference's hd suite as data (round 5)."""
    fn = lambda name: nv_arrays(function_body(text, name))
    HC, INSUFF = -523, -525
    out = {}
    # ---- deflate sequences: one deflater and one inflater, list by list
    d = fn("test_nghttp2_hd_deflate")
    seqs = [{"test": "test_nghttp2_hd_deflate :68-181", "deflate_max": 4096, "settings": [],
             "lists": [{"nva": d["nva%d" % k], "expect": {"rv": 0, "blocklen_gt": 0}}
                       for k in range(1, 6)]}]
    s = fn("test_nghttp2_hd_deflate_same_indexed_repr")
    seqs.append({"test": "test_nghttp2_hd_deflate_same_indexed_repr :183-240",
                 "deflate_max": 4096, "settings": [],
                 "lists": [{"nva": s["nva1"], "expect": {"rv": 0, "blocklen_gt": 0}},
                           {"nva": s["nva2"], "expect": {"rv": 0, "blocklen": 3}}]})
    # ringbuf_reserve: name "a", the 4 bytes of int i (little endian) as value
    body = function_body(text, "test_nghttp2_hd_ringbuf_reserve")
    assert "i < 150" in body and "init2(&deflater, 8000" in body
    seqs.append({"test": "test_nghttp2_hd_ringbuf_reserve :726-777", "deflate_max": 8000,
                 "settings": [8000], "values_hex": True,
                 "lists": [{"nva": [["a", i.to_bytes(4, "little").hex()]],
                            "expect": {"rv": 0, "blocklen_gt": 0}} for i in range(150)]})
    out["deflate_sequences"] = seqs
    # ---- inflate sequences
    iseq = []
    iseq.append({"test": "test_nghttp2_hd_inflate_indexed :242-281", "blocks": [
        {"block": "84", "expect": {"fields": [[":path", "/"]]}},
        {"block": "80", "expect": {"rv": HC}}]})
    ni = fn("test_nghttp2_hd_inflate_indname_noinc")["nv"]
    iseq.append({"test": "test_nghttp2_hd_inflate_indname_noinc :283-324", "blocks": [
        {"block": hexs(indname(57, v.encode(), WITHOUT)),
         "expect": {"fields": [[n, v]], "table_len": 0, "num_entries": 61}} for n, v in ni]})
    body = function_body(text, "test_nghttp2_hd_inflate_indname_inc")
    m = re.search(r'MAKE_NV\("([^"]*)", "([^"]*)"\)', body)
    n, v = m.group(1), m.group(2)
    iseq.append({"test": "test_nghttp2_hd_inflate_indname_inc :326-362", "blocks": [
        {"block": hexs(indname(57, v.encode(), WITH)),
         "expect": {"fields": [[n, v]], "table_len": 1, "num_entries": 62,
                    "newest": [n, v]}}]})
    body = function_body(text, "test_nghttp2_hd_inflate_indname_inc_eviction")
    assert "value[1025]" in body and "memset(value, '0'" in body
    val = b"0" * 1024
    blk = b"".join(indname(i, val, WITH) for i in (14, 15, 16, 17))
    iseq.append({"test": "test_nghttp2_hd_inflate_indname_inc_eviction :364-419", "blocks": [
        {"block": hexs(blk), "expect": {"nfields": 4, "field0_name": "accept-charset",
                                        "field0_valuelen": 1024, "table_len": 3,
                                        "num_entries": 64}}]})
    nn = fn("test_nghttp2_hd_inflate_newname_noinc")["nv"]
    iseq.append({"test": "test_nghttp2_hd_inflate_newname_noinc :421-464", "blocks": [
        {"block": hexs(newname(n.encode(), v.encode(), WITHOUT)),
         "expect": {"fields": [[n, v]], "table_len": 0}} for n, v in nn]})
    body = function_body(text, "test_nghttp2_hd_inflate_newname_inc")
    m = re.search(r'MAKE_NV\("([^"]*)", "([^"]*)"\)', body)
    n, v = m.group(1), m.group(2)
    iseq.append({"test": "test_nghttp2_hd_inflate_newname_inc :466-500", "blocks": [
        {"block": hexs(newname(n.encode(), v.encode(), WITH)),
         "expect": {"fields": [[n, v]], "table_len": 1, "newest": [n, v]}}]})
    body = function_body(text, "test_nghttp2_hd_inflate_clearall_inc")
    assert "value[4061]" in body and 'hd_name[] = "alpha"' in body
    big = newname(b"alpha", b"0" * 4060, WITH)    # 4097 bytes of table space
    fits = newname(b"alpha", b"0" * 4059, WITH)   # 4096: just fits
    iseq.append({"test": "test_nghttp2_hd_inflate_clearall_inc :502-575", "blocks": [
        {"block": hexs(big), "expect": {"fields": [["alpha", "0" * 4060]], "table_len": 0}},
        {"block": hexs(big), "expect": {"fields": [["alpha", "0" * 4060]], "table_len": 0}},
        {"block": hexs(fits), "expect": {"fields": [["alpha", "0" * 4059]], "table_len": 1}}]})
    # whether a block carries a Huffman literal (the H bit of any string
    # literal the emit helpers wrote): such a block needs the GPU decode
    def has_huff(block_hex):
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
        from oracle import hpack_oracle as HO
        return HO.block_has_huffman(bytes.fromhex(block_hex))
    for sq in iseq:
        for b in sq["blocks"]:
            b["huffman"] = has_huff(b["block"])
    out["inflate_sequences"] = iseq
    # ---- change_table_size (:779-1051), as a script over one deflater and
    # one inflater at a time; "dmax"/"imax" are the reference's
    # ctx.hd_table_bufsize_max (get_max_dynamic_table_size), "dlen"/"ilen"
    # hd_table.len, "dent"/"ient" get_num_table_entries; "iset" / "dmin" are
    # settings_hd_table_bufsize_max / min_hd_table_bufsize_max (internal:
    # checked on the restated oracle only)
    c = fn("test_nghttp2_hd_change_table_size")
    U32 = 0xFFFFFFFF
    script = [
        {"op": "new", "deflate_max": 4096},
        {"op": "ichange", "v": 8000, "line": 804}, {"op": "dchange", "v": 8000, "line": 805},
        {"op": "check", "dmax": 4096, "imax": 4096, "iset": 8000, "line": 807},
        {"op": "roundtrip", "nva": "nva", "line": 813,
         "check": {"dlen": 2, "dent": 63, "dmax": 4096, "ilen": 2, "ient": 63, "imax": 4096, "iset": 8000}},
        {"op": "ichange", "v": 1024, "line": 832}, {"op": "dchange", "v": 1024, "line": 833},
        {"op": "check", "dmax": 1024, "imax": 1024, "iset": 1024, "line": 835},
        {"op": "roundtrip", "nva": "nva", "line": 840,
         "check": {"dlen": 2, "dent": 63, "dmax": 1024, "ilen": 2, "ient": 63, "imax": 1024, "iset": 1024}},
        {"op": "ichange", "v": 0, "line": 859}, {"op": "dchange", "v": 0, "line": 860},
        {"op": "check", "dlen": 0, "dent": 61, "dmax": 0, "ilen": 0, "ient": 61, "imax": 0, "iset": 0, "line": 862},
        {"op": "roundtrip", "nva": "nva", "line": 871,
         "check": {"dlen": 0, "dent": 61, "dmax": 0, "ilen": 0, "ient": 61, "imax": 0, "iset": 0}},
        {"op": "new", "deflate_max": 8192, "line": 896},
        {"op": "ichange", "v": 8000, "line": 900}, {"op": "dchange", "v": 8000, "line": 901},
        {"op": "check", "dmax": 8000, "imax": 4096, "iset": 8000, "line": 903},
        {"op": "roundtrip", "nva": "nva", "line": 911,
         "check": {"dlen": 2, "dmax": 8000, "ilen": 2, "imax": 8000, "iset": 8000}},
        {"op": "ichange", "v": 16383, "line": 927}, {"op": "dchange", "v": 16383, "line": 928},
        {"op": "check", "dmax": 8192, "imax": 8000, "iset": 16383, "line": 930},
        {"op": "roundtrip", "nva": "nva", "line": 939,
         "check": {"dlen": 2, "dmax": 8192, "ilen": 2, "imax": 8192, "iset": 16383}},
        {"op": "inflate", "block": hexs(encode_int(25600, 5, 0x20)), "expect_rv": HC, "line": 957},
        {"op": "new", "deflate_max": 1024, "line": 970},
        {"op": "check", "dmax": 1024, "line": 973},
        {"op": "roundtrip", "nva": "nva", "line": 976,
         "check": {"dlen": 2, "dmax": 1024, "ilen": 2, "imax": 1024, "iset": 4096}},
        {"op": "new", "deflate_max": U32, "line": 996},
        {"op": "ichange", "v": U32, "line": 999}, {"op": "dchange", "v": U32, "line": 1001},
        {"op": "roundtrip", "nva": "nva", "line": 1004,
         "check": {"dmax": U32, "imax": U32, "iset": U32}},
        {"op": "new", "deflate_max": 4096, "line": 1021},
        {"op": "ichange", "v": 0, "line": 1024}, {"op": "ichange", "v": 3000, "line": 1025},
        {"op": "dchange", "v": 0, "line": 1026}, {"op": "dchange", "v": 3000, "line": 1027},
        {"op": "check", "dmin": 0, "dmax": 3000, "line": 1029},
        {"op": "roundtrip", "nva": "nva2", "line": 1032, "blocklen_gt": 3,
         "check": {"dmax": 3000, "dmin": U32, "imax": 3000, "iset": 3000}},
    ]
    out["change_table_size"] = {"test": "test_nghttp2_hd_change_table_size :779-1051",
                                "nva": c["nva"], "nva2": c["nva2"], "script": script}
    # ---- public_api (:1322-1365)
    pa = fn("test_nghttp2_hd_public_api")["nva"]
    out["public_api"] = {"test": "test_nghttp2_hd_public_api :1322-1365", "nva": pa,
                         "insuff": INSUFF}
    # ---- deflate_hd_vec (:1367-1512): chunk layouts relative to the bound
    hv = fn("test_nghttp2_hd_deflate_hd_vec")["nva"]
    out["deflate_hd_vec"] = {"test": "test_nghttp2_hd_deflate_hd_vec :1367-1512", "nva": hv,
                             "cases": [
                                 {"chunks": "half_half", "expect": "ok", "line": 1396},
                                 {"chunks": "null", "expect": INSUFF, "line": 1427},
                                 {"chunks": "zero_zero", "expect": INSUFF, "line": 1435},
                                 {"chunks": "half_half_plus1", "expect": "ok", "line": 1454},
                                 {"chunks": "ones", "expect": "ok", "line": 1488}]}
    # ---- decode_length (:1542-1603)
    u32max = encode_int(U32, 7)
    out["decode_length"] = {"test": "test_nghttp2_hd_decode_length :1542-1603", "cases": [
        {"bytes": hexs(u32max), "prefix": 7, "rv": len(u32max), "fin": 1, "res": U32, "line": 1553},
        {"bytes": hexs(u32max), "prefix": 7, "bytewise": True, "fin_at": len(u32max) - 1,
         "res": U32, "line": 1568},
        {"bytes": hexs(encode_int(1 << 32, 7)), "prefix": 7, "rv": -1, "line": 1585},
        {"bytes": hexs(bytes([255, 128, 128, 128, 128, 128, 1])), "prefix": 8, "rv": -1, "line": 1592}]}
    out["not_applicable"] = {
        "test_nghttp2_hd_huff_encode :1605-1633 / huff_decode :1635-1670":
            "covered by the link-level drop-in (tests/c/test_compat.c, tests/test_compat.py)"}
    return out


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
    out.update(more_cases(text))
    with open(os.path.join(HERE, "ref_hd_tests.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote ref_hd_tests.json: %d sets, %d inflate cases" % (len(sets), len(inflate_cases)))


if __name__ == "__main__":
    main()
