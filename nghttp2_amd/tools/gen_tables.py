#!/usr/bin/env python3
"""Generate the HPACK Huffman device tables (nghttp2_amd/csrc/hd_huff_tables.inc).

The product's tables are derived here from the 257 RFC 7541 Appendix B code
lengths alone, using canonical-code arithmetic (the RFC code is canonical:
codes are assigned in (length, symbol) order -- checked against the
reference's own generator by oracle/pin_reference.py).  This replaces the
reference's generated data file lib/nghttp2_hd_huffman_data.c and its
generator mkhufftbl.py with a different derivation that yields the same
state numbering and transition semantics:

* encode table (ref: huff_sym_table, lib/nghttp2_hd_huffman_data.c:29-94):
  per symbol {MSB-aligned code, nbits}.
* nibble FSM (ref: huff_decode_table, lib/nghttp2_hd_huffman_data.c:96-4980;
  semantics lib/nghttp2_hd_huffman.h:39-52): state = pre-order index of an
  internal node of the code tree (0 = root, 256 = failure sink); for each
  4-bit input the entry holds {next state u16, flags u8, sym u8} packed as
  one little-endian u32: ``fstate | flags << 16 | sym << 24``.
  flags: 0x01 ACCEPTED (state is the root or an all-ones prefix of <= 7
  bits), 0x02 SYM (a symbol completed inside the nibble).  Completing EOS
  (symbol 256) leads to the sink with flags 0.
* canonical decode helpers for the fast kernels: per code length L the first
  code (left-justified to 32 bits) and the symbol index base, plus the
  symbol list sorted in canonical order, and a per-depth map from an internal
  prefix to its FSM state id so a canonical decoder can report the exact
  reference state at the end of a string.

Run: python3 nghttp2_amd/tools/gen_tables.py  (rewrites the .inc file).
"""
import hashlib
import os
import struct
import sys

# RFC 7541 Appendix B: code length of symbols 0..255 and EOS (256).
RFC7541_LEN = [
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28, 28, 28, 28,
    28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28, 6, 10, 10, 12, 13, 6,
    8, 11, 10, 10, 8, 11, 8, 6, 6, 6, 5, 5, 5, 6, 6, 6, 6, 6, 6,
    6, 7, 8, 15, 6, 12, 10, 13, 6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7,
    7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 8, 7, 8, 13, 19, 13, 14,
    6, 15, 5, 6, 5, 6, 5, 6, 6, 6, 5, 7, 7, 6, 6, 6, 5, 6, 7,
    6, 5, 5, 6, 7, 7, 7, 7, 7, 15, 11, 14, 13, 28, 20, 22, 20, 20, 22,
    22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23, 24, 24, 22, 23, 24, 23, 23, 23,
    23, 21, 22, 23, 22, 23, 23, 24, 22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22,
    24, 21, 22, 23, 23, 21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22,
    22, 23, 26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25, 19,
    21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27, 20, 24, 20, 21,
    22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23, 26, 27, 26, 26, 27, 27, 27,
    27, 27, 28, 27, 27, 27, 27, 27, 26, 30]

ACCEPTED = 0x01
SYM = 0x02
LUT_BITS = 14  # the primary lookup (a 13-bit set is generated beside it)
FAIL_STATE = 256
EOS = 256


def canonical_codes():
    """Return (codes, order): codes[s] = (value, length) LSB-aligned."""
    order = sorted(range(257), key=lambda s: (RFC7541_LEN[s], s))
    codes = [None] * 257
    code, prev = 0, RFC7541_LEN[order[0]]
    for s in order:
        L = RFC7541_LEN[s]
        code <<= (L - prev)
        prev = L
        codes[s] = (code, L)
        code += 1
    return codes, order


def build():
    codes, order = canonical_codes()
    leaf = {(v, L): s for s, (v, L) in enumerate(codes)}
    maxlen = max(RFC7541_LEN)
    # A prefix (v, d) is an internal node iff some code longer than d starts
    # with it.  Collect internal prefixes, then number them in pre-order
    # (root, then the 0-subtree, then the 1-subtree).
    internal = set()
    for s, (v, L) in enumerate(codes):
        for d in range(L):
            internal.add((v >> (L - d), d))
    ids = {}

    def preorder(v, d):
        if (v, d) not in internal:
            return
        ids[(v, d)] = len(ids)
        preorder(v << 1, d + 1)
        preorder((v << 1) | 1, d + 1)

    preorder(0, 0)
    assert len(ids) == 256, len(ids)

    def accepts(v, d):
        return d <= 7 and v == (1 << d) - 1

    fsm = [[0] * 16 for _ in range(257)]
    for (v0, d0), sid in ids.items():
        for nib in range(16):
            v, d, sym = v0, d0, None
            failed = False
            for k in range(3, -1, -1):
                v = (v << 1) | ((nib >> k) & 1)
                d += 1
                s = leaf.get((v, d))
                if s is not None:
                    if s == EOS:
                        failed = True
                        # bits after EOS inside the nibble are irrelevant:
                        # the sink absorbs everything.
                        break
                    sym = s
                    v, d = 0, 0
            if failed:
                fsm[sid][nib] = FAIL_STATE
                continue
            flags = 0
            if sym is not None:
                flags |= SYM
            if d == 0:
                nxt = 0
                flags |= ACCEPTED
            else:
                nxt = ids[(v, d)]
                if accepts(v, d):
                    flags |= ACCEPTED
            fsm[sid][nib] = nxt | (flags << 16) | ((sym or 0) << 24)
    for nib in range(16):
        fsm[256][nib] = FAIL_STATE

    enc = []
    for s in range(257):
        v, L = codes[s]
        enc.append(((v << (32 - L)) & 0xFFFFFFFF, L))

    # canonical decode helpers: for each length L in 1..30, the first code of
    # that length left-justified to 32 bits ("limit" style), the count and
    # the index of its first symbol in canonical order.
    count = [0] * (maxlen + 2)
    for s in range(257):
        count[RFC7541_LEN[s]] += 1
    first = [0] * (maxlen + 2)
    base = [0] * (maxlen + 2)
    code = 0
    idx = 0
    for L in range(1, maxlen + 1):
        first[L] = code
        base[L] = idx
        code = (code + count[L]) << 1
        idx += count[L]
    # internal-prefix -> state id, grouped by depth: for depth d the internal
    # prefixes form the contiguous range [lo_d, 2^d) (canonical code property,
    # asserted here).
    depth_lo = [0] * 30
    depth_base = [0] * 30
    id_list = []
    for d in range(30):
        vs = sorted(v for (v, dd) in internal if dd == d)
        assert vs == list(range(vs[0], (1 << d))), d
        depth_lo[d] = vs[0]
        depth_base[d] = len(id_list)
        id_list.extend(ids[(v, d)] for v in vs)
    assert len(id_list) == 256

    # LUT_BITS-bit multi-symbol lookup table for the canonical decoder: for
    # every window, the first code if it is <= LUT_BITS bits (sym1, L1) and,
    # when the rest of the window holds another whole code, the second (sym2).
    # Entry: sym1 | L1 << 8 | cnt << 13 | sym2 << 16 | used << 27, with
    # cnt = symbols in the entry (1 or 2), used = bits they take, and sym2 = 0
    # when cnt = 1: the output bytes are bits 0..7 and 16..23 (a decoder
    # stores the second with no shift, ds_write_b8_d16_hi), and (e >> 10) &
    # 0x18 the output bits.  A zero entry means the first code is longer than
    # LUT_BITS (all such codes start with >= 10 ones).
    lut = []
    for w in range(1 << LUT_BITS):
        def first_code(v, nbits):
            for L in range(1, nbits + 1):
                sym = leaf.get((v >> (nbits - L), L))
                if sym is not None:
                    return sym, L
            return None, 0
        s1, L1 = first_code(w, LUT_BITS)
        e = 0
        if s1 is not None:
            assert s1 != EOS
            r = LUT_BITS - L1
            s2, L2 = first_code(w & ((1 << r) - 1), r) if r else (None, 0)
            e = s1 | (L1 << 8) | (1 << 13) | (L1 << 27)
            if s2 is not None:
                assert L1 + L2 <= LUT_BITS < 32
                e = s1 | (L1 << 8) | (2 << 13) | (s2 << 16) | ((L1 + L2) << 27)
        lut.append(e)
    # second level for codes of LUT_BITS+1..16 bits: every code longer than 12
    # bits starts with 10 ones; indexed by the 6 window bits after them.  Entry
    # as above with cnt 1 (sym | L << 8 | 1 << 13 | L << 27); 0 = longer code.
    lut2 = []
    for v in range(64):
        w16 = (0x3FF << 6) | v
        e = 0
        for L in range(LUT_BITS + 1, 17):
            sym = leaf.get((w16 >> (16 - L), L))
            if sym is not None:
                assert sym != EOS
                e = sym | (L << 8) | (1 << 13) | (L << 27)
                break
        lut2.append(e)
    for code, L in enc:
        if L > LUT_BITS:
            assert code >> 22 == 0x3FF, "long code without 10 leading ones"
    # long codes: (L, left-justified exclusive limit as a 32-bit-window
    # compare, first code, canonical index base) for every length > LUT_BITS
    longc = []
    for L in range(LUT_BITS + 1, maxlen + 1):
        if count[L]:
            lim = (first[L] + count[L]) << (32 - L)
            longc.append((L, lim, first[L], base[L]))
    return dict(enc=enc, fsm=fsm, order=order, count=count, first=first,
                base=base, depth_lo=depth_lo, depth_base=depth_base,
                id_list=id_list, lut=lut, lut2=lut2, longc=longc)


LONG1_N0 = 12    # the fewest leading ones of a code longer than 13 bits
LONG1_ROWS = 20  # n1 = 12 .. 31 (30 and more ones: EOS)


def long_ones_table(t):
    """hd_huff_long1: for n1 = LONG1_N0 .. LONG1_N0 + LONG1_ROWS - 1 leading
    ones, a zero and 5 more bits, the code that bit string starts with, as
    sym | len << 9 (30 or more ones: EOS, len 30).  Built by matching the
    canonical code words as bit strings."""
    words = {}
    codes = canonical_codes()[0]  # (code value, length) per symbol
    for sym, (c, L) in enumerate(codes):
        words[format(c, "0%db" % L)] = (sym, L)
    maxlen = max(L for _, L in codes)
    out = []
    for r in range(LONG1_ROWS):
        n1 = LONG1_N0 + r
        for b in range(32):
            bits = "1" * n1 + "0" + format(b, "05b")
            if n1 >= 30:
                bits = "1" * 30
            hit = None
            for L in range(1, min(len(bits), maxlen) + 1):
                if bits[:L] in words:
                    hit = words[bits[:L]]
                    break
            assert hit is not None and hit[1] >= 14, (n1, b, hit)
            out.append(hit[0] | (hit[1] << 9))
    return out


def packed_ref_layout(t):
    """Bytes of the tables in the reference's struct layouts (for pinning):
    huff_sym_table as {u32 nbits; u32 code}, huff_decode_table as
    {u16 fstate; u8 flags; u8 sym}, both little-endian."""
    sym = b"".join(struct.pack("<II", L, c) for c, L in t["enc"])
    dec = b"".join(struct.pack("<I", e) for row in t["fsm"] for e in row)
    return sym, dec


def write_inc(t, path):
    sym, dec = packed_ref_layout(t)
    lines = []
    w = lines.append
    w("/* GENERATED by nghttp2_amd/tools/gen_tables.py -- do not edit. */")
    w("/* sha256 sym  (ref layout): %s */" % hashlib.sha256(sym).hexdigest())
    w("/* sha256 fsm  (ref layout): %s */" % hashlib.sha256(dec).hexdigest())
    w("#define HD_HUFF_FSM_STATES 257")
    w("#define HD_HUFF_FAIL_STATE 256")
    w("/* encode: MSB-aligned code, code length */")
    w("HD_TBL const unsigned int hd_huff_enc_code[257] = {")
    for i in range(0, 257, 6):
        w("  " + ", ".join("0x%08Xu" % c for c, _ in t["enc"][i:i + 6]) + ",")
    w("};")
    w("HD_TBL const unsigned char hd_huff_enc_len[257] = {")
    for i in range(0, 257, 20):
        w("  " + ", ".join("%d" % L for _, L in t["enc"][i:i + 20]) + ",")
    w("};")
    w("/* nibble FSM: fstate | flags << 16 | sym << 24 */")
    w("HD_TBL const unsigned int hd_huff_fsm[257 * 16] = {")
    for s, row in enumerate(t["fsm"]):
        w("  /* %3d */ " % s + ", ".join("0x%08Xu" % e for e in row) + ",")
    w("};")
    w("/* canonical order of symbols (by length, then value) */")
    w("HD_TBL const unsigned short hd_huff_canon_sym[257] = {")
    for i in range(0, 257, 16):
        w("  " + ", ".join("%d" % s for s in t["order"][i:i + 16]) + ",")
    w("};")
    for name, arr, n in (("hd_huff_first", t["first"], 32),
                         ("hd_huff_base", t["base"], 32),
                         ("hd_huff_count", t["count"], 32)):
        vals = list(arr) + [0] * (n - len(arr))
        w("HD_TBL const unsigned int %s[%d] = {" % (name, n))
        w("  " + ", ".join("%du" % v for v in vals[:n]) + ",")
        w("};")
    w("HD_TBL const unsigned int hd_huff_depth_lo[30] = {")
    w("  " + ", ".join("%du" % v for v in t["depth_lo"]) + ",")
    w("};")
    w("HD_TBL const unsigned short hd_huff_depth_base[30] = {")
    w("  " + ", ".join("%d" % v for v in t["depth_base"]) + ",")
    w("};")
    w("HD_TBL const unsigned char hd_huff_depth_ids[256] = {")
    for i in range(0, 256, 16):
        w("  " + ", ".join("%d" % v for v in t["id_list"][i:i + 16]) + ",")
    w("};")
    w("/* canonical decoder: %d-bit lookup, sym1 | L1 << 8 | cnt << 13 | sym2 << 16 | used << 27 */" % LUT_BITS)
    w("#define HD_HUFF_LUT_BITS %d" % LUT_BITS)
    w("HD_TBL const unsigned int hd_huff_lut[%d] = {" % (1 << LUT_BITS))
    for i in range(0, 1 << LUT_BITS, 8):
        w("  " + ", ".join("0x%08Xu" % e for e in t["lut"][i:i + 8]) + ",")
    w("};")
    w("/* codes longer than the lookup: X(len, limit32 (exclusive, left-justified),"
      " first code, canonical base); limit of the last is 2^32 */")
    w("/* second-level lookup for 13..16-bit codes: window bits 10..15 (after ten ones) */")
    w("HD_TBL const unsigned int hd_huff_lut2[64] = {")
    for i in range(0, 64, 8):
        w("  " + ", ".join("0x%08Xu" % e for e in t["lut2"][i:i + 8]) + ",")
    w("};")
    w("#define HD_HUFF_LONG_CODES(X) \\")
    for L, lim, fc, b in t["longc"]:
        w("  X(%d, 0x%XULL, 0x%Xu, %du) \\" % (L, lim, fc, b))
    w("")
    lo = long_ones_table(t)
    w("/* codes of 14..30 bits by their leading ones (round 5): a window with n1")
    w("   leading ones (n1 >= %d, clamped to %d), then a zero, then bits b (5 of them)" % (LONG1_N0, LONG1_N0 + LONG1_ROWS - 1))
    w("   is the code hd_huff_long1[(n1 - %d) * 32 + b] = sym | len << 9 (every code" % LONG1_N0)
    w("   past 13 bits has n1 >= %d and at most 5 bits after its first zero; 30+" % LONG1_N0)
    w("   ones is EOS) */")
    w("#define HD_HUFF_LONG1_N0 %d" % LONG1_N0)
    w("#define HD_HUFF_LONG1_ROWS %d" % LONG1_ROWS)
    w("HD_TBL const unsigned short hd_huff_long1[%d] = {" % len(lo))
    for i in range(0, len(lo), 16):
        w("  " + ", ".join("0x%04X" % v for v in lo[i:i + 16]) + ",")
    w("};")
    w("")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def write_lut_set(t, bits, path):
    """The decoder tables of a second lookup width (suffix = width), appended."""
    lines = []
    w = lines.append
    w("/* canonical decoder, %d-bit lookup (same entry layout) */" % bits)
    w("HD_TBL const unsigned int hd_huff_lut%d[%d] = {" % (bits, 1 << bits))
    for i in range(0, 1 << bits, 8):
        w("  " + ", ".join("0x%08Xu" % e for e in t["lut"][i:i + 8]) + ",")
    w("};")
    w("HD_TBL const unsigned int hd_huff_lut2_%d[64] = {" % bits)
    for i in range(0, 64, 8):
        w("  " + ", ".join("0x%08Xu" % e for e in t["lut2"][i:i + 8]) + ",")
    w("};")
    w("#define HD_HUFF_LONG_CODES%d(X) \\" % bits)
    for L, lim, fc, b in t["longc"]:
        w("  X(%d, 0x%XULL, 0x%Xu, %du) \\" % (L, lim, fc, b))
    w("")
    with open(path, "a") as f:
        f.write("\n".join(lines) + "\n")


def main():
    global LUT_BITS
    here = os.path.dirname(os.path.abspath(__file__))
    out = os.path.join(here, "..", "csrc", "hd_huff_tables.inc")
    if len(sys.argv) > 1:
        out = sys.argv[1]
    t = build()
    write_inc(t, out)
    primary = LUT_BITS
    LUT_BITS = 13
    write_lut_set(build(), 13, out)
    LUT_BITS = primary
    sym, dec = packed_ref_layout(t)
    print("sym sha256", hashlib.sha256(sym).hexdigest())
    print("fsm sha256", hashlib.sha256(dec).hexdigest())


if __name__ == "__main__":
    main()
