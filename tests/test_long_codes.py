"""The item decoder's long-code path (csrc/hd_huff.hip `long_entry`, the
table staged by `stage_dec_tables`) proven over every window, not sampled.

A code longer than the first-level lookup (RFC 7541 codes of 14..30 bits,
/root/reference/lib/nghttp2_hd_huffman_data.c:29-94) is named by the
window's count of leading ones n1 (>= 12) and the 5 bits after the first
zero: one read of `hd_huff_long1[(n1 - 12) * 32 + b]` (round 5; it replaced
a second-level lookup plus a search over left-justified limits).  Every
window with the same n1 and the same 5 bits reads the same entry, and --
since every HPACK code past 13 bits ends within 5 bits of its first zero --
starts the same code, so checking one window per (n1, b) class, at both ends
of the class, covers all 2^32 windows.  The CPU test does that against the
canonical code for both lookup widths, from the product's own generated
tables (`csrc/hd_huff_tables.inc`).

The GPU test decodes, through both decode_batch_auto instances, every code
past 13 bits at eight bit alignments, each followed by tails of its 32-bit
window (every tail for codes past 16 bits, a sample for 14..16), against the
oracle (status, context, bytes).
"""
import os
import re

import numpy as np
import pytest

from nghttp2_amd.tools.gen_tables import RFC7541_LEN, canonical_codes

INC = os.path.join(os.path.dirname(__file__), "..", "nghttp2_amd", "csrc", "hd_huff_tables.inc")


def inc_array(name, suffix="u"):
    txt = open(INC).read()
    m = re.search(r"%s\[\d+\] = \{(.*?)\};" % name, txt, re.S)
    assert m, name
    return np.array([int(x, 16) for x in re.findall(r"0x([0-9A-Fa-f]+)" + suffix, m.group(1))],
                    dtype=np.uint64)


def inc_define(name):
    m = re.search(r"#define %s (\d+)" % name, open(INC).read())
    assert m, name
    return int(m.group(1))


CODES = canonical_codes()[0]  # (code, len) per symbol 0..256


def true_code(win):
    for s, (c, L) in enumerate(CODES):
        if (win >> (32 - L)) == c:
            return s, L
    raise AssertionError("window %08x starts no code" % win)


def long_entry(win, long1, n0, rows):
    """hd_huff.hip long_entry's table read, restated: (sym, len)."""
    inv = ~win & 0xFFFFFFFF
    clz = 32 - inv.bit_length()
    n1 = min(max(clz, n0), n0 + rows - 1)
    b = ((win << (n1 + 1)) & 0xFFFFFFFF) >> 27
    v = int(long1[(n1 - n0) * 32 + b])
    return v & 511, v >> 9


@pytest.mark.parametrize("bits", [13, 14])
def test_long_table_exhaustive(bits):
    long1 = inc_array("hd_huff_long1", "")
    n0, rows = inc_define("HD_HUFF_LONG1_N0"), inc_define("HD_HUFF_LONG1_ROWS")
    assert len(long1) == 32 * rows
    lut = inc_array("hd_huff_lut13" if bits == 13 else "hd_huff_lut")
    assert len(lut) == 1 << bits
    checked, seen = 0, set()
    for n1 in range(33):
        for b in range(32):
            if n1 >= 32:
                lo = hi = 0xFFFFFFFF
            else:
                head = ((0xFFFFFFFF << (32 - n1)) & 0xFFFFFFFF) if n1 else 0
                rest = 31 - n1  # bits after the first zero
                if rest >= 5:
                    lo = head | (b << (rest - 5))
                    hi = lo | ((1 << (rest - 5)) - 1)
                else:  # fewer than 5 bits remain: b's top bits only
                    if b & ((1 << (5 - rest)) - 1):
                        continue
                    lo = hi = head | (b >> (5 - rest))
            for w in (lo, hi):
                if lut[w >> (32 - bits)] != 0:  # a first-level hit: no table read
                    continue
                sym, L = long_entry(w, long1, n0, rows)
                if n1 >= 30:
                    assert (sym, L) == (256, 30), "window %08x" % w
                else:
                    assert (sym, L) == true_code(w), "window %08x" % w
                seen.add(sym)
                checked += 1
    # every code past the lookup was met
    assert {s for s, (c, L) in enumerate(CODES) if L > bits} <= seen
    assert checked > 0


def test_long_table_shape():
    """The invariant the table rests on: every code past 13 bits has at
    least 12 leading ones and at most 5 bits after its first zero."""
    for c, L in CODES:
        if L <= 13:
            continue
        s = format(c, "0%db" % L)
        n1 = len(s) - len(s.lstrip("1"))
        assert n1 >= 12 and L - n1 - 1 <= 5, (c, L)


def long_code_batch():
    """Every code past 13 bits, after 0..7 five-bit codes (00000, symbol
    '0': eight bit alignments) and followed by every (32 - L)-bit tail of its
    window, then 64 bits of 5-bit codes and one-bit padding."""
    strs = []
    fill = 0
    for _ in range(12):
        fill = (fill << 5) | 0b00011  # 'a'
    rng = np.random.default_rng(0x10C0DE)
    for s, (c, L) in enumerate(CODES):
        if L <= 13:
            continue
        tl = 32 - L
        # every tail past 16 bits; 14..16 bits: the 64 tails of its first six
        # bits (each with random low bits) and the extremes
        tails = (range(1 << tl) if L > 16 else
                 sorted({0, (1 << tl) - 1} | {(t << (tl - 6)) | int(rng.integers(0, 1 << (tl - 6)))
                                              for t in range(64)}))
        for k in range(8):
            for tail in tails:
                v = c
                nb = 5 * k + L
                v = (v << tl) | tail
                nb += tl
                v = (v << 60) | fill
                nb += 60
                pad = (-nb) % 8
                v = (v << pad) | ((1 << pad) - 1)
                nb += pad
                strs.append(v.to_bytes(nb // 8, "big"))
    off = np.zeros(len(strs) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(x) for x in strs])
    return np.frombuffer(b"".join(strs), dtype=np.uint8).copy(), off


def test_long_code_batch_shape():
    enc, off = long_code_batch()
    n = len(off) - 1
    n16 = sum(1 for _, L in CODES if 13 < L <= 16)
    assert n == 8 * sum(1 << (32 - L) for _, L in CODES if L > 16) + 8 * 66 * n16
    assert sum(1 for _, L in CODES if L > 13) == sum(1 for x in RFC7541_LEN if x > 13)


@pytest.mark.gpu
@pytest.mark.parametrize("pick", ["items64", "pieces40"])
def test_long_codes_all_tails_gpu(codec, dev, pick):
    from tests.test_parity_gpu import auto_decode_check
    enc, eoff = long_code_batch()
    st, _ = auto_decode_check(codec, dev, enc, eoff, "long codes " + pick, pick=pick, nthreads=8)
    assert (st >= 0).any() and (st < 0).any()
