"""The item decoder's long-code search (csrc/hd_huff.hip `long_entry`, tables
staged by `stage_dec_tables`) proven over every window, not sampled.

A code longer than the first-level lookup and the 16-bit second level (RFC
7541 codes of 19..30 bits, /root/reference/lib/nghttp2_hd_huffman_data.c:
29-94) is found by the window's count of leading ones: `long_n1[n1]` gives
the first candidate row, two compares against the left-justified limits pick
the row.  The CPU test restates that pick from the product's own generated
rows (`csrc/hd_huff_tables.inc`, both lookup widths) and checks it against
the canonical code length at every window value where any input of the
pick or of the true length changes (limits, leading-ones thresholds, code
starts, each +-1): the pick and the truth are constant between consecutive
such points, so this covers all 2^32 windows.

The GPU test decodes, through both decode_batch_auto instances, every long
code at eight bit alignments followed by every possible tail of its 32-bit
window, against the oracle (status, context, bytes).
"""
import os
import re

import numpy as np
import pytest

from nghttp2_amd.tools.gen_tables import RFC7541_LEN, canonical_codes

INC = os.path.join(os.path.dirname(__file__), "..", "nghttp2_amd", "csrc", "hd_huff_tables.inc")
NLONG_PAD = 16


def inc_rows(macro):
    """(len, limit, first, base) rows of HD_HUFF_LONG_CODES[13] from the .inc."""
    txt = open(INC).read()
    m = re.search(r"#define %s\(X\) \\\n((?:  X\(.*\) \\\n)+)" % macro, txt)
    assert m, macro
    rows = []
    for a, b, c, d in re.findall(r"X\((\d+), (0x[0-9A-F]+)ULL, (0x[0-9A-F]+)u, (\d+)u\)", m.group(1)):
        rows.append((int(a), int(b, 16), int(c, 16), int(d)))
    return rows


def inc_array(name):
    txt = open(INC).read()
    m = re.search(r"%s\[\d+\] = \{(.*?)\};" % name, txt, re.S)
    assert m, name
    return np.array([int(x, 16) for x in re.findall(r"0x([0-9A-Fa-f]+)u", m.group(1))], dtype=np.uint64)


def staged(rows):
    """stage_dec_tables: limits clamped to 32 bits, padded to NLONG_PAD rows,
    and long_n1[t] = rows below every window with t leading ones."""
    nl = len(rows)
    lim = [min(r[1], 0xFFFFFFFF) for r in rows] + [0xFFFFFFFF] * (NLONG_PAD - nl)
    ln = [r[0] for r in rows] + [rows[-1][0]] * (NLONG_PAD - nl)
    n1 = []
    for t in range(32):
        wmin = (0xFFFFFFFF << (32 - t)) & 0xFFFFFFFF if t else 0
        n1.append(min(sum(1 for r in range(nl) if lim[r] <= wmin), nl - 1))
    return lim, ln, n1, nl


def pick_len(win, lim, ln, n1, nl):
    """long_entry's row pick (hd_huff.hip), restated."""
    inv = ~win & 0xFFFFFFFF
    clz = 32 - inv.bit_length()
    i = n1[min(clz, 31)]
    l0, l1 = lim[i], lim[min(i + 1, NLONG_PAD - 1)]
    i += (1 if l0 <= win else 0) + (1 if l1 <= win else 0)
    return ln[min(i, nl - 1)]


CODES = canonical_codes()[0]  # (code, len) per symbol 0..256


def true_len(win):
    for s, (c, L) in enumerate(CODES):
        if (win >> (32 - L)) == c:
            return L
    raise AssertionError("window %08x starts no code" % win)


@pytest.mark.parametrize("bits", [13, 14])
def test_long_search_exhaustive(bits):
    rows = inc_rows("HD_HUFF_LONG_CODES13" if bits == 13 else "HD_HUFF_LONG_CODES")
    lim, ln, n1, nl = staged(rows)
    lut = inc_array("hd_huff_lut13" if bits == 13 else "hd_huff_lut")
    lut2 = inc_array("hd_huff_lut2_13" if bits == 13 else "hd_huff_lut2")
    assert len(lut) == 1 << bits and len(lut2) == 64
    pts = {0, 0xFFFFFFFF}
    pts.update(lim[:nl])
    pts.update(((0xFFFFFFFF << (32 - t)) & 0xFFFFFFFF) for t in range(1, 33))
    for c, L in CODES:
        pts.add(c << (32 - L))
        pts.add(((c + 1) << (32 - L)) - 1)
    pts = sorted({min(max(p + d, 0), 0xFFFFFFFF) for p in pts for d in (-1, 0, 1)})
    checked = 0
    for w in pts:
        # slow_entry reaches long_entry only when both lookup levels miss
        if lut[w >> (32 - bits)] != 0 or lut2[(w >> 16) & 63] != 0:
            continue
        assert pick_len(w, lim, ln, n1, nl) == true_len(w), "window %08x" % w
        checked += 1
    # every code past 16 bits has its start among the checked windows
    starts = {c << (32 - L) for c, L in CODES if L > 16}
    assert starts <= set(pts)
    assert checked >= len(starts)


def test_long_search_three_candidates():
    """The invariant the search rests on: windows with t leading ones (t <
    32) start codes of at most three distinct lengths past 16 bits."""
    for t in range(32):
        lens = set()
        for c, L in CODES:
            if L <= 16:
                continue
            v = c << (32 - L)
            lo = (0xFFFFFFFF << (32 - t)) & 0xFFFFFFFF if t else 0  # t ones, then a zero
            hi = lo | ((1 << (31 - t)) - 1) if t < 32 else 0xFFFFFFFF
            last = v | ((1 << (32 - L)) - 1)
            if last >= lo and v <= hi:
                lens.add(L)
        assert len(lens) <= 3, (t, sorted(lens))


def long_code_batch():
    """Every code past 16 bits, after 0..7 five-bit codes (00000, symbol
    '0': eight bit alignments) and followed by every (32 - L)-bit tail of its
    window, then 64 bits of 5-bit codes and one-bit padding."""
    strs = []
    fill = 0
    for _ in range(12):
        fill = (fill << 5) | 0b00011  # 'a'
    for s, (c, L) in enumerate(CODES):
        if L <= 16:
            continue
        tl = 32 - L
        for k in range(8):
            for tail in range(1 << tl):
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
    nlong = sum(1 for _, L in CODES if L > 16)
    assert n == 8 * sum(1 << (32 - L) for _, L in CODES if L > 16)
    assert nlong == sum(1 for x in RFC7541_LEN if x > 16)


@pytest.mark.gpu
@pytest.mark.parametrize("pick", ["items64", "pieces40"])
def test_long_codes_all_tails_gpu(codec, dev, pick):
    from tests.test_parity_gpu import auto_decode_check
    enc, eoff = long_code_batch()
    st, _ = auto_decode_check(codec, dev, enc, eoff, "long codes " + pick, pick=pick, nthreads=8)
    assert (st >= 0).any() and (st < 0).any()
