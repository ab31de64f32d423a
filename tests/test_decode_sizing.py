"""Host-side checks of the item decoder's LDS sizing (csrc/hd_huff.hip,
di_rb / di_obb / di_ibw / di_span, restated here): a round's output regions
never pass the output buffer, and its staged input never passes the staging
buffer, for plain rounds (64 items of at most P bytes) and budgeted rounds
(as many of the next 64 items as fit BI bytes).  The kernel relies on these
bounds without a runtime check; the decode bound itself is the reference's
(lib/nghttp2_hd.c:2082, floor(8 E / 5) symbols plus the item's 29-bit stop
overshoot)."""
import numpy as np

WAVE = 64
DD_OV = 20


def di_rb(ip):  # a lane's output region for ip input bytes (dword aligned)
    return (((8 * ip + 29) // 5) + 2 + 3) & ~3


def di_span(ip, bi):
    return bi if bi else WAVE * ip


def di_obb(ip, bi):
    return ((8 * bi) // 5 + 692 + 15) & ~15 if bi else WAVE * di_rb(ip)


def di_ibw(span):  # staged dwords
    return (((span + DD_OV + 64) // 4 + 8) + 3) & ~3


INSTANCES = [(64, 0), (40, 0), (32, 0), (64, 2048), (64, 2304), (96, 2304), (128, 2304), (32, 1280)]


def _rounds(sizes, ip, bi):
    """Split a task's item sizes into rounds as the kernel does."""
    i = 0
    while i < len(sizes):
        cand = sizes[i:i + WAVE]
        if bi:
            c = np.cumsum(cand)
            nv = int((c <= bi).sum())
        else:
            nv = len(cand)
        assert nv >= 1
        yield cand[:nv]
        i += nv


def test_output_regions_fit():
    rng = np.random.default_rng(5)
    for ip, bi in INSTANCES:
        for trial in range(400):
            # item sizes: full pieces, short last pieces, empty strings
            sizes = rng.integers(0, ip + 1, size=int(rng.integers(1, 300)))
            if trial % 4 == 0:
                sizes[:] = ip  # every item full: the worst case
            for r in _rounds(list(sizes), ip, bi):
                regions = [di_rb(int(x)) if bi else di_rb(ip) for x in r]
                assert sum(regions) <= di_obb(ip, bi), (ip, bi, r)
                # the byte sink writes up to two bytes past its count: inside
                # the item's own region
                for x in r:
                    nsym_max = (8 * int(x) + 29) // 5
                    assert nsym_max + 2 <= (di_rb(int(x)) if bi else di_rb(ip))


def test_staged_input_fits():
    for ip, bi in INSTANCES:
        span = di_span(ip, bi)
        # staged range [R0 - OV, min(R0 + span, Z) + 8), 16-byte aligned at
        # both ends, written at dword 4 onwards
        worst = (span + DD_OV + 8 + 15 + 15) // 16 * 16
        assert 16 + worst <= 4 * di_ibw(span), (ip, bi)
