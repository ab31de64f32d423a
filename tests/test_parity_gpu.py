"""GPU parity: the HIP engine (through the C ABI) vs the oracle, bit-exact.

Encode: encoded offsets (== nghttp2_hd_huff_encode_count per string) and
every encoded byte.  Decode: per-string status (length / -523 / -502), final
decode context {fstate, flags}, and the whole zero-initialised output slot
pool (decoded bytes plus the bytes a failing string leaves behind, exactly as
lib/nghttp2_hd_huffman.c:122-133 writes them).
"""
import hashlib

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden import make_golden

pytestmark = pytest.mark.gpu


def to_dev(a, dev, dtype=None):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).to(dev)


def pad16(pool, used):
    out = np.zeros(int(used) + (-int(used)) % 16 + 16, dtype=np.uint8)
    out[:int(used)] = pool[:int(used)]
    return out


def gpu_encode(codec, dev, pool, off):
    src = to_dev(pad16(pool, off[-1]), dev)
    enc, enc_off = codec.encode(src, to_dev(off, dev), raw_bytes=int(off[-1]))
    eo = enc_off.cpu().numpy().view(np.uint32).copy()
    return enc.cpu().numpy()[:int(eo[-1])], eo


def gpu_decode(codec, dev, enc, eoff):
    import torch
    src = to_dev(pad16(enc, eoff[-1]), dev)
    so = to_dev(eoff, dev)
    dst_off = codec.decode_slots(so)
    cap = int(dst_off[-1].item())
    dst = torch.zeros(cap + 16, dtype=torch.uint8, device=dev)
    dst, dst_off, st, fs, fl = codec.decode(src, so, dst_off=dst_off, dst=dst, want_ctx=True)
    torch.cuda.synchronize()
    return (dst.cpu().numpy()[:cap], dst_off.cpu().numpy().view(np.uint32),
            st.cpu().numpy(), fs.cpu().numpy().view(np.uint16), fl.cpu().numpy())


def check_decode(codec, dev, enc, eoff, tag):
    d, do, st, fs, fl = gpu_decode(codec, dev, enc, eoff)
    rd, rdo, rst, rfs, rfl = O.decode_batch(enc, eoff)
    assert np.array_equal(do, rdo), tag + ": slots"
    bad = np.nonzero(st != rst)[0]
    assert bad.size == 0, "%s: status differs at %s (gpu %s, ref %s)" % (
        tag, bad[:5], st[bad[:5]], rst[bad[:5]])
    assert np.array_equal(fs, rfs), tag + ": fstate"
    assert np.array_equal(fl, rfl), tag + ": flags"
    if not np.array_equal(d, rd[:len(d)]):
        i = int(np.nonzero(d != rd[:len(d)])[0][0])
        s = int(np.searchsorted(do, i, side="right") - 1)
        raise AssertionError("%s: output differs at byte %d (string %d)" % (tag, i, s))
    return st


def check_roundtrip(codec, dev, pool, off, tag):
    enc, eoff = gpu_encode(codec, dev, pool, off)
    renc, reoff = O.encode_batch(pool, off)
    assert np.array_equal(eoff, reoff), tag + ": encoded offsets"
    if not np.array_equal(enc, renc):
        i = int(np.nonzero(enc != renc)[0][0])
        raise AssertionError("%s: encoded byte %d differs" % (tag, i))
    st = check_decode(codec, dev, enc, eoff, tag)
    assert np.array_equal(st, np.diff(off.astype(np.int64))), tag + ": round trip lengths"


@pytest.mark.parametrize("name", make_golden.CASES)
def test_golden(codec, dev, name):
    g = make_golden.load(name)
    if g["kind"] == "roundtrip":
        enc, eoff = gpu_encode(codec, dev, g["raw"], g["raw_off"])
        assert np.array_equal(eoff, g["enc_off"])
        assert np.array_equal(enc, g["enc"][:int(eoff[-1])])
    enc, eoff = g["enc"], g["enc_off"]
    d, do, st, fs, fl = gpu_decode(codec, dev, enc, eoff)
    assert np.array_equal(st, g["status"])
    assert np.array_equal(fs, g["fstate"])
    assert np.array_equal(fl, g["flags"])
    assert hashlib.sha256(make_golden.decoded_bytes(d, do, st)).hexdigest() == g["dec_sha256"]


def test_known_answers(codec, dev):
    import json, os
    ka = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
    vecs = [v for v in ka["ref_unit_decode"] if v["final"]]
    strs = [bytes.fromhex(v["src"]) for v in vecs]
    strs += [bytes.fromhex(h) for _, h in ka["rfc7541"]]
    lens = np.array([len(s) for s in strs], dtype=np.int64)
    from nghttp2_amd import workloads as W
    pool, off = W._pool_from_lengths(lens, np.frombuffer(b"".join(strs), np.uint8))
    d, do, st, fs, fl = gpu_decode(codec, dev, pool, off)
    for i, v in enumerate(vecs):
        exp = v["rv"] if v["rv"] < 0 else len(bytes.fromhex(v.get("out", "")))
        assert st[i] == exp, v
        if "failure_state" in v:
            assert (fs[i] == 0x100) == v["failure_state"], v
    for j, (s, h) in enumerate(ka["rfc7541"]):
        i = len(vecs) + j
        assert st[i] == len(s)
        assert bytes(d[do[i]:do[i] + len(s)]) == s.encode()
    raw = [s.encode() for s, _ in ka["rfc7541"]]
    lens = np.array([len(s) for s in raw], dtype=np.int64)
    pool, off = W._pool_from_lengths(lens, np.frombuffer(b"".join(raw), np.uint8))
    enc, eoff = gpu_encode(codec, dev, pool, off)
    for j, (s, h) in enumerate(ka["rfc7541"]):
        assert bytes(enc[eoff[j]:eoff[j + 1]]).hex() == h


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 4095, 4096, 4097, 20000])
def test_batch_sizes(codec, dev, n):
    from nghttp2_amd import workloads as W
    pool, off = W.gen_pseudo_headers(n, seed=100 + n)
    check_roundtrip(codec, dev, pool, off, "pseudo n=%d" % n)


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 200, 255, 256, 257, 300])
def test_single_tile_one_launch(codec, dev, n):
    """A batch of at most 256 strings (one tile) is counted and packed in one
    launch (k_encode<FR, ONE>): encode and string literals on both sides of
    the threshold, with empty strings, every byte value (codes to 30 bits),
    long strings and multi-byte literal lengths among them."""
    rng = np.random.Generator(np.random.PCG64(0x1E + n))
    strs = [b"", bytes(range(256)), b"\xff" * 127, b"a" * 128, b"0" * 16600]
    strs += [bytes(rng.integers(0, 256, size=int(k), dtype=np.uint8))
             for k in rng.integers(0, 300, size=max(0, n - len(strs)))]
    strs = strs[:n]
    off = np.zeros(len(strs) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(x) for x in strs])
    pool = np.frombuffer(b"".join(strs), dtype=np.uint8)
    check_roundtrip(codec, dev, pool, off, "one tile n=%d" % n)
    check_emit(codec, dev, pool, off, "one tile n=%d" % n)


def test_all_byte_values(codec, dev):
    from nghttp2_amd import workloads as W
    pool, off = W.gen_all_bytes(30000, seed=5)
    check_roundtrip(codec, dev, pool, off, "allbytes")


def test_empty_and_ragged(codec, dev):
    from nghttp2_amd import workloads as W
    rng = np.random.default_rng(9)
    lens = rng.choice([0, 0, 1, 2, 3, 15, 16, 17, 31, 33, 300], size=9000)
    chars = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8)
    pool, off = W._pool_from_lengths(lens, chars)
    check_roundtrip(codec, dev, pool, off, "ragged")
    lens = np.zeros(5000, dtype=np.int64)
    pool, off = W._pool_from_lengths(lens, np.zeros(0, np.uint8))
    check_roundtrip(codec, dev, pool, off, "all-empty")


def test_max_length_strings(codec, dev):
    # NGHTTP2_HD_MAX_NV (lib/nghttp2_hd.h:45) sized literals
    from nghttp2_amd import workloads as W
    rng = np.random.default_rng(12)
    lens = np.array([65536, 1, 65536, 70000, 0, 65535], dtype=np.int64)
    chars = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8)
    pool, off = W._pool_from_lengths(lens, chars)
    check_roundtrip(codec, dev, pool, off, "max-len")


def test_adversarial_decode(codec, dev):
    from nghttp2_amd import workloads as W
    pool, off, cats = W.gen_adversarial(50000, seed=77)
    st = check_decode(codec, dev, pool, off, "adversarial")
    # every malformed category produces errors somewhere
    for c in (1, 2, 4):
        assert (st[cats == c] < 0).any()


def test_random_garbage_decode(codec, dev):
    from nghttp2_amd import workloads as W
    pool, off = W.gen_all_bytes(40000, seed=21, lo=0, hi=48)
    check_decode(codec, dev, pool, off, "garbage")


def test_small_slots_buffer_error(codec, dev):
    """Caller-provided slots smaller than the decoded length -> -502, no
    write outside the slot."""
    import torch
    from nghttp2_amd import workloads as W
    pool, off = W.gen_pseudo_headers(2000, seed=3)
    enc, eoff = O.encode_batch(pool, off)
    raw = np.diff(off.astype(np.int64))
    cap = raw.copy()
    cap[::3] -= 1
    cap = np.maximum(cap, 0)
    doff = np.zeros(len(off), dtype=np.uint32)
    doff[1:] = np.cumsum(cap)
    src = to_dev(pad16(enc, eoff[-1]), dev)
    dst = torch.full((int(doff[-1]) + 16,), 0xAB, dtype=torch.uint8, device=dev)
    _, _, st = codec.decode(src, to_dev(eoff, dev), dst_off=to_dev(doff, dev), dst=dst)
    st = st.cpu().numpy()
    exp = np.where(cap < raw, O.NGHTTP2_ERR_BUFFER_ERROR, raw)
    assert np.array_equal(st, exp)
    d = dst.cpu().numpy()
    assert (d[int(doff[-1]):] == 0xAB).all()
    for i in range(0, 2000, 7):
        k = min(cap[i], raw[i])
        assert bytes(d[doff[i]:doff[i] + k]) == bytes(pool[off[i]:off[i] + k])


@pytest.mark.parametrize("cfg", [2, 3])
def test_full_size_config_roundtrip(codec, dev, cfg):
    """BASELINE.json configs 2/3 at full size (1M strings): bit-exact vs the
    oracle (multi-threaded) and decode(encode(x)) == x."""
    from nghttp2_amd import workloads as W
    n = 1 << 20
    pool, off = W.gen_pseudo_headers(n) if cfg == 2 else W.gen_mixed_values(n)
    enc, eoff = gpu_encode(codec, dev, pool, off)
    renc, reoff = O.encode_batch(pool, off, nthreads=16)
    assert np.array_equal(eoff, reoff)
    assert hashlib.sha256(enc.tobytes()).digest() == hashlib.sha256(renc.tobytes()).digest()
    d, do, st, fs, fl = gpu_decode(codec, dev, enc, eoff)
    raw = np.diff(off.astype(np.int64))
    assert np.array_equal(st, raw)
    assert (fl & 1).all()
    # checksum of checksums: every string's bytes land in its slot
    idx = np.repeat(do[:-1].astype(np.int64), raw) + (np.arange(int(raw.sum()))
                                                      - np.repeat(off[:-1].astype(np.int64), raw))
    assert np.array_equal(d[idx], pool[:int(off[-1])])


def check_dense_layout(d, do, enc, eoff, tag):
    """decode_batch_auto's layout: the strings of a task (64 consecutive
    strings, or a split task of 32) back to back from the task's base
    auto_slot(x_t0, t0); string
    i's bytes -- every byte the reference writes, the partial output of a
    failing string included (lib/nghttp2_hd_huffman.c:122-133) -- at
    dst[dst_off[i]:]."""
    n = len(eoff) - 1
    eo = eoff.astype(np.int64)
    g = (8 * (eo - eo[0])) // 5
    base = 4 * ((g + 3) // 4 + np.arange(n + 1))
    for i in range(n):
        _, out, _ = O.decode(bytes(enc[eo[i]:eo[i + 1]]), final=1)
        w = len(out)
        if i % 64 == 0:
            assert do[i] == base[i], (tag, i)
        if i + 1 < n and (i + 1) % 32:
            assert do[i + 1] == do[i] + w, (tag, i, "not dense")
        elif i + 1 < n and (i + 1) % 64:  # a task of 64, or the second of a split one
            assert do[i + 1] in (do[i] + w, base[i + 1]), (tag, i, "not dense / no base")
        elif i + 1 == n:
            assert do[n] == do[i] + w, (tag, "end")
        assert bytes(d[do[i]:do[i] + w]) == out, (tag, i)


def _variant_inputs():
    from nghttp2_amd import workloads as W
    pool, off, _ = W.gen_adversarial(20000, seed=31)
    yield "adversarial", pool, off
    p2, o2 = W.gen_all_bytes(20000, seed=32, lo=0, hi=40)
    yield "garbage", p2, o2
    p3, o3 = W.gen_mixed_values(3000, seed=33)
    e3, eo3 = O.encode_batch(p3, o3)
    yield "mixed", e3, eo3


@pytest.mark.parametrize("variant", ["auto", "items64", "pieces40", "fsm"])
def test_decode_variants_match_oracle(codec, dev, variant):
    """decode_batch_auto (dense item decoder: the library's pick and both
    instances) and the batched reference FSM kernel agree with the oracle on
    status, final context and every written byte."""
    import torch
    for tag, enc, eoff in _variant_inputs():
        rd, rdo, rst, rfs, rfl = O.decode_batch(enc, eoff)
        src = to_dev(pad16(enc, eoff[-1]), dev)
        so = to_dev(eoff, dev)
        n = len(eoff) - 1
        if variant != "fsm":
            cap = codec.decode_bound(int(eoff[-1]), n)
            dst = torch.zeros(cap, dtype=torch.uint8, device=dev)
            pick = None if variant == "auto" else variant
            dst, do, st, fs, fl = codec.decode_auto(src, so, enc_bytes=int(eoff[-1]), dst=dst,
                                                    want_ctx=True, pick=pick)
            do = do.cpu().numpy().view(np.uint32)
            check_dense_layout(dst.cpu().numpy(), do, enc, eoff, tag)
        else:
            do_t = to_dev(rdo, dev)
            dst = torch.zeros(int(rdo[-1]) + 16, dtype=torch.uint8, device=dev)
            st, fs, fl = codec.decode_fsm(src, so, do_t, dst)
            do = rdo
        torch.cuda.synchronize()
        st = st.cpu().numpy()
        assert np.array_equal(st, rst), tag
        assert np.array_equal(fs.cpu().numpy().view(np.uint16), rfs), tag
        assert np.array_equal(fl.cpu().numpy(), rfl), tag
        d = dst.cpu().numpy()
        written = np.where(rst >= 0, rst, 0)
        for i in range(n):
            # compare every byte the oracle wrote (also on failure: the
            # oracle's slot pool is zero-initialised like ours)
            k = int(rdo[i + 1] - rdo[i]) if variant == "fsm" else int(written[i])
            assert bytes(d[do[i]:do[i] + k]) == bytes(rd[rdo[i]:rdo[i] + k]), (tag, i)


def test_fsm_streaming_chunks(codec, dev):
    """Chunked decode through the batched FSM kernel, carrying the decode
    context between calls (fin=0 then fin=1), equals whole-string decode --
    the streaming contract of tests/nghttp2_test_helper.c:165-205."""
    import torch
    from nghttp2_amd import workloads as W
    pool, off, _ = W.gen_adversarial(6000, seed=41)
    n = len(off) - 1
    lens = np.diff(off.astype(np.int64))
    rng = np.random.default_rng(2)
    cut = (rng.random(n) * (lens + 1)).astype(np.int64)
    rd, rdo, rst, rfs, rfl = O.decode_batch(pool, off)
    outs = []
    state = flags = None
    for part in range(2):
        lo = np.where(part == 0, 0, cut)
        hi = np.where(part == 0, cut, lens)
        plen = hi - lo
        chunks = np.concatenate([pool[off[i] + lo[i]: off[i] + hi[i]] for i in range(n)]) \
            if plen.sum() else np.zeros(0, np.uint8)
        cpool, coff = W._pool_from_lengths(plen, chunks)
        slots = np.zeros(n + 1, dtype=np.int64)
        slots[1:] = np.cumsum(plen * 8 // 5 + 1)
        dst = torch.zeros(int(slots[-1]) + 16, dtype=torch.uint8, device=dev)
        st, fs, fl = codec.decode_fsm(to_dev(cpool, dev), to_dev(coff, dev),
                                      to_dev(slots.astype(np.uint32), dev), dst,
                                      init_fstate=state, init_flags=flags, final=(part == 1))
        torch.cuda.synchronize()
        d = dst.cpu().numpy()
        stn = st.cpu().numpy()
        outs.append([bytes(d[slots[i]:slots[i] + max(0, stn[i])]) if part == 0 or stn[i] >= 0
                     else None for i in range(n)])
        state, flags = fs, fl
    assert np.array_equal(fs.cpu().numpy().view(np.uint16), rfs)
    assert np.array_equal(fl.cpu().numpy(), rfl)
    assert np.array_equal(np.where(stn < 0, stn, 0), np.where(rst < 0, rst, 0))
    for i in range(n):
        if rst[i] >= 0:
            assert outs[0][i] + outs[1][i] == bytes(rd[rdo[i]:rdo[i] + rst[i]]), i


# ---- HPACK string literals (emit_string) ----
def gpu_emit(codec, dev, pool, off):
    src = to_dev(pad16(pool, off[-1]), dev)
    dst, dst_off = codec.emit_strings(src, to_dev(off, dev), raw_bytes=int(off[-1]))
    do = dst_off.cpu().numpy().view(np.uint32).copy()
    return dst.cpu().numpy()[:int(do[-1])], do


def check_emit(codec, dev, pool, off, tag):
    d, do = gpu_emit(codec, dev, pool, off)
    rd, rdo = O.emit_strings_batch(pool, off)
    assert np.array_equal(do, rdo), tag + ": literal offsets"
    if not np.array_equal(d, rd):
        i = int(np.nonzero(d != rd)[0][0])
        s = int(np.searchsorted(do, i, side="right") - 1)
        raise AssertionError("%s: literal byte %d differs (string %d)" % (tag, i, s))


def test_emit_strings_rfc7541(codec, dev):
    import json, os
    ka = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
    vecs = ka["rfc7541_string_literals"]["vectors"]
    strs = [v[0].encode() for v in vecs]
    off = np.zeros(len(strs) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(s) for s in strs])
    pool = np.frombuffer(b"".join(strs), dtype=np.uint8)
    d, do = gpu_emit(codec, dev, pool, off)
    for i, v in enumerate(vecs):
        assert bytes(d[do[i]:do[i + 1]]).hex() == v[1], v[2]


@pytest.mark.parametrize("kind", ["pseudo", "mixed", "allbytes", "edge"])
def test_emit_strings_parity(codec, dev, kind):
    from nghttp2_amd import workloads as W
    if kind == "pseudo":
        pool, off = W.gen_pseudo_headers(20000)
    elif kind == "mixed":
        pool, off = W.gen_mixed_values(3000)
    elif kind == "allbytes":
        pool, off = W.gen_all_bytes(3000)
    else:
        # empty strings, raw-vs-Huffman choices and multi-byte length prefixes
        rng = np.random.Generator(np.random.PCG64(0xE1))
        strs = [b"", b"a", b"", bytes(range(256)), b"\xff" * 126, b"\xff" * 127,
                b"\xff" * 128, b"a" * 126, b"a" * 127, b"a" * 160, b"a" * 254, b"a" * 255,
                b"0" * (16383 + 127), b"0" * (16384 + 127), b"", b"\x00" * 300]
        strs += [bytes(rng.integers(0, 256, size=int(k), dtype=np.uint8))
                 for k in rng.integers(0, 400, size=500)]
        off = np.zeros(len(strs) + 1, dtype=np.uint32)
        off[1:] = np.cumsum([len(s) for s in strs])
        pool = np.frombuffer(b"".join(strs), dtype=np.uint8)
    check_emit(codec, dev, pool, off, kind)


@pytest.mark.parametrize("pick", [None, "items64", "pieces40"])
def test_dense_decode_edges(codec, dev, pick):
    """decode_batch_auto (each item-decoder instance) on strings that stress
    its pieces:
    ends on and near piece and round boundaries, runs of empty strings (also
    at a task's end and whole empty tasks), strings longer than a round,
    random bytes (EOS, bad padding) -- every written byte, status and final
    context against the oracle."""
    import torch
    from nghttp2_amd import workloads as W
    rng = np.random.default_rng(0xDD)
    parts = []
    # encoded strings of chosen lengths (random symbols, valid padding)
    for L in list(range(0, 70)) + [127, 128, 129, 2047, 2048, 2049, 4100, 9000]:
        parts.append(bytes(rng.integers(0x20, 0x7F, size=max(0, L * 5 // 4), dtype=np.uint8)))
    raw = parts + [b""] * 70 + [bytes(rng.integers(0, 256, size=int(k), dtype=np.uint8))
                               for k in rng.integers(0, 90, size=600)]
    raw += [b""] * 130  # whole empty tasks and empty strings at the end
    rng.shuffle(raw[:-130])
    lens = np.array([len(x) for x in raw], dtype=np.int64)
    pool, off = W._pool_from_lengths(lens, np.frombuffer(b"".join(raw), np.uint8))
    enc, eoff = O.encode_batch(pool, off)
    garbage, goff = W.gen_all_bytes(3000, seed=77, lo=0, hi=100)
    for tag, e, eo in (("encoded", enc, eoff), ("garbage", garbage[:int(goff[-1])], goff)):
        rd, rdo, rst, rfs, rfl = O.decode_batch(e, eo)
        n = len(eo) - 1
        src = to_dev(pad16(e, eo[-1]), dev)
        dst = torch.zeros(codec.decode_bound(int(eo[-1]), n), dtype=torch.uint8, device=dev)
        dst, do, st, fs, fl = codec.decode_auto(src, to_dev(eo, dev), enc_bytes=int(eo[-1]),
                                                dst=dst, want_ctx=True, pick=pick)
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), rst), tag
        assert np.array_equal(fs.cpu().numpy().view(np.uint16), rfs), tag
        assert np.array_equal(fl.cpu().numpy(), rfl), tag
        check_dense_layout(dst.cpu().numpy(), do.cpu().numpy().view(np.uint32), e, eo, tag)


def test_decode_descending_offsets_refused(codec, dev):
    """Offsets out of order (a caller error) end in INVALID_ARGUMENT for the
    strings of the task that holds them, not in an endless item walk; the
    other tasks decode normally."""
    import torch
    from nghttp2_amd import workloads as W
    pool, off = W.gen_pseudo_headers(256, seed=5)
    enc, eoff = O.encode_batch(pool, off)
    bad = eoff.copy()
    bad[70] = bad[72]  # string 70 ends before it starts (task 1: strings 64..127)
    src = to_dev(pad16(enc, eoff[-1]), dev)
    dst = torch.zeros(codec.decode_bound(int(eoff[-1]), 256) + 4096, dtype=torch.uint8, device=dev)
    dst, do, st = codec.decode_auto(src, to_dev(bad, dev), dst=dst)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert (st[64:128] == -501).all()
    rst = O.decode_batch(enc, eoff)[2]
    assert np.array_equal(st[:64], rst[:64]) and np.array_equal(st[128:], rst[128:])


# ---- decode_batch_auto (the bench-timed path) under the same parity bar ----
def auto_decode_check(codec, dev, enc, eoff, tag, pick=None, nthreads=1):
    """decode_auto vs the oracle: status, {fstate, flags}, and every byte the
    reference writes for each string (its partial output on failure too),
    gathered from the dense layout."""
    import torch
    n = len(eoff) - 1
    E = int(eoff[-1])
    src = to_dev(pad16(enc, E), dev)
    dst = torch.zeros(codec.decode_bound(E, n), dtype=torch.uint8, device=dev)
    dst, do, st, fs, fl = codec.decode_auto(src, to_dev(eoff, dev), enc_bytes=E, dst=dst,
                                            want_ctx=True, pick=pick)
    torch.cuda.synchronize()
    rd, rdo, rst, rfs, rfl = O.decode_batch(enc, eoff, nthreads=nthreads)
    st = st.cpu().numpy()
    bad = np.nonzero(st != rst)[0]
    assert bad.size == 0, "%s: status differs at %s (gpu %s, ref %s)" % (
        tag, bad[:5], st[bad[:5]], rst[bad[:5]])
    assert np.array_equal(fs.cpu().numpy().view(np.uint16), rfs), tag + ": fstate"
    assert np.array_equal(fl.cpu().numpy(), rfl), tag + ": flags"
    # the bytes the oracle wrote per string: its decoded length, or on
    # failure what it left in the (zero-initialised) slot before the error
    written = np.where(rst >= 0, rst, 0).astype(np.int64)
    fail = np.nonzero(rst < 0)[0]
    for i in fail:
        _, out, _ = O.decode(bytes(enc[int(eoff[i]):int(eoff[i + 1])]), final=1)
        written[i] = len(out)
    d = dst.cpu().numpy()
    do = do.cpu().numpy().view(np.uint32).astype(np.int64)
    tot = int(written.sum())
    rel = np.arange(tot) - np.repeat(np.cumsum(written) - written, written)
    got = d[np.repeat(do[:-1], written) + rel]
    want = rd[np.repeat(rdo[:-1].astype(np.int64), written) + rel]
    if not np.array_equal(got, want):
        k = int(np.nonzero(got != want)[0][0])
        i = int(np.searchsorted(np.cumsum(written), k, side="right"))
        raise AssertionError("%s: decoded byte differs in string %d" % (tag, i))
    return st, do


def window_edge_batch():
    """Encoded strings aimed at the item decoder's register window (round 3):
    30-bit codes and 5-bit codes at every bit alignment inside and across
    pieces, strings of whole 32-bit words, and invalid encodings (EOS inside a
    pair, all-ones tails, random bytes) that fail at varied bit positions."""
    rng = np.random.default_rng(31)
    long_syms = [10, 13, 22]  # 30-bit codes (RFC 7541 Appendix B)
    strs = []
    for shift in range(64):
        strs.append(b"0" * shift + bytes([10]) + b"a" * (shift % 7))
        strs.append(bytes([13]) * (1 + shift % 5) + b"0" * shift)
        strs.append(b"e" * shift + bytes(rng.choice(long_syms, 3).astype(np.uint8)) + b"t" * (63 - shift))
    for k in range(40):
        body = bytearray(rng.choice(np.frombuffer(b"0123456789aceiost", np.uint8), 300 + 17 * k))
        for p in rng.integers(0, len(body), 1 + k % 6):
            body[int(p)] = int(rng.choice(long_syms))
        strs.append(bytes(body))
    for w in range(1, 40):
        strs.append(b"0" * (32 * w))  # 160 w bits: ends on a word boundary, no padding
    strs.append(b"")
    off = np.zeros(len(strs) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(x) for x in strs])
    pool = np.frombuffer(b"".join(strs), dtype=np.uint8).copy()
    enc, eoff = O.encode_batch(pool, off)
    bad = [b"\xff" * k for k in range(1, 12)]  # EOS after 30 bits, or a bad tail
    for k in range(60):  # a valid prefix, then EOS at a varied bit position
        v = bytes(enc[int(eoff[k]):int(eoff[k + 1])])
        bad.append(v[: len(v) // 2] + b"\xff\xff\xff\xfc" + v[len(v) // 2:])
    bad += [bytes(rng.integers(0, 256, int(rng.integers(1, 200)), dtype=np.uint8)) for _ in range(60)]
    enc2 = np.concatenate([enc[:int(eoff[-1])], np.frombuffer(b"".join(bad), dtype=np.uint8)])
    eoff2 = np.concatenate([eoff, int(eoff[-1]) + np.cumsum([len(x) for x in bad]).astype(np.uint32)])
    return enc2, eoff2.astype(np.uint32)


@pytest.mark.parametrize("pick", ["items64", "pieces40"])
def test_decode_auto_window_edges(codec, dev, pick):
    """window_edge_batch through both decode_batch_auto instances: status,
    final context and every written byte against the oracle."""
    enc, eoff = window_edge_batch()
    st, _ = auto_decode_check(codec, dev, enc, eoff, "window edges " + pick, pick=pick)
    assert (st < 0).sum() >= 60  # the invalid encodings do fail


@pytest.mark.parametrize("cfg", [2, 3])
def test_decode_auto_full_size(codec, dev, cfg):
    """BASELINE.json configs 2 / 3 at full size (1M strings) through
    decode_batch_auto with the library's own pick (the instance bench.py
    times): status, final context and every byte against the oracle."""
    from nghttp2_amd import workloads as W
    n = 1 << 20
    pool, off = W.gen_pseudo_headers(n) if cfg == 2 else W.gen_mixed_values(n)
    enc, eoff = O.encode_batch(pool, off, nthreads=16)
    st, do = auto_decode_check(codec, dev, enc, eoff, "config %d" % cfg, nthreads=16)
    assert np.array_equal(st, np.diff(off.astype(np.int64)))


@pytest.mark.parametrize("name", make_golden.CASES)
def test_decode_auto_golden(codec, dev, name):
    """The committed golden fixtures through decode_batch_auto."""
    g = make_golden.load(name)
    for pick in (None, "items64", "pieces40"):
        st, _ = auto_decode_check(codec, dev, g["enc"][:int(g["enc_off"][-1])], g["enc_off"],
                                  name, pick=pick)
        assert np.array_equal(st, g["status"])


def test_decode_auto_max_length_strings(codec, dev):
    """NGHTTP2_HD_MAX_NV (lib/nghttp2_hd.h:45) sized literals, and longer,
    through decode_batch_auto: each instance, mixed with short strings."""
    from nghttp2_amd import workloads as W
    rng = np.random.default_rng(13)
    lens = np.array([65536, 1, 70000, 0, 65535, 5, 131072] + [20] * 200, dtype=np.int64)
    chars = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8)
    pool, off = W._pool_from_lengths(lens, chars)
    enc, eoff = O.encode_batch(pool, off)
    for pick in (None, "items64", "pieces40"):
        st, _ = auto_decode_check(codec, dev, enc, eoff, "max-len %s" % pick, pick=pick)
        assert np.array_equal(st, lens)


@pytest.mark.parametrize("pick", ["items64", "pieces40"])
def test_decode_auto_small_pool(codec, dev, pick):
    """A pool smaller than decode_bound: a string whose task span
    4 (ceil(floor(8 x_{i+1} / 5) / 4) + i + 1) passes dst_cap gets -502, no
    byte at or past dst_cap is written (guard bytes), dst_off saturates at
    dst_cap, and every other string is oracle-exact."""
    import torch
    from nghttp2_amd import workloads as W
    pool, off = W.gen_mixed_values(3000, seed=44)
    enc, eoff = O.encode_batch(pool, off)
    n = len(eoff) - 1
    E = int(eoff[-1])
    bound = codec.decode_bound(E, n)
    for cut in (700, 300, 37):
        cap = bound - cut
        dst = torch.full((bound + 4096,), 0x5A, dtype=torch.uint8, device=dev)
        src = to_dev(pad16(enc, E), dev)
        _, do, st, fs, fl = codec.decode_auto(src, to_dev(eoff, dev), enc_bytes=E,
                                              dst=dst[:cap], want_ctx=True, pick=pick)
        torch.cuda.synchronize()
        st = st.cpu().numpy()
        do = do.cpu().numpy().view(np.uint32).astype(np.int64)
        d = dst.cpu().numpy()
        assert (d[cap:] == 0x5A).all(), (pick, cut, "wrote at or past dst_cap")
        eo = eoff.astype(np.int64)
        g = (8 * (eo - eo[0])) // 5
        span_end = 4 * ((g[1:] + 3) // 4 + np.arange(1, n + 1))
        rd, rdo, rst, rfs, rfl = O.decode_batch(enc, eoff)
        over = span_end > cap
        assert over.any() and not over.all()
        assert (st[over] == O.NGHTTP2_ERR_BUFFER_ERROR).all(), (pick, cut)
        assert np.array_equal(st[~over], rst[~over]), (pick, cut)
        assert (do <= cap).all() and do[-1] == min(do[-1], cap)
        for i in np.nonzero(~over & (rst > 0))[0][::5]:
            assert bytes(d[do[i]:do[i] + rst[i]]) == bytes(rd[rdo[i]:rdo[i] + rst[i]]), (pick, i)


def test_fresh_codec_on_a_side_stream(dev):
    """A fresh codec whose first encode, emit_strings and decode_auto run on a
    non-current stream while the current stream is busy: every result equals
    the oracle (its workspaces are allocated on, and ordered by, the side
    stream)."""
    import torch
    import nghttp2_amd
    from nghttp2_amd import workloads as W
    pool, off = W.gen_pseudo_headers(40000, seed=61)
    c = nghttp2_amd.HuffmanBatchCodec(dev)
    side = torch.cuda.Stream(dev)
    src = to_dev(pad16(pool, off[-1]), dev)
    so = to_dev(off, dev)
    busy = torch.randn(4096, 4096, device=dev)
    side.wait_stream(torch.cuda.current_stream())  # (the inputs were copied on the current stream)
    for _ in range(16):
        busy = busy @ busy * 1e-3  # keeps the current stream busy meanwhile
    enc, eo = c.encode(src, so, raw_bytes=int(off[-1]), stream=side)
    lit, lo = c.emit_strings(src, so, raw_bytes=int(off[-1]), stream=side)
    dst, do, st = c.decode_auto(enc, eo, stream=side)
    side.synchronize()
    renc, reoff = O.encode_batch(pool, off)
    eo_h = eo.cpu().numpy().view(np.uint32)
    assert np.array_equal(eo_h, reoff)
    assert np.array_equal(enc.cpu().numpy()[:int(reoff[-1])], renc)
    rlit, rlo = O.emit_strings_batch(pool, off)
    assert np.array_equal(lo.cpu().numpy().view(np.uint32), rlo)
    assert np.array_equal(lit.cpu().numpy()[:int(rlo[-1])], rlit)
    raw = np.diff(off.astype(np.int64))
    assert np.array_equal(st.cpu().numpy(), raw)
    d = dst.cpu().numpy()
    do = do.cpu().numpy().view(np.uint32).astype(np.int64)
    rel = np.arange(int(raw.sum())) - np.repeat(np.cumsum(raw) - raw, raw)
    assert np.array_equal(d[np.repeat(do[:-1], raw) + rel], pool[:int(off[-1])])


@pytest.mark.gpu
@pytest.mark.parametrize("pick", ["pieces40", "items64"])
@pytest.mark.parametrize("n", [1, 31, 33, 63, 65, 1000, 2049, 5000, 70001])
def test_decode_instance_batch_sizes(codec, dev, n, pick):
    """Each decode instance's task claiming at every batch size shape: one
    string, less than a unit, ragged units and tasks, fewer tasks than
    waves, and ranges whose units are all tail units (claimed largest first
    once wave 0 has ranked them) -- status, state and bytes per string
    against the oracle."""
    from nghttp2_amd import workloads as W
    pool, off = W.gen_mixed_values(n, seed=1000 + n)
    enc, eoff = O.encode_batch(pool, off, nthreads=8)
    auto_decode_check(codec, dev, enc, eoff, "%s n=%d" % (pick, n), pick=pick, nthreads=8)


@pytest.mark.parametrize("where", ["tail", "head"])
def test_decode_pieces40_skewed_lengths(codec, dev, where):
    """Just-in-time tail claims with the work skewed: 60,000 short values and
    2,000 of 1-4 KB placed at the batch's end (every workgroup range's tail
    units are the heavy ones) or its start -- status, state and bytes per
    string against the oracle."""
    rng = np.random.default_rng(4242)
    short = rng.integers(16, 41, size=60000)
    long_ = rng.integers(1000, 4097, size=2000)
    lengths = np.concatenate([short, long_] if where == "tail" else [long_, short]).astype(np.int64)
    off = np.zeros(len(lengths) + 1, dtype=np.uint32)
    off[1:] = np.cumsum(lengths)
    pool = rng.integers(32, 127, size=int(off[-1]), dtype=np.uint8)
    enc, eoff = O.encode_batch(pool, off, nthreads=8)
    auto_decode_check(codec, dev, enc, eoff, "skewed %s" % where, pick="pieces40", nthreads=8)


def test_decode_auto_concurrent_streams(codec, dev):
    """The 40-byte instance's just-in-time tail claims with launches that run
    at the same time (round 5 also measured, and dropped, cross-workgroup
    stealing whose records such launches share): three streams each decode
    their own batch of long values four times, launched back to back; every
    string's status and bytes equal its raw input (a lost tail unit would
    leave its strings' status and bytes unwritten)."""
    import torch
    from nghttp2_amd import workloads as W
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    batches = []
    for k in range(3):
        pool, off = W.gen_mixed_values(60000 + 7000 * k, seed=7700 + k)
        enc, eoff = gpu_encode(codec, dev, pool, off)
        batches.append((pool, off, to_dev(pad16(enc, eoff[-1]), dev), to_dev(eoff, dev), int(eoff[-1])))
    torch.cuda.synchronize()
    outs = []
    for rep in range(4):
        for s, (pool, off, src, so, eb) in zip(streams, batches):
            s.wait_stream(torch.cuda.current_stream())
            outs.append((rep, pool, off) + tuple(codec.decode_auto(src, so, enc_bytes=eb, stream=s)))
    torch.cuda.synchronize()
    for rep, pool, off, dst, do, st in outs:
        raw = np.diff(off.astype(np.int64))
        assert np.array_equal(st.cpu().numpy(), raw), rep
        d = dst.cpu().numpy()
        do = do.cpu().numpy().view(np.uint32).astype(np.int64)
        rel = np.arange(int(raw.sum())) - np.repeat(np.cumsum(raw) - raw, raw)
        assert np.array_equal(d[np.repeat(do[:-1], raw) + rel], pool[:int(off[-1])]), rep
