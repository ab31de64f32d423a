"""Large batches on the GPU: BASELINE.json config 4 (16M strings sharded over
8 GPUs) and config 5 (1M adversarial strings, decode only) at full size, the
uint32 offset limits, the multi-rank bench path, and the link-level drop-in's
per-call latency.

- config 4, rank 0's byte-balanced shard of the 16M set (~2M strings,
  ~314 MB): encode + decode_auto bit-exact against the oracle (16 threads);
- config 4, the whole 16M set on one GPU (~2.5 GB raw): size-independent
  properties, decode(encode(x)) == x and status == length for every string;
- config 5: status, final {fstate, flags} and every written byte (the
  partial output of failing strings included) against the oracle;
- an encoded total past 4 GiB is refused (NGHTTP2_AMD_OFF_OVERFLOW), a
  decode pool past 4 GiB is refused (INVALID_ARGUMENT);
- bench.py as 2 ranks (gloo) sharing the one GPU: the N > 1 code path.
"""
import ctypes
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def to_dev(a, dev):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).to(dev)


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def test_config4_rank0_shard_bit_exact(codec, dev):
    import torch
    from nghttp2_amd import shard as S
    from nghttp2_amd import workloads as W
    lengths = W.mixed_lengths(1 << 24)
    all_off = np.zeros(len(lengths) + 1, dtype=np.int64)
    np.cumsum(lengths, out=all_off[1:])
    s0, s1 = S.byte_balanced_bounds(all_off, 8)[0]
    pool, off = W.gen_mixed_range(lengths, s0, s1)
    n, raw = s1 - s0, int(off[-1])
    assert n > 1_900_000 and raw > 300_000_000
    src, so = to_dev(pool, dev), to_dev(off, dev)
    enc, eoff = codec.encode(src, so, raw_bytes=raw)
    eo = _u32(eoff)
    renc, reoff = O.encode_batch(pool, off, nthreads=16)
    assert np.array_equal(eo, reoff)
    E = int(eo[-1])
    assert np.array_equal(enc[:E].cpu().numpy(), renc)
    dst, doff, st, fs, fl = codec.decode_auto(enc, eoff, enc_bytes=E, want_ctx=True)
    torch.cuda.synchronize()
    rd, rdo, rst, rfs, rfl = O.decode_batch(renc, reoff, nthreads=16)
    assert np.array_equal(st.cpu().numpy(), rst)
    assert np.array_equal(fs.cpu().numpy().view(np.uint16), rfs)
    assert np.array_equal(fl.cpu().numpy(), rfl)
    ln = np.diff(off.astype(np.int64))
    assert np.array_equal(rst, ln)
    # every decoded byte: the engine slot of string i against the oracle's
    do = _u32(doff).astype(np.int64)
    rel = np.arange(raw) - np.repeat(off[:-1].astype(np.int64), ln)
    d = dst.cpu().numpy()
    assert np.array_equal(d[np.repeat(do[:-1], ln) + rel],
                          rd[np.repeat(rdo[:-1].astype(np.int64), ln) + rel])


def test_config4_full_16m_one_gpu_properties(codec, dev):
    """All 16,777,216 config-4 strings (their lengths from the config-4
    generator; bytes uniform printable ASCII drawn on the GPU) in ONE batch:
    the encoded and decoded pools stay inside the uint32 offsets; every
    string decodes to its bytes with status == length and an accepting
    final state."""
    import torch
    from nghttp2_amd import workloads as W
    lengths = W.mixed_lengths(1 << 24)
    n = len(lengths)
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lengths, out=off[1:])
    raw = int(off[-1])
    assert raw < 2 ** 32
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0004)
    src = torch.randint(0x20, 0x7F, (raw + (-raw) % 16 + 16,), generator=g, device=dev,
                        dtype=torch.uint8)
    so = to_dev(off.astype(np.uint32), dev)
    enc, eoff = codec.encode(src, so, raw_bytes=raw)
    torch.cuda.synchronize()
    E = int(eoff[-1].item()) & 0xFFFFFFFF
    assert E != 0xFFFFFFFF and E > raw // 2
    dst, doff, st, fs, fl = codec.decode_auto(enc, eoff, enc_bytes=E, want_ctx=True)
    torch.cuda.synchronize()
    ln_t = torch.from_numpy(lengths.astype(np.int32)).to(dev)
    assert torch.equal(st, ln_t)
    assert bool(((fl & 1) == 1).all())
    do = doff.to(torch.int64) & 0xFFFFFFFF
    so64 = so.to(torch.int64) & 0xFFFFFFFF
    chunk = 1 << 21
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        ln = ln_t[a:b].to(torch.int64)
        tot = int(ln.sum().item())
        first = torch.cumsum(ln, 0) - ln
        rel = torch.arange(tot, device=dev) - torch.repeat_interleave(first, ln)
        got = dst[torch.repeat_interleave(do[a:b], ln) + rel]
        want = src[torch.repeat_interleave(so64[a:b], ln) + rel]
        assert torch.equal(got, want), "strings [%d, %d)" % (a, b)


def test_config5_full_size_bit_exact(codec, dev):
    """BASELINE.json config 5 at full size (1,048,576 strings, seed
    0x5EED0005): engine slots (decode_auto) and the reference's caller slots
    (decode), status, final context and every written byte -- including the
    partial output of the failing strings -- against the oracle."""
    import torch
    from nghttp2_amd import workloads as W
    pool, off, cats = W.gen_adversarial(1 << 20)
    n, E = len(off) - 1, int(off[-1])
    rd, rdo, rst, rfs, rfl = O.decode_batch(pool[:E], off, nthreads=16)
    assert (rst < 0).sum() > 100_000 and (rst >= 0).sum() > 400_000
    src, so = to_dev(pool, dev), to_dev(off, dev)
    # the reference's slots, zero-initialised like the oracle's pool: the
    # whole pool compares, partial outputs included
    dst = torch.zeros(int(rdo[-1]) + 16, dtype=torch.uint8, device=dev)
    _, _, st, fs, fl = codec.decode(src, so, dst_off=to_dev(rdo, dev), dst=dst, want_ctx=True)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), rst)
    assert np.array_equal(fs.cpu().numpy().view(np.uint16), rfs)
    assert np.array_equal(fl.cpu().numpy(), rfl)
    assert np.array_equal(dst[:int(rdo[-1])].cpu().numpy(), rd[:int(rdo[-1])])
    # engine slots: the same results, the decoded bytes of every success
    d2, doff, st2, fs2, fl2 = codec.decode_auto(src, so, enc_bytes=E, want_ctx=True)
    torch.cuda.synchronize()
    assert np.array_equal(st2.cpu().numpy(), rst)
    assert np.array_equal(fs2.cpu().numpy().view(np.uint16), rfs)
    assert np.array_equal(fl2.cpu().numpy(), rfl)
    ok = np.nonzero(rst > 0)[0]
    ln = rst[ok].astype(np.int64)
    rel = np.arange(int(ln.sum())) - np.repeat(np.cumsum(ln) - ln, ln)
    do = _u32(doff).astype(np.int64)
    assert np.array_equal(d2.cpu().numpy()[np.repeat(do[ok], ln) + rel],
                          rd[np.repeat(rdo[ok].astype(np.int64), ln) + rel])


def test_decode_pool_past_4gib_refused(codec, dev):
    import torch
    from nghttp2_amd import hd
    from nghttp2_amd import workloads as W
    pool, off = W.gen_pseudo_headers(100)
    src, so = to_dev(pool, dev), to_dev(off, dev)
    dst = torch.zeros(4096 * 4, dtype=torch.uint8, device=dev)
    doff = torch.empty(101, dtype=torch.int32, device=dev)
    st = torch.empty(100, dtype=torch.int32, device=dev)
    L = hd.lib()
    rv = L.nghttp2_amd_hd_huff_decode_batch_auto(
        hd._p(src), hd._p(so), 100, int(off[-1]), hd._p(dst), (1 << 32) + 64, hd._p(doff),
        hd._p(st), None, None, hd._stream(None))
    assert rv == hd.NGHTTP2_ERR_INVALID_ARGUMENT


def test_encode_total_past_limit_marks_overflow(codec, dev):
    """A capacity smaller than the encoded total: no byte past dst_cap, the
    tiles that fit are encoded exactly, dst_off[n] = NGHTTP2_AMD_OFF_OVERFLOW."""
    import torch
    from nghttp2_amd import workloads as W
    pool, off = W.gen_pseudo_headers(5000, seed=4)
    renc, reoff = O.encode_batch(pool, off)
    cap = int(reoff[2600])  # strings past ~2600 do not fit
    dst = torch.full((cap + 4096,), 0xAB, dtype=torch.uint8, device=dev)
    eoff = torch.empty(5001, dtype=torch.int32, device=dev)
    codec.encode(to_dev(pool, dev), to_dev(off, dev), raw_bytes=int(off[-1]),
                 dst=dst[:cap], dst_off=eoff)
    torch.cuda.synchronize()
    eo = _u32(eoff)
    assert eo[-1] == 0xFFFFFFFF
    assert (dst[cap:].cpu().numpy() == 0xAB).all()
    # the first tiles (256 strings each) are whole and exact
    k = 2560
    assert np.array_equal(eo[:k + 1], reoff[:k + 1])
    assert np.array_equal(dst[:int(reoff[k])].cpu().numpy(), renc[:int(reoff[k])])


def test_encode_total_past_4gib_marks_overflow(codec, dev):
    """A real 64-bit total: 1.4 GB of 0xFF bytes (26-bit codes) encode to
    ~4.5 GB, past the uint32 offsets; the batch reports the overflow and the
    strings before the limit are exact."""
    import torch
    n, L = 1_400_000, 1000
    raw = n * L
    off = np.arange(n + 1, dtype=np.int64) * L
    src = torch.full((raw + 32,), 0xFF, dtype=torch.uint8, device=dev)
    enc, eoff = codec.encode(src, to_dev(off.astype(np.uint32), dev), raw_bytes=raw)
    torch.cuda.synchronize()
    eo = _u32(eoff)
    assert eo[-1] == 0xFFFFFFFF
    one, _ = O.encode_batch(np.full(L + 16, 0xFF, np.uint8), np.array([0, L], np.uint32))
    E1 = len(one)
    assert E1 == (26 * L + 7) // 8
    k = 1000  # strings of the first tiles: offsets i * E1 and the same bytes
    assert np.array_equal(eo[:k + 1].astype(np.int64), np.arange(k + 1) * E1)
    e = enc[:k * E1].cpu().numpy().reshape(k, E1)
    assert (e == np.frombuffer(bytes(one), np.uint8)).all()
    del enc, src
    torch.cuda.empty_cache()


def test_encode_string_past_max_marks_overflow(codec, dev):
    """A string of more than NGHTTP2_AMD_ENCODE_MAX_STRING raw bytes (its code
    bits would pass the kernels' 32-bit counts) marks the batch overflowed,
    even when the encoded total would fit the pool (as the header says); the
    tiles before it are exact."""
    import torch
    max_string = 0xFFFFFFFF // 30
    L0 = 600
    n_small = 300  # two tiles of 256 strings before ... the long one lies in the second
    huge = max_string + 1
    lens = [L0] * n_small + [huge]
    off = np.zeros(len(lens) + 1, dtype=np.int64)
    off[1:] = np.cumsum(lens)
    raw = int(off[-1])
    src = torch.full((raw + 32,), ord("a"), dtype=torch.uint8, device=dev)
    enc, eoff = codec.encode(src, to_dev(off.astype(np.uint32), dev), raw_bytes=raw)
    torch.cuda.synchronize()
    eo = _u32(eoff)
    assert eo[-1] == 0xFFFFFFFF, "overflow mark"
    one, _ = O.encode_batch(np.full(L0 + 16, ord("a"), np.uint8), np.array([0, L0], np.uint32))
    E1 = len(one)
    assert np.array_equal(eo[:257].astype(np.int64), np.arange(257) * E1), "first tile exact"
    del enc, src
    torch.cuda.empty_cache()


def test_encode_wave_output_near_2_32_bits(codec, dev):
    """Four 30 MB strings of 0xFF (26-bit codes) in one wave: each far below
    NGHTTP2_AMD_ENCODE_MAX_STRING, one wave writes 3.3e9 bits (390 MB, under
    the 2^29-byte tile limit): every byte and offset equals the oracle's.
    Six of them (585 MB in one 256-string tile, 4.7e9 bits, past 32-bit bit
    positions) mark the batch overflowed, even with a pool that holds them,
    and no byte is written past dst_cap."""
    import torch
    L = 30 << 20
    one, _ = O.encode_batch(np.full(L + 16, 0xFF, np.uint8), np.array([0, L], np.uint32))
    E1 = len(one)
    assert E1 == (26 * L + 7) // 8
    src = torch.full((6 * L + 32,), 0xFF, dtype=torch.uint8, device=dev)
    ref = torch.from_numpy(np.frombuffer(bytes(one), np.uint8).copy()).to(dev)
    n = 4
    off = (np.arange(n + 1, dtype=np.int64) * L).astype(np.uint32)
    assert 8 * E1 * n > (3 << 30) and E1 * n < (1 << 29)
    enc, eoff = codec.encode(src, to_dev(off, dev), raw_bytes=n * L)
    torch.cuda.synchronize()
    eo = _u32(eoff).astype(np.int64)
    assert np.array_equal(eo, np.arange(n + 1) * E1), "offsets"
    for i in range(n):
        assert torch.equal(enc[i * E1:(i + 1) * E1], ref), "string %d" % i
    del enc
    n = 6
    off = (np.arange(n + 1, dtype=np.int64) * L).astype(np.uint32)
    assert E1 * n >= (1 << 29)
    cap = codec.encode_bound(n * L, n)
    dst = torch.full((cap + 4096,), 0xAB, dtype=torch.uint8, device=dev)
    eoff2 = torch.empty(n + 1, dtype=torch.int32, device=dev)
    codec.encode(src, to_dev(off, dev), raw_bytes=n * L, dst=dst[:cap], dst_off=eoff2)
    torch.cuda.synchronize()
    assert _u32(eoff2)[-1] == 0xFFFFFFFF, "overflow mark"
    assert bool((dst[cap:] == 0xAB).all()), "a byte past dst_cap was written"
    del dst, src, ref
    torch.cuda.empty_cache()


def test_encode_large_batch_scanned_tile_prefix(codec, dev):
    """Past 16,384 tiles of 256 strings the tile prefixes are scanned in their
    own launch (k_tile_prefix64) instead of summed by every k_encode
    workgroup: 4.5M config-2 strings (17,579 tiles), offsets and encoded
    bytes bit-exact against the oracle (emit_strings takes the same path)."""
    import hashlib
    import torch
    from nghttp2_amd import workloads as W
    n = 4_500_000
    pool, off = W.gen_pseudo_headers(n, seed=0x5CA9)
    assert (n + 255) // 256 > 16384
    renc, reoff = O.encode_batch(pool, off, nthreads=16)
    src = to_dev(np.concatenate([pool, np.zeros(16, np.uint8)]), dev)
    so = to_dev(off, dev)
    enc, eoff = codec.encode(src, so, raw_bytes=int(off[-1]))
    torch.cuda.synchronize()
    assert np.array_equal(_u32(eoff), reoff.astype(np.uint32)), "offsets"
    E = int(reoff[-1])
    assert hashlib.sha256(enc[:E].cpu().numpy().tobytes()).digest() == \
        hashlib.sha256(renc[:E].tobytes()).digest(), "encoded bytes"
    del enc, eoff
    torch.cuda.empty_cache()


def test_encode_dst_cap_below_bound_guard(codec, dev):
    """A pool smaller than the encoded batch (dst_cap below encode_bound and
    below the output itself, not a multiple of 16): the tiles that fit are
    exact, the first one that does not and every later one write nothing
    (saturated offsets, the overflow mark), and no byte at or past dst_cap
    is written (guard bytes intact)."""
    import torch
    from nghttp2_amd import workloads as W
    pool, off = W.gen_mixed_values(40000, seed=77)
    renc, reoff = O.encode_batch(pool, off, nthreads=8)
    E = int(reoff[-1])
    cap = (E * 3) // 5 + 7
    dst = torch.full((cap + 8192,), 0xAB, dtype=torch.uint8, device=dev)
    eoff = torch.empty(len(off), dtype=torch.int32, device=dev)
    src = to_dev(np.concatenate([pool, np.zeros(16, np.uint8)]), dev)
    codec.encode(src, to_dev(off, dev), raw_bytes=int(off[-1]), dst=dst[:cap], dst_off=eoff)
    torch.cuda.synchronize()
    eo = _u32(eoff).astype(np.int64)
    assert eo[-1] == 0xFFFFFFFF, "overflow mark"
    assert bool((dst[cap:] == 0xAB).all()), "a byte at or past dst_cap was written"
    # the strings whose tile fits: offsets and bytes equal the oracle's
    ok = np.nonzero(reoff[1:].astype(np.int64) <= cap)[0]
    fits = ok[ok < (len(ok) // 256) * 256]  # whole tiles before the cut
    assert fits.size > 0
    k = int(fits[-1]) + 1
    assert np.array_equal(eo[:k], reoff[:k].astype(np.int64))
    d = dst[:int(reoff[k])].cpu().numpy()
    assert np.array_equal(d, renc[:int(reoff[k])])
    assert (eo[k:-1] <= cap).all(), "offsets saturate at dst_cap"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench_ranks_gloo_one_gpu(nranks, total, tmp_path):
    """bench.py's N > 1 path (init, byte-balanced config-4 shard per rank,
    barrier, max-over-ranks time, summed bytes) as `nranks` ranks on the one
    GPU, collectives over gloo; each rank's encoded shard (bytes and offsets)
    is then checked against the oracle's encode of the same shard, and its
    decode (status, dense offsets and every decoded byte) against the
    shard's raw strings."""
    from nghttp2_amd import shard as S
    from nghttp2_amd import workloads as W
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % nranks,
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", str(nranks), "--backend", "gloo",
           "--config", "4", "--strings", str(total), "--steps", "3", "--warmup", "1",
           "--streams", "1", "--no-cpu-baseline", "--dump-dir", str(tmp_path)]
    # (rank 0's progress lines pass through to the test's output: a long run
    # keeps printing)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=540, env=env, cwd=REPO)
    assert r.returncode == 0, "bench.py ranks failed (rc %d)" % r.returncode
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == nranks and out["scaling"] == "strong" and out["value"] > 0
    lengths = W.mixed_lengths(total)
    all_off = np.zeros(total + 1, dtype=np.int64)
    np.cumsum(lengths, out=all_off[1:])
    bounds = S.byte_balanced_bounds(all_off, nranks)
    # the shards cover the set, and rank 0 ran its byte-balanced shard
    assert bounds[0][0] == 0 and bounds[-1][1] == total
    assert all(bounds[k][1] == bounds[k + 1][0] for k in range(nranks - 1))
    assert out["config"]["strings_per_gpu"] == bounds[0][1] - bounds[0][0]
    for rk, (s0, s1) in enumerate(bounds):
        print("checking rank %d: strings [%d, %d)" % (rk, s0, s1), flush=True)
        d = np.load(str(tmp_path / ("rank%d.npz" % rk)))
        pool, off = W.gen_mixed_range(lengths, s0, s1, threads=8)
        renc, reoff = O.encode_batch(pool, off, nthreads=16)
        assert np.array_equal(d["enc_off"], reoff), "rank %d: encoded offsets" % rk
        assert np.array_equal(d["enc"], renc[:int(reoff[-1])]), "rank %d: encoded bytes" % rk
        ln = np.diff(off.astype(np.int64))
        assert np.array_equal(d["status"], ln), "rank %d: status" % rk
        # decoded bytes: dense per task, string i at dec_off[i]
        do = d["dec_off"].astype(np.int64)
        dec = d["dec"]
        assert int(do[-1]) == len(dec) >= int(ln.sum()), "rank %d: decoded extent" % rk
        for a in range(0, len(ln), 1 << 19):
            b = min(len(ln), a + (1 << 19))
            lc = ln[a:b]
            rel = np.arange(int(lc.sum())) - np.repeat(np.cumsum(lc) - lc, lc)
            got = dec[np.repeat(do[a:b], lc) + rel]
            want = pool[np.repeat(off[a:b].astype(np.int64), lc) + rel]
            assert np.array_equal(got, want), "rank %d: decoded bytes of strings [%d, %d)" % (rk, a, b)


def test_bench_two_ranks_gloo_one_gpu(dev, tmp_path):
    _bench_ranks_gloo_one_gpu(2, 1 << 21, tmp_path)


@pytest.mark.timeout(900)
def test_bench_eight_ranks_gloo_one_gpu_config4(dev, tmp_path):
    """The 8-way split of the whole config-4 set (16M strings, BASELINE.json
    configs[3]) as 8 bench.py ranks sharing the one GPU: each rank's encode
    and decode checked byte for byte.  (Still one physical GPU: the 8-GPU
    node's scaling is measured only by the driver.)"""
    _bench_ranks_gloo_one_gpu(8, 1 << 24, tmp_path)


def test_compat_per_call_latency(dev):
    """The link-level drop-in (one string per call, as emit_string and
    hd_inflate_read_huff call it) against the port, per call; results equal.
    The numbers go to gpurun_out/compat_latency.json for INTEGRATION.md."""
    import tempfile
    libdir = os.path.join(REPO, "nghttp2_amd", "lib")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "compat_latency")
        subprocess.run(["gcc", "-O2", "-Wall", "-I", os.path.join(REPO, "include"),
                        os.path.join(REPO, "tests", "c", "compat_latency.c"), "-L" + libdir,
                        "-lnghttp2_amd_hd", "-Wl,-rpath," + libdir, "-ldl", "-lpthread", "-o", exe], check=True)
        r = subprocess.run([exe, O.lib_path() if hasattr(O, "lib_path") else
                            os.path.join(REPO, "oracle", "_build", "libhuff_oracle.so"), "2000"],
                           capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["mismatches"] == 0 and res["threads4_mismatches"] == 0
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "compat_latency.json"), "w") as f:
        json.dump(res, f)
    print(res)
