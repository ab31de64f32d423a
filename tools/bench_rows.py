#!/usr/bin/env python3
"""Throughput of the SURVEY.md 8(f) rows built beside the hot path:

  emit     nghttp2_amd_hd_emit_strings_batch: HPACK string literals
           (emit_string, lib/nghttp2_hd.c:1001-1044) for the config-2 batch,
           device-resident; GB/s of raw in + literals out.
  inflate  nghttp2_amd_hd_inflate_blocks: header blocks of many connections
           (host memory), Huffman literals decoded in one GPU batch per
           call; wire MB/s and fields/s, with the split between host passes
           and the GPU round trip.
  names    nghttp2_amd_hd_name_tokens_batch: lookup_token + name_hash
           (lib/nghttp2_hd.c:137, :536) over 1M header names, device-resident;
           algorithmic bytes sum(L) + 12 N (name bytes + offset in, token +
           hash out) over the kernel time (HIP events on its stream).

Prints one JSON object.  Not the bench.py contract (that is the hot path
itself); the numbers go to DESIGN.md."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def bench_emit(steps=20, cfg=2):
    """emit_strings on the config-2 (pseudo-headers) or config-3 (mixed
    values) batch: wall time per batch, and the launch pair's time by HIP
    events on its stream; roofline bytes R + F + 12 N (raw in, literals out,
    offsets) per batch against 8 TB/s."""
    import torch
    import nghttp2_amd
    from nghttp2_amd import workloads as W
    from oracle import oracle as O
    dev = torch.device("cuda:0")
    pool, off = W.gen_pseudo_headers(1 << 20) if cfg == 2 else W.gen_mixed_values(1 << 20)
    raw = int(off[-1])
    n = len(off) - 1
    codec = nghttp2_amd.HuffmanBatchCodec(dev)
    src = torch.from_numpy(pool).to(dev)
    so = torch.from_numpy(off.view(np.int32)).to(dev)
    dst, do = codec.emit_strings(src, so, raw_bytes=raw)
    torch.cuda.synchronize()
    # parity on a sample of the batch
    k = 20000
    rd, rdo = O.emit_strings_batch(pool, off[:k + 1])
    assert np.array_equal(do[:k + 1].cpu().numpy().view(np.uint32), rdo)
    assert np.array_equal(dst[:int(rdo[-1])].cpu().numpy(), rd)
    for _ in range(3):
        codec.emit_strings(src, so, raw_bytes=raw, dst=dst, dst_off=do)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        codec.emit_strings(src, so, raw_bytes=raw, dst=dst, dst_off=do)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    s = torch.cuda.current_stream()
    ev = []
    for _ in range(steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        codec.emit_strings(src, so, raw_bytes=raw, dst=dst, dst_off=do)
        b.record(s)
        ev.append((a, b))
    torch.cuda.synchronize()
    tk = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e-3
    F = int(do[-1].item())
    alg = raw + F + 12 * n
    return {"config": cfg, "strings": n, "raw_bytes": raw, "literal_bytes": F,
            "ms_per_batch": round(t * 1e3, 4), "GBps_raw_plus_out": round((raw + F) / t / 1e9, 1),
            "roofline": {"kernels": "k_enc_count<true> + k_encode<true>", "launch_pair_ms": round(tk * 1e3, 4),
                         "alg_bytes": alg, "achieved_GBps": round(alg / tk / 1e9, 1),
                         "frac_of_8TBps": round(alg / tk / 8e12, 4)}}


def bench_names(steps=50, long_frac=0.02):
    import torch
    import nghttp2_amd
    from nghttp2_amd import workloads as W
    from oracle import hpack_oracle as H
    dev = torch.device("cuda:0")
    pool, off = W.gen_names(1 << 20, long_frac=long_frac)
    n, raw = len(off) - 1, int(off[-1])
    codec = nghttp2_amd.HuffmanBatchCodec(dev)
    names = torch.from_numpy(pool).to(dev)
    no = torch.from_numpy(off.view(np.int32)).to(dev)
    tok, h = codec.name_tokens(names, no)
    torch.cuda.synchronize()
    k = 20000  # parity on a sample
    et, eh = H.name_tokens([pool[off[i]:off[i + 1]].tobytes() for i in range(k)])
    assert np.array_equal(tok[:k].cpu().numpy(), np.array(et, np.int32))
    assert np.array_equal(h[:k].cpu().numpy().view(np.uint32), np.array(eh, np.uint32))
    for _ in range(5):
        codec.name_tokens(names, no, token=tok, hash=h)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(steps):
        codec.name_tokens(names, no, token=tok, hash=h)
    e1.record(s)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / steps
    B = raw + 12 * n
    return {"names": n, "name_bytes": raw, "us_per_batch": round(t * 1e6, 2),
            "GBps_algorithmic": round(B / t / 1e9, 1), "hbm_frac": round(B / t / 8.0e12, 4),
            "Gnames_per_s": round(n / t / 1e9, 3), "long_wave_frac": long_frac}


def make_blocks(nconn, per_conn, fields_per_block, seed=7, index=False):
    """Header blocks of two indexed static fields and `fields_per_block`
    literal fields with a new name (Huffman when shorter), without indexing
    or (`index`) with incremental indexing, so every field enters the
    connection's dynamic table and evicts older ones."""
    from oracle import oracle as O
    from nghttp2_amd import workloads as W
    rng = np.random.Generator(np.random.PCG64(seed))
    pool, off = W.gen_mixed_values(nconn * per_conn * fields_per_block, seed=seed, hi=120)
    names = [b"cookie", b"user-agent", b"x-request-id", b"accept", b"referer", b"x-trace"]
    blocks, conns = [], []
    v = 0
    for r in range(per_conn):
        for c in range(nconn):
            out = bytearray(b"\x82\x87")  # :method GET, :scheme https
            for _ in range(fields_per_block):
                name = names[rng.integers(0, len(names))]
                val = bytes(pool[off[v]:off[v + 1]])
                v += 1
                out.append(0x40 if index else 0x00)  # literal, new name
                out += O.emit_string(name)
                out += O.emit_string(val)
            blocks.append(bytes(out))
            conns.append(c)
    return blocks, conns


def bench_inflate(nconn=256, per_conn=8, fields=16, reps=5, index=False):
    """The batched inflate front-end on `nconn` connections x `per_conn`
    blocks of `fields` literal fields: the C call alone
    (nghttp2_amd_hd_inflate_blocks: host parse, one GPU decode of every
    Huffman literal with its H2D/D2H, host replay, placement), timed around
    the ctypes call with the arrays built once, and the Python wrapper
    (inflate_blocks: marshalling the blocks in and the fields out) around it.
    Without `index` the blocks insert nothing into the tables, so repeated
    calls see the same state; with it every call starts from fresh
    inflaters (made outside the timed region)."""
    import ctypes
    import nghttp2_amd
    from nghttp2_amd import hd
    from oracle import hpack_oracle as HO
    blocks, conns = make_blocks(nconn, per_conn, fields, index=index)
    wire = sum(len(b) for b in blocks)
    infs = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
    # the wrapper, parity on the first connection's blocks against the restatement
    best_py = None
    for r in range(reps):
        if index and r:
            infs = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
        t0 = time.perf_counter()
        st, f = nghttp2_amd.inflate_blocks([infs[c] for c in conns], blocks)
        t = time.perf_counter() - t0
        best_py = t if best_py is None or t < best_py else best_py
    ref = HO.Inflater()
    for k, (c, b) in enumerate(zip(conns, blocks)):
        if c == 0:
            assert ref.inflate_block(b) == (st[k], f[k])
    nf = sum(len(x) for x in f)
    # the C call alone
    L = hd._inflate_lib()
    m = len(blocks)
    keep = [ctypes.create_string_buffer(b, len(b)) for b in blocks]
    ptrs = (ctypes.c_void_p * m)(*[ctypes.cast(k, ctypes.c_void_p) for k in keep])
    lens = (ctypes.c_size_t * m)(*[len(b) for b in blocks])
    ip = (ctypes.c_void_p * m)(*[infs[c].p.value for c in conns])
    nva_cap, arena_cap = wire + 16, 8 * wire + 4096
    nva = (hd._Nv * nva_cap)()
    arena = (ctypes.c_uint8 * arena_cap)()
    stc = (ctypes.c_int32 * m)()
    nv_used, ar_used = ctypes.c_size_t(), ctypes.c_size_t()
    import torch
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    best_c = None
    for _ in range(3 * reps):
        if index:
            fresh = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
            ip = (ctypes.c_void_p * m)(*[fresh[c].p.value for c in conns])
        t0 = time.perf_counter()
        rv = L.nghttp2_amd_hd_inflate_blocks(ip, m, ptrs, lens, nva, nva_cap, ctypes.byref(nv_used),
                                             arena, arena_cap, ctypes.byref(ar_used), stc, s)
        t = time.perf_counter() - t0
        assert rv == 0 and nv_used.value == nf
        best_c = t if best_c is None or t < best_c else best_c
    assert list(stc) == list(st)
    # CPU baseline: the oracle's C inflater (oracle/hpack_inflate_oracle.c,
    # the same algorithm, fresh inflaters per run) on 1 and 16 threads
    cpu = {}
    for t in (1, 16):
        best = None
        for _ in range(3):
            dt, nfc = HO.c_inflate_batch_timed(blocks, conns, nconn, t)
            assert nfc == nf
            best = dt if best is None or dt < best else best
        cpu["cpu_port_%dt_s" % t] = round(best, 5)
        cpu["cpu_port_%dt_wire_MBps" % t] = round(wire / best / 1e6, 1)
    return {"blocks": len(blocks), "connections": nconn, "fields": nf, "wire_bytes": wire, **cpu,
            "incremental_indexing": index,
            "c_s_per_call": round(best_c, 5), "c_wire_MBps": round(wire / best_c / 1e6, 1),
            "c_fields_per_s": round(nf / best_c),
            "py_s_per_call": round(best_py, 4), "py_wire_MBps": round(wire / best_py / 1e6, 1),
            "note": "c: nghttp2_amd_hd_inflate_blocks alone (host parse, one GPU decode of every "
                    "Huffman literal with H2D/D2H, host replay, placement), best of %d; py: the "
                    "inflate_blocks wrapper, Python marshalling in and out included" % (3 * reps)}


def bench_inflate_alt(nconn=256, per_conn=8, fields=16, alternations=7, index=False):
    """The batched inflate front-end's C call against the 16-thread CPU port
    of the same inflater (oracle/hpack_inflate_oracle.c) on the same blocks,
    in one process, alternating: each alternation times 5 front-end calls and
    3 CPU-port runs and keeps the median of each; the row reports the
    medians over the alternations and their ratio (the host threads are a
    share of a larger machine and swing between runs, so neither side is
    timed in isolation)."""
    import ctypes
    import statistics
    import nghttp2_amd
    from nghttp2_amd import hd
    from oracle import hpack_oracle as HO
    blocks, conns = make_blocks(nconn, per_conn, fields, index=index)
    wire = sum(len(b) for b in blocks)
    L = hd._inflate_lib()
    m = len(blocks)
    keep = [ctypes.create_string_buffer(b, len(b)) for b in blocks]
    ptrs = (ctypes.c_void_p * m)(*[ctypes.cast(k, ctypes.c_void_p) for k in keep])
    lens = (ctypes.c_size_t * m)(*[len(b) for b in blocks])
    nva_cap, arena_cap = wire + 16, 8 * wire + 4096
    nva = (hd._Nv * nva_cap)()
    arena = (ctypes.c_uint8 * arena_cap)()
    stc = (ctypes.c_int32 * m)()
    nv_used, ar_used = ctypes.c_size_t(), ctypes.c_size_t()
    import torch
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    infs = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
    ip = (ctypes.c_void_p * m)(*[infs[c].p.value for c in conns])
    nf = None
    gpu_med, cpu_med = [], []
    for a in range(alternations):
        ts = []
        for _ in range(5):
            if index:
                fresh = [nghttp2_amd.HpackInflater() for _ in range(nconn)]
                ip = (ctypes.c_void_p * m)(*[fresh[c].p.value for c in conns])
            t0 = time.perf_counter()
            rv = L.nghttp2_amd_hd_inflate_blocks(ip, m, ptrs, lens, nva, nva_cap, ctypes.byref(nv_used),
                                                 arena, arena_cap, ctypes.byref(ar_used), stc, s)
            ts.append(time.perf_counter() - t0)
            assert rv == 0
            nf = nv_used.value if nf is None else nf
            assert nv_used.value == nf
        gpu_med.append(statistics.median(ts))
        cs = []
        for _ in range(3):
            dt, nfc = HO.c_inflate_batch_timed(blocks, conns, nconn, 16)
            assert nfc == nf
            cs.append(dt)
        cpu_med.append(statistics.median(cs))
    g, c = statistics.median(gpu_med), statistics.median(cpu_med)
    return {"blocks": m, "connections": nconn, "fields": nf, "wire_bytes": wire,
            "incremental_indexing": index, "alternations": alternations,
            "c_s_per_call_median": round(g, 6), "c_wire_MBps": round(wire / g / 1e6, 1),
            "cpu_port_16t_s_median": round(c, 6), "cpu_port_16t_wire_MBps": round(wire / c / 1e6, 1),
            "ratio_front_end_over_cpu16": round(c / g, 3),
            "per_alternation_c_s": [round(x, 6) for x in gpu_med],
            "per_alternation_cpu16_s": [round(x, 6) for x in cpu_med]}


if __name__ == "__main__":
    rows = sys.argv[1:] or ["emit", "emit3", "inflate", "names"]
    fns = {"emit": bench_emit, "emit3": lambda: bench_emit(cfg=3), "inflate": bench_inflate,
           "inflate_index": lambda: bench_inflate(index=True),
           "inflate_alt": bench_inflate_alt,
           "inflate_alt_index": lambda: bench_inflate_alt(index=True),
           "names": bench_names,
           "names_short": lambda: bench_names(long_frac=0.0)}
    print(json.dumps({r: fns[r]() for r in rows}, indent=1))
