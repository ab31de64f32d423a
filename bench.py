#!/usr/bin/env python3
"""bench.py -- HPACK Huffman encode+decode, device-resident, batched headers.

Metric (BASELINE.json): "GB/s HPACK Huffman enc+dec (device-resident,
batched headers); %HBM roofline".  One step = one batched encode of the
rank's synthetic header strings (count -> scan -> pack, the emit_string
pair lib/nghttp2_hd.c:1009/:1037) followed by one batched decode of the
result (engine-assigned output slots, decode with final=1, exact reference
status and decode context; hd_inflate_read_huff lib/nghttp2_hd.c:1728-1751).  Inputs are resident in HBM before timing.

value = sum over ranks of the algorithmic bytes B = 2R + 2E + 24 per string
 / max-over-ranks wall time of the K timed steps.
Multi-GPU: independent batches per rank (weak scaling), no collective on the
data path; the only collectives are the timing barrier and the max.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
CONFIG_NAMES = {
    2: "1M short pseudo-header strings (8-64 B), encode+decode, 1xMI355X",
    3: "1M mixed-length header values (16-1024 B, Zipf), encode+decode, 1xMI355X",
    4: "16M mixed-length header strings (16-1024 B, Zipf) sharded by bytes across the GPUs "
       "(no collective), encode+decode",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4])
    ap.add_argument("--strings", type=int, default=None,
                    help="strings per GPU (configs 2/3) or in total (config 4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=2,
                    help="pipeline the steps over this many streams (step i on stream i %% S)")
    ap.add_argument("--graph", action="store_true",
                    help="time replays of one HIP graph of the step instead of plain stream "
                         "launches (slower on ROCm 7 here: 0.131 vs 0.124 ms per step)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--host-resident", action="store_true",
                    help="also time the pinned-host H2D+D2H round trip")
    return ap.parse_args()


def cpu_cores_available():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(pool, off, threads):
    """Oracle (port of lib/nghttp2_hd_huffman.c) timed on host cores:
    count+encode then decode(final=1), best of repeats; same B accounting."""
    from oracle import oracle as O
    n = len(off) - 1
    raw = int(off[-1])
    res = {}
    for nth in sorted({1, threads}):
        best = None
        reps = 3 if nth == 1 else 5
        for _ in range(reps + 1):  # first rep is the warm-up
            te, td, etot, st = O.roundtrip_timed(pool, off, nth)
            assert (st >= 0).all()
            t = te + td
            best = t if best is None or t < best else best
        B = 2 * raw + 2 * etot + 24 * n
        res[nth] = (B / best / 1e9, best)
    return res


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import nghttp2_amd
    from nghttp2_amd import workloads as W

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    seed = W.SEED[args.config] + 7919 * rank  # each rank its own batch (weak scaling)
    scaling = "weak"
    if args.config == 2:
        n = args.strings or (1 << 20)
        pool, off = W.gen_pseudo_headers(n, seed=seed)
    elif args.config == 3:
        n = args.strings or (1 << 20)
        pool, off = W.gen_mixed_values(n, seed=seed)
    else:  # one fixed set, byte-balanced contiguous shard per rank (strong)
        from nghttp2_amd import shard as S
        n_total = args.strings or (1 << 24)
        lengths = W.mixed_lengths(n_total)
        all_off = np.zeros(n_total + 1, dtype=np.int64)
        np.cumsum(lengths, out=all_off[1:])
        s0, s1 = S.byte_balanced_bounds(all_off, world)[rank]
        pool, off = W.gen_mixed_range(lengths, s0, s1)
        n = s1 - s0
        scaling = "strong"
    raw_bytes = int(off[-1])

    src = torch.from_numpy(pool).to(dev)
    src_off = torch.from_numpy(off.view(np.int32)).to(dev)

    class Pipe:
        """One stream with its own output buffers and workspace: --streams S
        pipelines S of them, step i on pipe i % S, so one step's decode can
        overlap the next step's encode (independent batches; every step
        does its whole encode + decode)."""

        def __init__(self, stream):
            self.codec = nghttp2_amd.HuffmanBatchCodec(dev)
            self.stream = stream
            self.enc_cap = self.codec.encode_bound(raw_bytes, n)
            self.enc = torch.empty(self.enc_cap, dtype=torch.uint8, device=dev)
            self.enc_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
            self.dec_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
            self.dec = torch.empty(self.codec.decode_bound(self.enc_cap, n), dtype=torch.uint8,
                                   device=dev)
            self.status = torch.empty(n, dtype=torch.int32, device=dev)
            self.src, self.src_off = src, src_off  # --host-resident: the pipe's own copies

        def run(self, evs=None):
            st = self.stream
            if evs is not None:
                evs[0].record(st)
            self.codec.encode(self.src, self.src_off, raw_bytes=raw_bytes, dst=self.enc,
                              dst_off=self.enc_off, stream=st)
            if evs is not None:
                evs[1].record(st)
            self.codec.decode_auto(self.enc, self.enc_off, dst=self.dec, dst_off=self.dec_off,
                                   status=self.status, stream=st)
            if evs is not None:
                evs[2].record(st)

    pipes = [Pipe(torch.cuda.current_stream() if k == 0 else torch.cuda.Stream(device=dev))
             for k in range(max(1, args.streams))]
    P0 = pipes[0]
    codec, enc, enc_off, dec, dec_off, status = (P0.codec, P0.enc, P0.enc_off, P0.dec,
                                                 P0.dec_off, P0.status)
    stream = P0.stream

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(i=None):
        P0.run(ev[i] if i is not None else None)

    for _ in range(args.warmup):
        for p in pipes:
            p.run()
    torch.cuda.synchronize()
    for p in pipes[1:]:  # every pipe decodes the batch exactly
        assert torch.equal(p.status, P0.status) and torch.equal(p.enc_off, P0.enc_off)

    # correctness gate on this rank's batch (fails loudly, never measured)
    st = status.cpu().numpy()
    raw_len = np.diff(off.astype(np.int64))
    assert np.array_equal(st, raw_len), "decode(encode(x)) length mismatch"
    enc_total = int(enc_off[-1].item())
    do = dec_off.cpu().numpy().view(np.uint32).astype(np.int64)
    dh = dec.cpu().numpy()
    idx = np.repeat(do[:-1], raw_len) + (np.arange(raw_bytes) - np.repeat(off[:-1].astype(np.int64), raw_len))
    assert np.array_equal(dh[idx], pool[:raw_bytes]), "decode(encode(x)) != x"

    # per-kernel timing (roofline): K plain steps with events on the stream
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()

    # the timed steps: plain launches on the stream (no events in between),
    # or (--graph) replays of one HIP graph of the step's launches
    graph = None
    if args.graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        graph.replay()
        torch.cuda.synchronize()
        assert np.array_equal(status.cpu().numpy(), raw_len), "graph replay mismatch"

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if graph is not None:
            graph.replay()
        else:
            pipes[i % len(pipes)].run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0

    B_rank = 2 * raw_bytes + 2 * enc_total + 24 * n
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        b = torch.tensor([float(B_rank)], dtype=torch.float64, device=dev)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
        B_total = float(b.item())
    else:
        B_total = float(B_rank)

    t_enc = np.mean([ev[i][0].elapsed_time(ev[i][1]) for i in range(args.steps)]) * 1e-3
    t_dec = np.mean([ev[i][1].elapsed_time(ev[i][2]) for i in range(args.steps)]) * 1e-3
    ms_per_step = elapsed / args.steps * 1e3
    value = B_total * args.steps / elapsed / 1e9

    # roofline of the dominant kernel: k_decode (one launch per step; the
    # encode is three launches, k_enc_count + k_scan_tiles + k_encode, whose
    # sum is reported beside it).  traffic: PMC-measured HBM bytes per launch
    # of the same kernel on the same config (profiles/, FETCH_SIZE x 2 +
    # WRITE_SIZE per MI355X_MICROARCH.md), when recorded.
    dec_alg = raw_bytes + enc_total + 12 * n  # reads E + offsets, writes R + status
    enc_alg = raw_bytes + enc_total + 12 * n
    achieved = dec_alg / t_dec / 1e9
    traffic = None
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "traffic.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath)).get("config%d" % args.config, {}).get("k_decode")
        if tj and tj.get("strings") == n:
            traffic = tj["hbm_bytes_per_launch"]
    roof = {"bound": "hbm", "kernel": "k_decode", "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic, "alg_bytes_per_launch": dec_alg,
            "launch_ms": round(t_dec * 1e3, 4), "dec_ms": round(t_dec * 1e3, 4),
            "enc_ms": round(t_enc * 1e3, 4),
            "enc_achieved": round(enc_alg / t_enc / 1e9, 2)}

    out = {"metric": "GB/s HPACK Huffman enc+dec (device-resident, batched headers)",
           "value": round(value, 3), "unit": "GB/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
           "scaling": scaling, "vs_baseline": None, "dtype": "u8",
           "data": ("synthetic (numpy PCG64, seed 0x%X + 7919*rank)" % W.SEED[args.config])
                   if args.config != 4 else "synthetic (numpy PCG64, chunk-seeded 0x%X)" % W.SEED[4],
           "config": {"workload": CONFIG_NAMES[args.config], "strings_per_gpu": n,
                      "raw_bytes_per_gpu": raw_bytes, "enc_bytes_per_gpu": enc_total,
                      "E_over_R": round(enc_total / raw_bytes, 4),
                      "alg_bytes_per_step_all_gpus": int(B_total),
                      "parallelism": "shard%d (independent batches, no collective)" % world,
                      "streams": len(pipes)},
           "roofline": roof}

    if args.host_resident:
        # The path as deployed: raw headers start in (pinned) host memory and
        # both results go back to it -- H2D raw pool + offsets, encode,
        # decode, D2H encoded pool + offsets and decoded slots + status, all
        # async on the pipe's stream.  Steps are pipelined over the same
        # --streams pipes as `value` (each pipe has its own device input and
        # pinned outputs), so one step's D2H overlaps the next step's H2D
        # (the two directions of the link).  Same B accounting as `value`.
        h_src = torch.from_numpy(pool).pin_memory()
        h_off = torch.from_numpy(off.view(np.int32)).pin_memory()
        dec_used = int(dec_off[-1].item())
        for k, p in enumerate(pipes):
            if k:
                p.src, p.src_off = torch.empty_like(src), torch.empty_like(src_off)
            p.h_enc = torch.empty(enc_total + 16, dtype=torch.uint8).pin_memory()
            p.h_eoff = torch.empty(n + 1, dtype=torch.int32).pin_memory()
            p.h_dec = torch.empty(dec_used, dtype=torch.uint8).pin_memory()
            p.h_st = torch.empty(n, dtype=torch.int32).pin_memory()

        def host_step(i):
            p = pipes[i % len(pipes)]
            with torch.cuda.stream(p.stream):
                p.src.copy_(h_src, non_blocking=True)
                p.src_off.copy_(h_off, non_blocking=True)
                p.run()
                p.h_enc[:enc_total].copy_(p.enc[:enc_total], non_blocking=True)
                p.h_eoff.copy_(p.enc_off, non_blocking=True)
                p.h_dec.copy_(p.dec[:dec_used], non_blocking=True)
                p.h_st.copy_(p.status, non_blocking=True)

        for i in range(max(1, args.warmup) * len(pipes)):
            host_step(i)
        torch.cuda.synchronize()
        for p in pipes:
            assert np.array_equal(p.h_st.numpy(), raw_len)
            p.h_st.zero_()
        if world > 1:
            dist.barrier()
        th0 = time.perf_counter()
        for i in range(args.steps):
            host_step(i)
        torch.cuda.synchronize()
        th = time.perf_counter() - th0
        for p in pipes[:min(len(pipes), args.steps)]:
            assert np.array_equal(p.h_st.numpy(), raw_len)
            assert np.array_equal(p.h_dec.numpy()[idx], pool[:raw_bytes])
        pcie = (raw_bytes + 4 * (n + 1)) + (enc_total + 4 * (n + 1)) + dec_used + 4 * n
        out["host_resident"] = {
            "value": round(B_rank * args.steps / th / 1e9, 3), "unit": "GB/s",
            "ms_per_step": round(th / args.steps * 1e3, 4),
            "pcie_bytes_per_step": pcie,
            "streams": len(pipes),
            "note": "pinned H2D raw+offsets, encode, decode, D2H encoded+offsets, "
                    "decoded slots+status, steps pipelined over the streams; same "
                    "algorithmic-B accounting as value"}

    if rank == 0 and not args.no_cpu_baseline and world == 1:
        threads = max(1, min(args.cpu_threads, cpu_cores_available()))
        res = cpu_baseline(pool, off, threads)
        out["cpu_baseline"] = {
            "value": round(res[threads][0], 4), "unit": "GB/s", "cores": threads,
            "kind": "port",
            "sample": "the same %d-string batch, oracle/huff_oracle.c (restatement of "
                      "lib/nghttp2_hd_huffman.c, gcc -O2), count+encode+decode(final=1), "
                      "best of 5 after 1 warm-up, %d pthreads; 1-thread: %.4f GB/s"
                      % (n, threads, res[1][0]),
            "value_1thread": round(res[1][0], 4)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
