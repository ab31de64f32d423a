#!/usr/bin/env python3
"""bench.py -- HPACK Huffman encode+decode, device-resident, batched headers.

Metric (BASELINE.json): "GB/s HPACK Huffman enc+dec (device-resident,
batched headers); %HBM roofline".  One step = one batched encode of the
rank's synthetic header strings (count -> pack, the emit_string pair
lib/nghttp2_hd.c:1009/:1037) followed by one batched decode of the result
(engine-assigned output slots, decode with final=1, exact reference status
and decode context; hd_inflate_read_huff lib/nghttp2_hd.c:1728-1751).
Inputs are resident in HBM before timing.

value = sum over ranks of the algorithmic bytes B = 2R + 2E + 24 per string
 / max-over-ranks wall time of the K timed steps.

Workloads (BASELINE.json configs; --config):
  3  (default at 1 GPU) 1M mixed-length values, 16-1024 B Zipf -- the largest
     single-GPU enc+dec config; the line also carries config 2 as
     `secondary.config2` (same steps, same accounting)
  2  1M short pseudo-header strings, 8-64 B
  4  (default for N > 1) 16M strings from the config-3 generator, one fixed
     set, byte-balanced contiguous shard per rank (strong scaling), no
     collective on the data path
  5  decode-only adversarial batch (1M strings, seed 0x5EED0005): status-
     checked decode GB/s, B = E + decoded bytes + 12 per string
Multi-GPU: one process per GPU (torch.distributed.run); the only collectives
are the timing barrier, the max of the times and the sum of the bytes.
--backend gloo runs the ranks' collectives on the CPU, so N ranks can share
one GPU (a test of the multi-rank path on a one-GPU box).
"""
import argparse
import json
import os
import platform
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
    5: "decode-only adversarial batch (1M strings: 30-bit codes, EOS, padding cases), 1xMI355X",
}
CPU_SAMPLE = 1 << 20  # strings of the cpu_baseline sample (bounded CPU work)
BATCH_SEED_STEP = 104729  # seed offset of rotated batch b (--batches)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=None, choices=[2, 3, 4, 5],
                    help="default: 3 on one GPU, 4 (16M sharded) on more")
    ap.add_argument("--strings", type=int, default=None,
                    help="strings per GPU (configs 2/3/5) or in total (config 4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="config 3: skip the config-2 secondary measurement")
    ap.add_argument("--batches", type=int, default=3,
                    help="configs 2/3: distinct input batches rotated over the steps (step i "
                         "encodes batch i %% B), so no step re-reads the raw input the step "
                         "before it left in the caches; config 4 keeps one fixed set")
    ap.add_argument("--secondary-ms", type=float, default=30.0,
                    help="config 2 secondary: at least this long a timed window")
    ap.add_argument("--streams", type=int, default=2,
                    help="pipeline the steps over this many streams (step i on stream i %% S)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="threads of the cpu_baseline leg (default: every core this job may "
                         "use: the affinity mask, capped by OMP_NUM_THREADS when set)")
    ap.add_argument("--host-resident", action="store_true",
                    help="also time the pinned-host H2D+D2H round trip")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (auto: nccl = RCCL)")
    ap.add_argument("--dump-dir", default=None,
                    help="(tests) each rank writes its shard bounds, encoded pool, offsets and "
                         "decode status there after the warm-up, for an outside check")
    return ap.parse_args()


def cpu_info():
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    usable = aff
    if omp and omp.isdigit() and int(omp) > 0:
        usable = min(aff, int(omp))
    return {"nproc": os.cpu_count(), "affinity": aff, "omp_num_threads": omp,
            "cpu_model": model, "usable": usable, "cgroup_cpu_limit": cgroup_cpu_limit()}


def cgroup_cpu_limit():
    """The CPU bandwidth this job's cgroup allows, in CPUs (cgroup v2
    cpu.max, or v1 cfs quota / period), or None when unlimited or unreadable:
    the evidence for the thread count of the cpu_baseline leg."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def cpu_baseline_roundtrip(pool, off, threads, extra=()):
    """Oracle (port of lib/nghttp2_hd_huffman.c) timed on host cores:
    count+encode then decode(final=1), best of repeats; same B accounting."""
    from oracle import oracle as O
    n = len(off) - 1
    raw = int(off[-1])
    res = {}
    for nth in sorted({1, threads} | set(extra)):
        best = None
        reps = 3 if nth == 1 or nth in extra else 5
        for _ in range(reps + 1):  # first rep is the warm-up
            te, td, etot, st = O.roundtrip_timed(pool, off, nth)
            assert (st >= 0).all()
            t = te + td
            best = t if best is None or t < best else best
        B = 2 * raw + 2 * etot + 24 * n
        res[nth] = (B / best / 1e9, best)
    return res


def cpu_baseline_decode(enc, eoff, threads, gpu_status):
    """Oracle decode(final=1) of the adversarial batch on host cores, best of
    repeats; also the per-string status check of the GPU run (the oracle as
    the checker)."""
    from oracle import oracle as O
    res = {}
    st_ref = None
    for nth in sorted({1, threads}):
        best = None
        for _ in range(4):
            t0 = time.perf_counter()
            _, _, st, _, _ = O.decode_batch(enc, eoff, nthreads=nth)
            t = time.perf_counter() - t0
            best = t if best is None or t < best else best
            st_ref = st
        B = int(eoff[-1]) + int(np.maximum(st_ref, 0).sum()) + 12 * (len(eoff) - 1)
        res[nth] = (B / best / 1e9, best)
    return res, bool(np.array_equal(st_ref, gpu_status))


def verify_roundtrip(dec, dec_off, pool, off, chunk=1 << 18):
    """decode(encode(x)) == x for every string, in chunks of strings (the
    index arrays of a whole 16M-string shard would not fit host memory)."""
    n = len(off) - 1
    off64 = off.astype(np.int64)
    do = dec_off.astype(np.int64)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        ln = off64[a + 1:b + 1] - off64[a:b]
        tot = int(ln.sum())
        rel = np.arange(tot) - np.repeat(np.cumsum(ln) - ln, ln)
        idx = np.repeat(do[a:b], ln) + rel
        lo, hi = int(idx.min()) if tot else 0, int(idx.max()) + 1 if tot else 0
        got = dec[lo:hi].cpu().numpy()[idx - lo] if tot else np.zeros(0, np.uint8)
        if not np.array_equal(got, pool[off64[a]:off64[b]]):
            raise AssertionError("decode(encode(x)) != x in strings [%d, %d)" % (a, b))
        if (a // chunk) % 16 == 15:
            progress("checked %d of %d strings" % (b, n))


_T0 = time.perf_counter()


def progress(msg):
    """A progress line on stderr (long runs: config 4 generates and checks 16M
    strings); stdout keeps the one JSON line."""
    if os.environ.get("RANK", "0") == "0":
        print("[bench %7.1fs] %s" % (time.perf_counter() - _T0, msg), file=sys.stderr, flush=True)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import nghttp2_amd
    from nghttp2_amd import workloads as W

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cfg = args.config or (3 if world == 1 else 4)
    backend = args.backend
    if backend == "auto":
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if world > 1:
        dist.init_process_group(backend)
    ndev = max(1, torch.cuda.device_count())
    torch.cuda.set_device(local % ndev)  # gloo: ranks may share one GPU
    dev = torch.device("cuda", local % ndev)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")

    def allreduce(x, op):
        t = torch.tensor([float(x)], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=op)
        return float(t.item())

    def gen(c, rank_, b=0):
        """(pool, off, scaling, seed text) of configuration c for this rank
        (b: the rotated batch's index; batch 0 is the one earlier rounds used)."""
        seed = W.SEED[c] + 7919 * rank_ + BATCH_SEED_STEP * b  # each rank its own batch (weak scaling)
        seed_txt = "numpy PCG64, seed 0x%X + 7919*rank + %d*batch" % (W.SEED[c], BATCH_SEED_STEP)
        if c == 2:
            n = args.strings or (1 << 20)
            pool, off = W.gen_pseudo_headers(n, seed=seed)
            return pool, off, "weak", seed_txt
        if c == 3:
            n = args.strings or (1 << 20)
            pool, off = W.gen_mixed_values(n, seed=seed)
            return pool, off, "weak", seed_txt
        # config 4: one fixed set, byte-balanced contiguous shard per rank
        from nghttp2_amd import shard as S
        n_total = args.strings or (1 << 24)
        lengths = W.mixed_lengths(n_total)
        all_off = np.zeros(n_total + 1, dtype=np.int64)
        np.cumsum(lengths, out=all_off[1:])
        s0, s1 = S.byte_balanced_bounds(all_off, world)[rank_]
        pool, off = W.gen_mixed_range(lengths, s0, s1, threads=max(1, min(8, 16 // world)))
        return pool, off, "strong", "numpy PCG64, chunk-seeded 0x%X, shard [%d, %d) of %d" % (
            W.SEED[4], s0, s1, n_total)

    progress("config %d, %d rank(s), backend %s" % (cfg, world, backend))
    if cfg == 5:
        out = run_decode_only(args, torch, dist, nghttp2_amd, W, dev, world, rank, allreduce)
    else:
        nb = 1 if cfg == 4 else max(1, args.batches)
        batches = [gen(cfg, rank, b) for b in range(nb)]
        pool, off, scaling, data = batches[0]
        progress("generated %d batch(es) of %d strings, %d bytes (batch 0)"
                 % (nb, len(off) - 1, int(off[-1])))
        out, ctx = run_roundtrip(args, torch, dist, nghttp2_amd, dev, world, allreduce,
                                 [(b[0], b[1]) for b in batches], cfg, scaling, data)
        if cfg == 3 and not args.no_secondary:
            b2 = [gen(2, rank, b)[:2] for b in range(nb)]
            sec, _ = run_roundtrip(args, torch, dist, nghttp2_amd, dev, world, allreduce,
                                   b2, 2, "weak", "", host_resident=False,
                                   min_window_ms=args.secondary_ms)
            out["secondary"] = {"config2": {k: sec[k] for k in ("value", "ms_per_step", "steps")}}
            out["secondary"]["config2"].update(
                timed_ms=round(sec["ms_per_step"] * sec["steps"], 2),
                workload=CONFIG_NAMES[2], strings_per_gpu=sec["config"]["strings_per_gpu"],
                raw_bytes_per_gpu=sec["config"]["raw_bytes_per_gpu"], roofline=sec["roofline"])
        if rank == 0 and not args.no_cpu_baseline and world == 1:
            progress("cpu baseline")
            info = cpu_info()
            threads = args.cpu_threads or info["usable"]
            ns = min(len(off) - 1, CPU_SAMPLE)
            sp, so = pool, off[:ns + 1]
            # also as many threads as the affinity mask holds (the whole
            # machine's CPUs on the GPU box), beside the job's share
            aff = info["affinity"]
            res = cpu_baseline_roundtrip(sp, so, threads, extra=(aff,) if aff != threads else ())
            out["cpu_baseline"] = {
                "value": round(res[threads][0], 4), "unit": "GB/s", "cores": threads,
                "kind": "port",
                "kind_note": "the oracle's C restatement: the reference's lib/nghttp2_hd_huffman.c "
                             "does not compile on its own here (nghttp2.h includes the generated "
                             "nghttp2ver.h), so it is not timed itself",
                "sample": "%d strings (%s) of this workload, oracle/huff_oracle.c (C restatement "
                          "of lib/nghttp2_hd_huffman.c, gcc -O2), count+encode+decode(final=1), "
                          "best of 5 after 1 warm-up, %d pthreads; 1 thread: %.4f GB/s"
                          % (ns, "the whole batch" if ns == len(off) - 1 else "the first",
                             threads, res[1][0]),
                "value_1thread": round(res[1][0], 4),
                "value_affinity_threads": round(res[aff][0], 4), "affinity_threads": aff,
                "host": {k: info[k] for k in ("cpu_model", "nproc", "affinity",
                                              "omp_num_threads", "cgroup_cpu_limit")}}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


# The per-kernel event pass (roofline launch times) runs at least this many
# steps, right before the timed steps: at the driver's 20 steps (6 ms) the
# launch times and the timed window sit partly in the GPU's clock ramp
# (round 5: decode launch 0.231 ms at 20 event steps vs 0.220 at 100); the
# timed region is still exactly --steps steps.
EVENT_STEPS_MIN = 100


def run_roundtrip(args, torch, dist, nghttp2_amd, dev, world, allreduce, batches, cfg,
                  scaling, data, host_resident=None, min_window_ms=0.0):
    """batches: [(pool, off)] rotated over the steps (step i encodes batch
    i % len(batches)); min_window_ms > 0 (the secondary): time more than
    --steps steps if that is needed for a timed window at least that long."""
    nb = len(batches)
    srcs, srcs_off, raws, ns, enc_totals = [], [], [], [], []
    codec0 = nghttp2_amd.HuffmanBatchCodec(dev)
    for pool_b, off_b in batches:
        n_b, raw_b = len(off_b) - 1, int(off_b[-1])
        srcs.append(torch.from_numpy(pool_b).to(dev))
        srcs_off.append(torch.from_numpy(off_b.view(np.int32)).to(dev))
        # the encoded size, once, to size every pipe's decode pool from the
        # actual E (not the 30-bit worst case)
        cap_b = codec0.encode_bound(raw_b, n_b)
        probe_enc = torch.empty(cap_b, dtype=torch.uint8, device=dev)
        probe_off = torch.empty(n_b + 1, dtype=torch.int32, device=dev)
        codec0.encode(srcs[-1], srcs_off[-1], raw_bytes=raw_b, dst=probe_enc, dst_off=probe_off)
        e_b = int(probe_off[-1].item()) & 0xFFFFFFFF
        assert e_b != 0xFFFFFFFF, "encoded total overflows the uint32 offsets"
        del probe_enc, probe_off
        raws.append(raw_b)
        ns.append(n_b)
        enc_totals.append(e_b)
    progress("config %d: %d batch(es) on the device, encoded %s bytes" % (cfg, nb, enc_totals))
    pool, off = batches[0]
    n, raw_bytes, enc_total = ns[0], raws[0], enc_totals[0]
    n_max = max(ns)
    enc_cap = max(e + 4096 for e in enc_totals)  # the kernels never write past dst_cap
    dec_cap = max(codec0.decode_bound(e, k) for e, k in zip(enc_totals, ns))

    class Pipe:
        """One stream with its own output buffers and workspace: --streams S
        pipelines S of them, step i on pipe i % S, so one step's decode can
        overlap the next step's encode (independent batches; every step
        does its whole encode + decode)."""

        def __init__(self, stream):
            self.codec = nghttp2_amd.HuffmanBatchCodec(dev)
            self.stream = stream
            self.enc = torch.empty(enc_cap, dtype=torch.uint8, device=dev)
            self.enc_off = torch.empty(n_max + 1, dtype=torch.int32, device=dev)
            self.dec_off = torch.empty(n_max + 1, dtype=torch.int32, device=dev)
            self.dec = torch.empty(dec_cap, dtype=torch.uint8, device=dev)
            self.status = torch.empty(n_max, dtype=torch.int32, device=dev)
            self.host_src = None  # --host-resident: the pipe's own copies of batch 0

        def run(self, b, evs=None):
            st = self.stream
            k = ns[b]
            src_b, off_b = (srcs[b], srcs_off[b]) if self.host_src is None else self.host_src
            if evs is not None:
                evs[0].record(st)
            self.codec.encode(src_b, off_b, raw_bytes=raws[b], dst=self.enc,
                              dst_off=self.enc_off[:k + 1], stream=st)
            if evs is not None:
                evs[1].record(st)
            self.codec.decode_auto(self.enc, self.enc_off[:k + 1], enc_bytes=enc_totals[b],
                                   dst=self.dec, dst_off=self.dec_off[:k + 1],
                                   status=self.status[:k], stream=st)
            if evs is not None:
                evs[2].record(st)

    pipes = [Pipe(torch.cuda.current_stream() if k == 0 else torch.cuda.Stream(device=dev))
             for k in range(max(1, args.streams))]
    P0 = pipes[0]
    KE = max(args.steps, EVENT_STEPS_MIN)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(KE)]

    for w in range(args.warmup):
        for k, p in enumerate(pipes):
            p.run((w * len(pipes) + k) % nb)
        torch.cuda.synchronize()
        progress("config %d: warm-up step %d" % (cfg, w))

    progress("config %d: warm-up done, checking the round trips" % cfg)
    # correctness gate on every batch of this rank (fails loudly, never
    # measured); batch 0 last, so P0 holds it for --dump-dir
    for b in reversed(range(nb)):
        for p in pipes:
            p.run(b)
        torch.cuda.synchronize()
        k = ns[b]
        for p in pipes[1:]:  # every pipe decodes the batch exactly
            assert torch.equal(p.status[:k], P0.status[:k])
            assert torch.equal(p.enc_off[:k + 1], P0.enc_off[:k + 1])
        st_b = P0.status[:k].cpu().numpy()
        assert np.array_equal(st_b, np.diff(batches[b][1].astype(np.int64))), \
            "decode(encode(x)) length mismatch"
        assert int(P0.enc_off[k].item()) & 0xFFFFFFFF == enc_totals[b]
        verify_roundtrip(P0.dec, P0.dec_off[:k + 1].cpu().numpy().view(np.uint32), *batches[b])
    st = P0.status[:n].cpu().numpy()
    raw_len = np.diff(off.astype(np.int64))
    if args.dump_dir:
        rk = int(os.environ.get("RANK", "0"))
        np.savez(os.path.join(args.dump_dir, "rank%d.npz" % rk), data=np.array(data),
                 enc=P0.enc[:enc_total].cpu().numpy(),
                 enc_off=P0.enc_off[:n + 1].cpu().numpy().view(np.uint32), status=st,
                 dec=P0.dec[:int(P0.dec_off[n].item()) & 0xFFFFFFFF].cpu().numpy(),
                 dec_off=P0.dec_off[:n + 1].cpu().numpy().view(np.uint32))

    progress("config %d: round trips checked, timing" % cfg)
    # per-kernel timing (roofline): K plain steps with events on the stream
    for i in range(KE):
        P0.run(i % nb, ev[i])
    torch.cuda.synchronize()
    t_enc = np.mean([ev[i][0].elapsed_time(ev[i][1]) for i in range(KE)]) * 1e-3
    t_dec = np.mean([ev[i][1].elapsed_time(ev[i][2]) for i in range(KE)]) * 1e-3

    steps = args.steps
    if min_window_ms > 0:  # (the two-stream step is shorter than enc + dec)
        steps = max(steps, int(np.ceil(min_window_ms / (0.7 * (t_enc + t_dec) * 1e3))))

    # the timed steps: plain launches on the streams (no events in between)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        pipes[i % len(pipes)].run(i % nb)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    B_b = [2 * r + 2 * e + 24 * k for r, e, k in zip(raws, enc_totals, ns)]
    B_rank = sum(B_b[i % nb] for i in range(steps))  # all the timed steps
    if world > 1:
        import torch.distributed as dist_
        elapsed = allreduce(elapsed, dist_.ReduceOp.MAX)
        B_total = allreduce(B_rank, dist_.ReduceOp.SUM)
    else:
        B_total = float(B_rank)

    ms_per_step = elapsed / steps * 1e3
    value = B_total / elapsed / 1e9

    # roofline of the dominant kernel: k_decode_items (one launch per step; the
    # encode is two launches, k_enc_count + k_encode, reported beside it).
    # traffic: PMC-measured HBM bytes per launch of the same kernel on the
    # same config (profiles/traffic.json, FETCH_SIZE x 2 + WRITE_SIZE per
    # MI355X_MICROARCH.md), when recorded for this batch size.
    # (per launch: the event pass's mean over the rotated batches)
    alg = [r + e + 12 * k for r, e, k in zip(raws, enc_totals, ns)]  # reads E + offsets, writes R + status
    dec_alg = int(round(np.mean([alg[i % nb] for i in range(KE)])))
    enc_alg = dec_alg
    achieved = dec_alg / t_dec / 1e9
    copy_gbs = device_copy_gbs(torch, dev)
    roof = {"bound": "hbm", "kernel": "k_decode_items", "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic_for(cfg, n, "k_decode_items"), "alg_bytes_per_launch": dec_alg,
            "launch_ms": round(t_dec * 1e3, 4), "event_steps": KE, "enc_ms": round(t_enc * 1e3, 4),
            "enc_achieved": round(enc_alg / t_enc / 1e9, 2),
            # secondary roofline: the device-to-device copy rate
            # measured here, the attainable HBM ceiling for a streaming kernel
            "copy_peak": round(copy_gbs, 1), "frac_vs_copy": round(achieved / copy_gbs, 5)}
    if cfg == 2:
        roof["note"] = ("config 2's working set per step (~118 MB) fits the 256 MiB Infinity "
                        "Cache: its GB/s and frac are partly cache-served, not pure HBM")

    out = {"metric": "GB/s HPACK Huffman enc+dec (device-resident, batched headers)",
           "value": round(value, 3), "unit": "GB/s", "n_gpus": world,
           "steps": steps, "warmup": args.warmup,
           "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
           "scaling": scaling, "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (%s)" % data,
           "config": {"workload": CONFIG_NAMES[cfg], "config_id": cfg, "strings_per_gpu": n,
                      "raw_bytes_per_gpu": raw_bytes, "enc_bytes_per_gpu": enc_total,
                      "E_over_R": round(enc_total / max(1, raw_bytes), 4),
                      "alg_bytes_per_step_all_gpus": int(round(B_total / steps)),
                      "parallelism": "shard%d (independent batches, no collective)" % world,
                      "streams": len(pipes), "batches": nb},
           "roofline": roof}

    if host_resident is None:
        host_resident = args.host_resident
    if host_resident:
        # The path as deployed: raw headers start in (pinned) host memory and
        # both results go back to it -- H2D raw pool + offsets, encode,
        # decode, D2H encoded pool + offsets and decoded slots + status, all
        # async on the pipe's stream, steps pipelined over the --streams
        # pipes (one step's D2H overlaps the next step's H2D).
        h_src = torch.from_numpy(pool).pin_memory()
        h_off = torch.from_numpy(off.view(np.int32)).pin_memory()
        P0.run(0)
        torch.cuda.synchronize()
        dec_used = int(P0.dec_off[n].item()) & 0xFFFFFFFF
        for p in pipes:
            p.host_src = (torch.empty_like(srcs[0]), torch.empty_like(srcs_off[0]))
            p.h_enc = torch.empty(enc_total + 16, dtype=torch.uint8).pin_memory()
            p.h_eoff = torch.empty(n + 1, dtype=torch.int32).pin_memory()
            p.h_dec = torch.empty(dec_used, dtype=torch.uint8).pin_memory()
            p.h_st = torch.empty(n, dtype=torch.int32).pin_memory()

        def host_step(i):
            p = pipes[i % len(pipes)]
            with torch.cuda.stream(p.stream):
                p.host_src[0].copy_(h_src, non_blocking=True)
                p.host_src[1].copy_(h_off, non_blocking=True)
                p.run(0)
                p.h_enc[:enc_total].copy_(p.enc[:enc_total], non_blocking=True)
                p.h_eoff.copy_(p.enc_off[:n + 1], non_blocking=True)
                p.h_dec.copy_(p.dec[:dec_used], non_blocking=True)
                p.h_st.copy_(p.status[:n], non_blocking=True)

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
        pcie = (raw_bytes + 4 * (n + 1)) + (enc_total + 4 * (n + 1)) + dec_used + 4 * n
        out["host_resident"] = {
            "value": round(B_b[0] * args.steps / th / 1e9, 3), "unit": "GB/s",
            "ms_per_step": round(th / args.steps * 1e3, 4),
            "pcie_bytes_per_step": pcie, "streams": len(pipes),
            "note": "pinned H2D raw+offsets, encode, decode, D2H encoded+offsets, "
                    "decoded slots+status, steps pipelined over the streams; same "
                    "algorithmic-B accounting as value"}
    return out, None


_COPY_GBS = {}


def device_copy_gbs(torch, dev, nbytes=1 << 30, reps=10):
    """Device-to-device copy rate of a 1 GiB buffer by the library's streaming
    copy kernel (nghttp2_amd_hd__copy_calib: four 16-byte loads in flight
    per lane): read + write bytes over the copy's event-timed duration,
    median of reps -- the measured HBM ceiling the decode's frac_vs_copy is
    taken against.  1 GiB is 4x the Infinity Cache, so it is HBM-bound."""
    import ctypes

    import nghttp2_amd
    key = str(dev)
    if key not in _COPY_GBS:
        L = nghttp2_amd.lib()
        L.nghttp2_amd_hd__copy_calib.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_size_t, ctypes.c_void_p]
        a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        a.fill_(1)
        s = torch.cuda.current_stream(dev)

        def copy():
            rc = L.nghttp2_amd_hd__copy_calib(ctypes.c_void_p(b.data_ptr()),
                                              ctypes.c_void_p(a.data_ptr()), nbytes,
                                              ctypes.c_void_p(s.cuda_stream))
            assert rc == 0, rc
        copy()
        ts = []
        for _ in range(reps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            copy()
            e1.record(s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        _COPY_GBS[key] = 2.0 * nbytes / float(np.median(ts)) / 1e9
        del a, b
    return _COPY_GBS[key]


def kernel_src_sha():
    """sha256 (first 16 hex digits) of the kernel sources the PMC traffic
    depends on: the traffic recorded in profiles/traffic.json is reported
    only for the tree it was measured on."""
    import hashlib
    h = hashlib.sha256()
    for f in ("hd_huff.hip", "hd_huff_tables.inc"):
        with open(os.path.join(REPO, "nghttp2_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def traffic_for(cfg, n, kernel):
    """PMC-measured HBM bytes per launch (profiles/traffic.json) when they were
    recorded for this batch size AND these kernel sources, else None."""
    tpath = os.path.join(REPO, "profiles", "traffic.json")
    if not os.path.exists(tpath):
        return None
    tj = json.load(open(tpath)).get("config%d" % cfg, {}).get(kernel)
    if tj and tj.get("strings") == n and tj.get("src_sha") == kernel_src_sha():
        return tj["hbm_bytes_per_launch"]
    return None


def run_decode_only(args, torch, dist, nghttp2_amd, W, dev, world, rank, allreduce):
    """Config 5: decode(final=1) of the adversarial batch, engine slots; the
    per-string status is checked against the generator's construction (valid
    categories decode to their symbol count, embedded EOS and over-long
    padding fail) and, in the cpu_baseline leg, against the oracle."""
    n = args.strings or (1 << 20)
    pool, off, cats, nsym = W.gen_adversarial(n, seed=W.SEED[5] + 7919 * rank, return_nsym=True)
    E = int(off[-1])
    src = torch.from_numpy(pool).to(dev)
    so = torch.from_numpy(off.view(np.int32)).to(dev)
    codec = nghttp2_amd.HuffmanBatchCodec(dev)
    cap = codec.decode_bound(E, n)
    pipes = []
    for k in range(max(1, args.streams)):
        s = torch.cuda.current_stream() if k == 0 else torch.cuda.Stream(device=dev)
        pipes.append((s, torch.empty(cap, dtype=torch.uint8, device=dev),
                      torch.empty(n + 1, dtype=torch.int32, device=dev),
                      torch.empty(n, dtype=torch.int32, device=dev)))

    def run(p):
        s, dst, doff, st = p
        codec.decode_auto(src, so, enc_bytes=E, dst=dst, dst_off=doff, status=st, stream=s)

    for _ in range(args.warmup):
        for p in pipes:
            run(p)
    torch.cuda.synchronize()
    st = pipes[0][3].cpu().numpy()
    valid = np.isin(cats, [0, 5, 6])
    assert np.array_equal(st[valid], nsym[valid]), "valid adversarial strings mis-decoded"
    assert (st[np.isin(cats, [1, 2])] == -523).all(), "EOS / long padding not rejected"
    written = int(np.maximum(st, 0).sum())
    KE = max(args.steps, EVENT_STEPS_MIN)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(KE)]
    s0 = pipes[0][0]
    for i in range(KE):
        ev[i][0].record(s0)
        run(pipes[0])
        ev[i][1].record(s0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        run(pipes[i % len(pipes)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    B_rank = E + written + 12 * n
    if world > 1:
        elapsed = allreduce(elapsed, dist.ReduceOp.MAX)
        B_total = allreduce(B_rank, dist.ReduceOp.SUM)
    else:
        B_total = float(B_rank)
    t_dec = np.mean([a.elapsed_time(b) for a, b in ev]) * 1e-3
    achieved = B_rank / t_dec / 1e9
    out = {"metric": "GB/s HPACK Huffman decode (device-resident, adversarial batch)",
           "value": round(B_total * args.steps / elapsed / 1e9, 3), "unit": "GB/s",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (gen_adversarial, seed 0x%X + 7919*rank)" % W.SEED[5],
           "config": {"workload": CONFIG_NAMES[5], "config_id": 5, "strings_per_gpu": n,
                      "enc_bytes_per_gpu": E, "decoded_bytes_per_gpu": written,
                      "failing_strings": int((st < 0).sum()),
                      "parallelism": "shard%d (independent batches, no collective)" % world,
                      "streams": len(pipes)},
           "roofline": {"bound": "hbm", "kernel": "k_decode_items", "achieved": round(achieved, 2),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 5),
                        "traffic": traffic_for(5, n, "k_decode_items"),
                        "alg_bytes_per_launch": B_rank, "launch_ms": round(t_dec * 1e3, 4),
                        "event_steps": KE}}
    copy_gbs = device_copy_gbs(torch, dev)
    out["roofline"].update(copy_peak=round(copy_gbs, 1),
                           frac_vs_copy=round(achieved / copy_gbs, 5))
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        info = cpu_info()
        threads = args.cpu_threads or info["usable"]
        res, same = cpu_baseline_decode(pool[:E + 16], off, threads, st)
        assert same, "GPU status differs from the oracle on the adversarial batch"
        out["cpu_baseline"] = {
            "value": round(res[threads][0], 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": "the whole %d-string batch, oracle/huff_oracle.c decode(final=1), best of "
                      "4, %d pthreads; 1 thread: %.4f GB/s; per-string status equal to the "
                      "GPU's" % (n, threads, res[1][0]),
            "value_1thread": round(res[1][0], 4),
            "host": {k: info[k] for k in ("cpu_model", "nproc", "affinity", "omp_num_threads")}}
    return out


if __name__ == "__main__":
    main()
