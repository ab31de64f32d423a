"""Multi-GPU sharding logic on CPU: byte-balanced partition, per-rank work,
reassembly -- including a real world_size=2 torch.distributed (gloo) run.

The per-rank worker here is the oracle (the CPU checker), standing in for
the GPU engine, so the test exercises the partition / rebase / gather logic
that bench.py and a multi-GPU deployment use; the GPU engine itself is
covered bit-exactly by tests/test_parity_gpu.py.
"""
import os
import socket

import numpy as np
import pytest

from nghttp2_amd import shard as S
from nghttp2_amd import workloads as W
from oracle import oracle as O


def test_bounds_cover_and_balance():
    pool, off = W.gen_mixed_values(20000, seed=5)
    for world in (1, 2, 3, 4, 8):
        b = S.byte_balanced_bounds(off, world)
        assert b[0][0] == 0 and b[-1][1] == len(off) - 1
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
        sizes = [int(off[s1]) - int(off[s0]) for s0, s1 in b]
        total = int(off[-1])
        # each shard within one max string of the ideal share
        assert max(abs(x - total / world) for x in sizes) <= 1024 + 1


def test_bounds_degenerate():
    off = np.zeros(6, dtype=np.uint32)  # 5 empty strings
    b = S.byte_balanced_bounds(off, 4)
    assert b[-1][1] == 5 and sum(s1 - s0 for s0, s1 in b) == 5
    off = np.array([0, 100], dtype=np.uint32)  # 1 string, 8 ranks
    b = S.byte_balanced_bounds(off, 8)
    assert sum(s1 - s0 for s0, s1 in b) == 1


def test_shard_encode_merge_equals_whole():
    pool, off = W.gen_pseudo_headers(30000, seed=8)
    whole, whole_off = O.encode_batch(pool, off)
    parts = []
    for s0, s1 in S.byte_balanced_bounds(off, 4):
        sp, so = S.shard(pool, off, s0, s1)
        parts.append(O.encode_batch(sp, so))
    merged, moff = S.merge(parts)
    assert np.array_equal(moff, whole_off.astype(np.uint64))
    assert np.array_equal(merged, whole)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pool, off = W.gen_mixed_values(6000, seed=11)  # every rank sees the same batch
    s0, s1 = S.byte_balanced_bounds(off, world)[rank]
    sp, so = S.shard(pool, off, s0, s1)
    enc, eoff = O.encode_batch(sp, so)  # this rank's shard only
    # round trip on the shard, as a rank would before reporting
    _, _, st, _, _ = O.decode_batch(enc, eoff)
    ok = bool(np.array_equal(st, np.diff(so.astype(np.int64))))
    objs = [None] * world
    dist.all_gather_object(objs, (enc[:int(eoff[-1])], eoff, ok))
    if rank == 0:
        merged, moff = S.merge([(e, o) for e, o, _ in objs])
        whole, woff = O.encode_batch(pool, off)
        q.put((all(o[2] for o in objs), bool(np.array_equal(merged, whole)),
               bool(np.array_equal(moff, woff.astype(np.uint64)))))
    dist.destroy_process_group()


def test_gloo_world2_shard_roundtrip():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) == (True, True, True)
