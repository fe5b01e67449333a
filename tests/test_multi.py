"""Multi-process (N>1) path of bench.py on CPU: gloo, world size 2.

Each rank decodes its own disjoint frames (weak scaling); the timed region's
max over ranks and the summed counters are the only collectives."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist

    import bench
    import qkd_ldpc_v_amd as Q

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b, q_acc = Q.bsc_frames(64, 0.05, 8, seed=bench.rank_seed(rank))
        elapsed = 1.0 + rank  # rank 1 is the slow one
        tot = bench.combine_ranks(dist, elapsed, 10 * (rank + 1), 8 - rank, 7, 8, 2.0 * (rank + 1),
                                  torch.device("cpu"))
        q.put((rank, tot, a.tobytes()))
    finally:
        dist.destroy_process_group()


def test_two_ranks_combine_and_shard():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    for _, tot, _ in res:  # every rank sees the same global figures
        assert tot["elapsed_max"] == 2.0 and tot["kernel_ms_max"] == 4.0
        assert tot["iters"] == 30 and tot["ok"] == 15 and tot["keys"] == 14 and tot["frames"] == 16
    assert res[0][2] != res[1][2], "ranks must decode disjoint trials"


def test_single_rank_combine_without_dist():
    import torch

    import bench

    tot = bench.combine_ranks(None, 3.0, 5, 4, 4, 4, 1.5, torch.device("cpu"))
    assert tot == {"elapsed_max": 3.0, "kernel_ms_max": 1.5, "iters": 5.0, "ok": 4.0, "keys": 4.0, "frames": 4.0}
