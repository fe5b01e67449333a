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
        # the slicing bench.main uses for its trials (bench.py: rank_trial_seeds)
        seeds = bench.rank_trial_seeds(Q, 1022025, 37, world, rank)
        elapsed = 1.0 + rank  # rank 1 is the slow one
        tot = bench.combine_ranks(dist, elapsed, 10 * (rank + 1), 8 - rank, 7, 8, 2.0 * (rank + 1),
                                  torch.device("cpu"))
        # every rank's slice, gathered over the process group
        mine = torch.from_numpy(seeds.view(np.int64).copy())
        got = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(got, mine)
        q.put((rank, tot, [g.numpy().view(np.uint64).copy() for g in got]))
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
    import qkd_ldpc_v_amd as Q

    full = Q.trial_seeds(1022025, 37 * world)
    for _, _, slices in res:
        assert all(sl.size == 37 for sl in slices)
        # contiguous, complete and in rank order: the concatenation IS the seed list
        assert np.array_equal(np.concatenate(slices), full)
    assert len(set(full.tolist())) == full.size, "ranks must decode disjoint trials"


def test_rank_trial_seeds_slices():
    """bench.rank_trial_seeds at world sizes 1..8: rank r's slice is trials
    [r * batch, (r + 1) * batch) of the reference's seed list."""
    import bench
    import qkd_ldpc_v_amd as Q

    for world in (1, 2, 3, 8):
        full = Q.trial_seeds(1022025, 16 * world)
        parts = [bench.rank_trial_seeds(Q, 1022025, 16, world, r) for r in range(world)]
        assert np.array_equal(np.concatenate(parts), full)
    # rank 0 of a larger job decodes the same first trials as a 1-GPU run
    assert np.array_equal(bench.rank_trial_seeds(Q, 5555, 64, 8, 0), bench.rank_trial_seeds(Q, 5555, 64, 1, 0))


def test_single_rank_combine_without_dist():
    import torch

    import bench

    tot = bench.combine_ranks(None, 3.0, 5, 4, 4, 4, 1.5, torch.device("cpu"))
    assert tot == {"elapsed_max": 3.0, "kernel_ms_max": 1.5, "iters": 5.0, "ok": 4.0, "keys": 4.0, "frames": 4.0}


# ---- device sharding in the product ---------------------------
def test_shard_ranges_contiguous_and_complete():
    from qkd_ldpc_v_amd.simulation import shard_ranges

    for total, shards in [(4097, 3), (10, 1), (2, 3), (0, 2), (4096, 8), (7, 7)]:
        r = shard_ranges(total, shards)
        assert len(r) == shards
        assert r[0][0] == 0 and r[-1][1] == total
        assert all(a[1] == b[0] for a, b in zip(r, r[1:])), "slices must be contiguous"
        per = -(-total // shards)
        assert all(0 <= e - b <= per for b, e in r)


@pytest.mark.gpu
def test_decode_batch_logical_shards_match_oracle(gpu_available):
    """qldpc_decode_batch's multi-device branch — one host thread, stream and
    graph replica per shard, contiguous uneven slices, per-shard error
    collection — exercised with G = 3 logical shards on device 0 and an uneven
    batch of 4097 frames, against the oracle and the single-shard decode."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import qkd_ldpc_v_amd as Q
    from conftest import load_fixture
    from oracle.pyoracle import Oracle

    H = load_fixture("c1_n1024_m220.alist")
    a, b, q = Q.bsc_frames(H.n, 0.03, 4097, seed=31)
    lp = Q.log_p(q)
    llr = np.where(b != 0, -lp, lp).astype(np.float64)
    s = H.syndrome(a)
    p = Q.Params(Q.SPA, 50, True, 100.0)
    g3 = Q.Graph(H, devices=[0, 0, 0])
    assert g3.info()["devices"] == 3
    out3 = g3.decode(p, llr, s, posterior=True)
    out1 = Q.Graph(H).decode(p, llr, s, posterior=True)
    assert np.array_equal(out3.bits, out1.bits) and np.array_equal(out3.iterations, out1.iterations)
    assert np.array_equal(out3.posterior.view(np.uint64), out1.posterior.view(np.uint64))
    O = Oracle(H)
    ob, oi, ok, _ = O.decode_batch(O.params(Q.SPA, 50, True, 100.0), llr, s, threads=16)
    assert np.array_equal(out3.bits, ob) and np.array_equal(out3.iterations, oi) and np.array_equal(out3.synd_ok, ok)
    # errors of any shard surface (no silent partial results)
    with pytest.raises(Q.QLDPCError):
        g3.decode(Q.Params(Q.SPA, 0, True, 100.0), llr, s)


@pytest.mark.gpu
def test_simulation_statistics_independent_of_sharding(gpu_available, tmp_path):
    """simulation.run over 3 logical shards on device 0 gives the same
    per-combination statistics as one shard (uneven slices of 40 trials)."""
    import json

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from qkd_ldpc_v_amd import simulation as S
    from test_simulation import cfg_path, mtrx_dir

    c = json.load(open(cfg_path("legacy_1k")))
    c["trials_number"] = 40
    c["code_rate_QBER_maps"] = [{"code_rate": 0.9, "QBER_begin": 0.02, "QBER_end": 0.03, "QBER_step": 0.01}]
    cp = tmp_path / "c1.json"
    cp.write_text(json.dumps(c))
    cfg = S.Config.load(str(cp))
    d = mtrx_dir(tmp_path, "c1_n1024_m220.alist")
    mats, combos = S.prepare(cfg, S.matrix_files(d))
    r1 = S.run(cfg, mats, combos, log=lambda *a: None)
    r3 = S.run(cfg, mats, combos, log=lambda *a: None, devices=[0, 0, 0])
    drop = ("tp_mean", "tp_std", "tp_min", "tp_max")
    strip = lambda rs: [{k: v for k, v in r.items() if k not in drop} for r in rs]  # noqa: E731
    assert strip(r1) == strip(r3)


# ---- bench.py --gpus N: the N-rank launch itself (verdict r05, item 1) ----------
def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


def test_bench_gpus_n_refuses_fewer_devices():
    """`bench.py --gpus 2` on a node with fewer than 2 GPUs exits non-zero
    (it must never decode on one rank and print a 1-GPU line)."""
    import subprocess

    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("node has >= 2 GPUs")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=_bench_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "needs 2 GPUs" in r.stderr
    assert r.stdout.strip() == "", "no JSON line may be printed"


def test_bench_world_size_must_equal_gpus():
    """Under a launcher, WORLD_SIZE and --gpus must agree."""
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=_bench_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                                      MASTER_PORT=str(_free_port())),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "disagrees with --gpus 2" in r.stderr


def test_spawn_ranks_starts_one_process_per_rank(tmp_path):
    """bench.spawn_ranks starts `world` processes with torchrun's one-node
    environment (RANK = LOCAL_RANK = r, WORLD_SIZE, one MASTER_PORT)."""
    import json

    import bench

    script = ("import json, os, sys; "
              "json.dump({k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', "
              "'MASTER_ADDR', 'MASTER_PORT')}, open(os.path.join(sys.argv[1], os.environ['RANK'] + '.json'), 'w'))")
    rc = bench.spawn_ranks(3, [sys.executable, "-c", script, str(tmp_path)], base_env=_bench_env())
    assert rc == 0
    got = [json.load(open(tmp_path / f"{r}.json")) for r in range(3)]
    assert [g["RANK"] for g in got] == ["0", "1", "2"] and [g["LOCAL_RANK"] for g in got] == ["0", "1", "2"]
    assert {g["WORLD_SIZE"] for g in got} == {"3"} and {g["LOCAL_WORLD_SIZE"] for g in got} == {"3"}
    assert {g["MASTER_ADDR"] for g in got} == {"127.0.0.1"} and len({g["MASTER_PORT"] for g in got}) == 1


def test_spawn_ranks_failure_ends_the_job():
    """A failing rank's exit code is the job's, and the ranks still waiting
    (at a barrier, in a real run) are terminated rather than left hanging."""
    import time

    import bench

    script = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(3) if r == 1 else time.sleep(600)"
    t0 = time.time()
    rc = bench.spawn_ranks(3, [sys.executable, "-c", script], base_env=_bench_env())
    assert rc == 3
    assert time.time() - t0 < 60


def _bench_line(args, env=None, launcher=False):
    import json
    import subprocess

    cmd = [sys.executable]
    if launcher:
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr", "127.0.0.1",
                "--master-port", str(_free_port())]
    cmd += [os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, env=env or _bench_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


_SMALL = ["--workload", "c1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--roofline-launches", "1"]


@pytest.mark.gpu
def test_bench_two_ranks_sum_to_one_rank_of_double_batch(gpu_available):
    """`bench.py --gpus 2` (no launcher: bench spawns the ranks; both on
    device 0 via --share-device, as a one-GPU box has no second card) decodes
    rank slices [0, 64) and [64, 128) of the seed list: its summed counters
    equal a 1-rank run of batch 128, n_gpus == 2 and global_batch == 2 x 64."""
    two = _bench_line(["--gpus", "2", "--share-device", "--batch", "64"] + _SMALL)
    one = _bench_line(["--gpus", "1", "--batch", "128"] + _SMALL)
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["global_batch"] == 128 and two["config"]["batch_per_gpu"] == 64
    assert one["config"]["global_batch"] == 128
    for k in ("fer", "key_mismatch_rate", "mean_iterations"):
        assert two[k] == one[k], k


@pytest.mark.gpu
def test_bench_under_launcher_runs_the_rccl_bracket(gpu_available):
    """torchrun with one rank: the process group (RCCL), its barriers and the
    max/sum combine run; the counters equal a plain 1-GPU run's."""
    ln = _bench_line(["--gpus", "1", "--batch", "64"] + _SMALL, launcher=True)
    plain = _bench_line(["--gpus", "1", "--batch", "64"] + _SMALL)
    assert ln["n_gpus"] == 1 and ln["config"]["global_batch"] == 64
    for k in ("fer", "key_mismatch_rate", "mean_iterations"):
        assert ln[k] == plain[k], k


def test_spawn_ranks_stopped_launcher_stops_the_ranks(tmp_path):
    """SIGTERM to the process running bench.spawn_ranks (a launcher's time
    limit) terminates its ranks instead of leaving them on the GPUs."""
    import signal
    import subprocess
    import time

    pidfile = tmp_path / "pids"
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            "bench.spawn_ranks(2, [sys.executable, '-c', "
            f"\"import os, time; open({str(pidfile)!r}, 'a').write(str(os.getpid()) + '\\\\n'); time.sleep(600)\"])")
    parent = subprocess.Popen([sys.executable, "-c", code], env=_bench_env())
    for _ in range(200):
        if pidfile.exists() and len(pidfile.read_text().split()) == 2:
            break
        time.sleep(0.1)
    pids = [int(x) for x in pidfile.read_text().split()]
    assert len(pids) == 2
    parent.send_signal(signal.SIGTERM)
    parent.wait(timeout=60)
    time.sleep(0.5)
    for pid in pids:
        try:
            os.kill(pid, 0)
            alive = open(f"/proc/{pid}/stat").read().split()[2] != "Z"
        except (ProcessLookupError, FileNotFoundError):
            alive = False
        assert not alive, f"rank {pid} survived its launcher"
