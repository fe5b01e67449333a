#!/usr/bin/env python3
"""Decoded info-bits/s of the QKD-LDPC decode hot path on MI355X.

A step = the reference's per-trial window (QKD_LDPC, src/qkd_ldpc_algorithm.cpp:
1031-1087; timed like src/simulation.cpp:559-568) for one batch of frames:
LLR build + Alice syndrome on device, the BP decode, the key comparison.  The
trials (synthetic BSC keys) are generated before timing and are resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c1|c4]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

One process per GPU.  `--gpus N > 1` without a launcher starts the N ranks
itself (child processes, before this process touches the GPU) with the same
environment torchrun would give them; under a launcher WORLD_SIZE must equal
N.  Either way the run exits non-zero when the node has fewer than N GPUs, so
`--gpus N` never silently measures fewer ranks.  Frames are sharded across
ranks with no data-path collective (weak scaling: every GPU decodes its own
batch); a barrier + max-over-ranks bracket the timed region.  Rank 0 prints
one JSON line.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded info-bits/sec (whole node), n=10k R=0.8 SPA 50-iter, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# Highest VALU issue rate measured on MI355X (issue slots/s, whole chip):
# tools/valu_bench.hip's SPA edge-math loop at 2.30 GHz (profiles/r04/
# valu_microbench_r04.json).  Dense v_fma_f64 chains reach only 4.4-5.1e11
# because the chip lowers its clock to 1.95-2.2 GHz on them; the decode
# kernels run at 2.3 GHz, so that rate understated their peak.
VALU_PEAK_WAVE_INSTR = 5.73e11

WORKLOADS = {
    # name: matrix fixture, format, algorithm, primary, secondary, qber, batch/GPU, description
    "c2": ("c2_n10240_m2201.alist", 1, 0, 0.0, 0.0, 0.0215, 4096,
           "C2: n=10k R=0.8 SPA 50-iter, batch 4096/GPU (configs_all/config 10k SPA FER=0.01.json bucket 0.795)"),
    "c3": ("c3_n10240_m1801.alist", 1, 3, 0.77, 0.0, 0.015, 4096,
           "C3: n=10k R=0.82 OMSA beta=0.77 50-iter, batch 4096/GPU"),
    "c1": ("c1_n1024_m220.alist", 1, 0, 0.0, 0.0, 0.013, 4096, "C1: n=1k R~0.8 SPA 50-iter"),
    "c4": ("c4s_n102400_m32001.alist", 1, 0, 0.0, 0.0, 0.038, 128,
           "C4 stand-in: n=100k R=0.69 SPA 50-iter, batch 128/GPU (R=0.79 file absent upstream)"),
    # the R=0.79 dv=4 file is absent upstream; a seeded
    # build-generated code of its shape (qkd_ldpc_v_amd/codes.py), QBER 0.022
    "c4g": (None, 0, 0, 0.0, 0.0, 0.022, 128,
            "C4 (ii): generated regular dv=4 n=102400 m=22001 R=0.785 (seed 777) SPA 50-iter, batch 128/GPU"),
    "c5": ("c5_n10240_m2048.sp2", 3, 5, 0.7, 0.99, 0.0156, 4096,
           "C5 decode: n=10k R=0.8 irregular (matrices_2, format 3) AOMSA beta=0.7 sigma=0.99 "
           "(configs/ADAPTIVE T.json, rate bucket 0.805) 50-iter, QBER 1.56%, batch 4096/GPU, no rate adaptation"),
    "c5ra": ("c5_n10240_m2048.sp2", 3, 5, 0.7, 0.99, 0.0156, 4096,
             "C5: n=10k R=0.8 irregular, rate-adapted (untainted puncturing, QBER 1.56%, delta 0.06, f_EC 1.39 -> "
             "configs/ADAPTIVE T.json), AOMSA beta=0.7 sigma=0.99 50-iter, batch 4096/GPU"),
}


# SIMULATION_SEED of the config each workload comes from (configs_all/*.json).
SIMULATION_SEEDS = {"c1": 9012025, "c2": 1022025, "c3": 10022025}
RATE_ADAPT = {"c5ra": (0.06, 1.39, "c5_n10240_m2048.untp")}  # delta, efficiency, untainted list

# The C5 sweep: configs/ADAPTIVE T.json's 26 (code rate,
# QBER, delta, f_EC) points (:102-130) with AOMSA beta / sigma per code rate
# (:51-76) and the format-3 matrices of sparse_matrices/matrices_2.
C5_MATRIX = {0.805: "c5_n10240_m2048", 0.655: "c5b_n10240_m3584", 0.505: "c5c_n10240_m5120"}
C5_BETA_SIGMA = {0.805: (0.7, 0.99), 0.655: (0.74, 0.94), 0.505: (0.72, 0.85)}
C5_POINTS = [
    (0.805, 0.0076, 0.10, 1.85), (0.805, 0.0116, 0.09, 1.50), (0.805, 0.0156, 0.06, 1.39),
    (0.805, 0.0196, 0.03, 1.28), (0.805, 0.0236, 0.01, 1.21), (0.805, 0.0276, 0.11, 1.20),
    (0.805, 0.0316, 0.22, 1.22), (0.655, 0.0368, 0.12, 1.22), (0.655, 0.0408, 0.10, 1.20),
    (0.655, 0.0448, 0.06, 1.18), (0.655, 0.0488, 0.06, 1.17), (0.655, 0.0528, 0.01, 1.16),
    (0.655, 0.0568, 0.06, 1.16), (0.655, 0.0608, 0.11, 1.17), (0.655, 0.0648, 0.16, 1.17),
    (0.655, 0.0688, 0.23, 1.19), (0.505, 0.0734, 0.12, 1.18), (0.505, 0.0774, 0.09, 1.17),
    (0.505, 0.0814, 0.08, 1.16), (0.505, 0.0854, 0.04, 1.15), (0.505, 0.0894, 0.01, 1.14),
    (0.505, 0.0934, 0.03, 1.14), (0.505, 0.0974, 0.06, 1.14), (0.505, 0.1014, 0.10, 1.15),
    (0.505, 0.1054, 0.13, 1.16), (0.505, 0.1094, 0.13, 1.15),
]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="frames per GPU (default: the workload's)")
    ap.add_argument("--max-iterations", type=int, default=50)
    ap.add_argument("--streams", type=int, default=2,
                    help="HIP streams the steps alternate over: step i+1's frames start on CUs freed by "
                         "step i's last frames (1 = strictly serial steps)")
    ap.add_argument("--roofline-launches", type=int, default=3,
                    help="serial decode launches after the timed region, timed alone for the roofline (with "
                         "--streams > 1 a timed step's decode shares CUs with its neighbours)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c5-point", type=int, default=-1,
                    help="with --workload c5ra: one of the 26 C5 sweep points (C5_POINTS index)")
    ap.add_argument("--share-device", action="store_true",
                    help="test only: every rank on device 0 (logical devices), gloo for the bracket collectives "
                         "(RCCL refuses two ranks on one GPU); the line's timing is then not a node figure")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")

    import torch

    launched = "WORLD_SIZE" in os.environ
    if not launched and args.gpus > 1:
        # no launcher: start the N ranks here, before any GPU call in this process
        check_devices(torch.cuda.device_count(), args.gpus, args.share_device)
        sys.exit(spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} from the launcher disagrees with --gpus {args.gpus}")
    check_devices(torch.cuda.device_count(), world, args.share_device)
    if args.share_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if launched:  # also at WORLD_SIZE 1 (torchrun --nproc-per-node 1): the same bracket and combine
        import torch.distributed as dist

        if args.share_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    import qkd_ldpc_v_amd as Q

    fixture, fmt, alg, prim, sec, qber, batch, desc = WORKLOADS[args.workload]
    batch = args.batch or batch
    ra = RATE_ADAPT.get(args.workload)
    if args.c5_point >= 0:
        if args.workload != "c5ra":
            raise SystemExit("--c5-point needs --workload c5ra")
        crate, qber, delta, eff = C5_POINTS[args.c5_point]
        fixture = C5_MATRIX[crate] + ".sp2"
        prim, sec = C5_BETA_SIGMA[crate]
        ra = (delta, eff, C5_MATRIX[crate] + ".untp")
        desc = (f"C5 sweep point {args.c5_point}: code rate {crate} ({fixture}), QBER {qber}, delta {delta}, "
                f"f_EC {eff}, AOMSA beta={prim} sigma={sec} 50-iter, batch {batch}/GPU (configs/ADAPTIVE T.json)")
    if fixture is None:
        H = Q.regular_code(102400, 22001, 4, 777)
    else:
        H = Q.load_matrix(os.path.join(ROOT, "tests", "golden", "matrices", fixture + ".gz"), fmt)
    n, m, E = H.n, H.m, H.nnz
    k_info = n - m
    g = Q.Graph(H)
    plan = g.plan(local, alg)
    params = Q.Params(alg, args.max_iterations, True, 100.0, prim, sec)

    # ---- trials (not timed): run_trial's keys, generated on device and resident in HBM ----
    # The reference's generator (src/simulation.cpp:540-551,713-719,743):
    # per-trial seeds drawn from Xoshiro256++(SIMULATION_SEED); each rank takes
    # its own contiguous slice of trials.
    sim_seed = 5555 if args.c5_point >= 0 else SIMULATION_SEEDS.get(args.workload, 1022025)  # ADAPTIVE T.json:5
    seeds = rank_trial_seeds(Q, sim_seed, batch, world, rank)
    d_seeds = torch.from_numpy(seeds.view(np.int64)).to(dev)
    ta = torch.empty((batch, n), dtype=torch.uint8, device=dev)
    tb = torch.empty((batch, n), dtype=torch.uint8, device=dev)
    if ra:  # adapt_code_rate on the host, then the rate-adapted trials
        import gzip

        untp = np.array(gzip.open(os.path.join(ROOT, "tests", "golden", "matrices", ra[2] + ".gz")).read().split(),
                        np.int32)
        punct, short, rate = Q.adapt_code_rate(n, m, qber, ra[0], ra[1], untp, Q.xoshiro_state(sim_seed))
        rplan = g.rate_plan(punct, short)
        pa = torch.empty((batch, max(1, punct.size)), dtype=torch.uint8, device=dev)
        pb = torch.empty_like(pa)
        tax = torch.empty((batch, n), dtype=torch.uint8, device=dev)  # Alice's extended key
        k_info = n - m - short.size  # information bits of the adapted code
        desc += f" [p={punct.size} s={short.size} R={rate:.4f}]"
    def generate():
        if ra:
            return Q.trials_rate_adapt_device(n, qber, d_seeds, punct.size, ta, tb, pa, pb)
        return Q.trials_device(n, qber, d_seeds, ta, tb)

    # untimed by the metric (the reference's window starts after run_trial's
    # keys exist, src/simulation.cpp:559); reported: the first call (it also
    # builds the generator's jump table) and a warm call
    gen_s = []
    for _ in range(2):
        torch.cuda.synchronize()
        tg0 = time.perf_counter()
        q_acc = generate()
        torch.cuda.synchronize()
        gen_s.append(time.perf_counter() - tg0)
    trial_gen_first_s, trial_gen_s = gen_s
    lp = Q.log_p(q_acc)
    tlp = torch.full((batch,), lp, dtype=torch.float64, device=dev)
    nst = max(1, args.streams)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nst - 1)]

    class Slot:  # per-stream frame workspace and outputs
        def __init__(self, s):
            self.stream = s
            # no f64 LLR workspace: the register decoders read the frame builder's
            # palette codes, so the fused entry skips the LLR write (NULL llr_ws)
            self.llr_ws = None
            self.syn_ws = torch.empty((batch, m), dtype=torch.uint8, device=dev)
            self.bits = torch.empty((batch, n), dtype=torch.uint8, device=dev)
            self.iters = torch.empty(batch, dtype=torch.int32, device=dev)
            self.ok = torch.empty(batch, dtype=torch.uint8, device=dev)
            self.km = torch.empty(batch, dtype=torch.uint8, device=dev)

    slots = [Slot(s) for s in streams]
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]

    def step(i, sl=None):
        """One batch through the fused per-trial window entry: frame build (LLR
        palette codes + Alice syndrome) -> decode -> key compare, all enqueued
        by the library on the slot's stream (no palettize pass: the frame
        builder writes the decoder's palette form directly)."""
        sl = sl or slots[i % nst]
        if ra:  # QKD_LDPC_RATE_ADAPT (src/qkd_ldpc_algorithm.cpp:1121-1218)
            g.qkd_ldpc_rate_adapt_device(rplan, params, ta, tb, pa, pb, tlp, tax, sl.llr_ws, sl.syn_ws, sl.bits,
                                         sl.iters, sl.ok, sl.km, stream=sl.stream)
        else:  # QKD_LDPC (:1031-1087)
            g.qkd_ldpc_device(params, ta, tb, tlp, sl.llr_ws, sl.syn_ws, sl.bits, sl.iters, sl.ok, sl.km,
                              stream=sl.stream)

    log(f"[rank {rank}] {desc}; plan {plan}; warmup {args.warmup}")
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        sl = slots[i % nst]
        ev0[i].record(sl.stream)
        step(i)
        ev1[i].record(sl.stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    step_ms_stream = float(np.mean([ev0[i].elapsed_time(ev1[i]) for i in range(args.steps)]))
    # Roofline: the decode kernel alone — a few serial steps on one stream with
    # the library's kernel timing on (HIP events around the decode kernel
    # launch only, on the stream it runs on), outside the timed region.
    kernel_ms = None
    if args.roofline_launches > 0:
        g.set_kernel_timing(True)
        kms = []
        for j in range(args.roofline_launches):
            step(j, slots[0])
            kms.append(g.last_decode_kernel_ms(slots[0].stream, local))
        g.set_kernel_timing(False)
        kernel_ms = float(np.mean(kms))
        # (the roofline steps decode the same trials as the timed ones)

    last = slots[(args.steps - 1) % nst]  # every step decodes the same trials
    it_sum = int(last.iters.to(torch.int64).sum().item())
    n_ok = int(last.ok.to(torch.int64).sum().item())
    n_keys = int(last.km.to(torch.int64).sum().item())
    tot = combine_ranks(dist, elapsed, it_sum, n_ok, n_keys, batch, kernel_ms or 0.0,
                        torch.device("cpu") if args.share_device else dev)
    elapsed_max, kernel_ms_max = tot["elapsed_max"], tot["kernel_ms_max"]
    it_total, ok_total, keys_total, frames_step = tot["iters"], tot["ok"], tot["keys"], tot["frames"]

    if rank == 0:
        frames_total = frames_step * args.steps
        value = frames_total * k_info / elapsed_max
        B = 8.0 * (2 * E + 2 * n)  # algorithmic bytes per frame-iteration
        # per-launch algorithmic bytes of THIS rank's decode kernel / its mean
        # duration (the serial roofline launches; without them, the timed
        # steps' per-stream step time, which also holds the frame build)
        kms = kernel_ms if kernel_ms else step_ms_stream
        achieved = (it_sum * B) / (kms * 1e-3) / 1e9
        traffic = None
        valu_per_launch = valu_busy = None
        # counters of THIS workload's kernel only: a C5 sweep point is priced by
        # a PMC pass of that point (profiles/pmc_c5ra_p<i>.json) or by its byte
        # model alone — never by another point's counts
        pmc_name = f"pmc_c5ra_p{args.c5_point}.json" if args.c5_point >= 0 else f"pmc_{args.workload}.json"
        pmc = os.path.join(ROOT, "profiles", pmc_name)
        if os.path.exists(pmc):
            with open(pmc) as f:
                pm = json.load(f)
            traffic = pm.get("hbm_bytes_per_launch")
            valu_per_launch = pm.get("valu_wave_instructions_per_launch")
            valu_busy = pm.get("valu_busy_cycles_per_launch")
        res = {
            "metric": METRIC,
            "value": value,
            "unit": "info-bits/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic sifted keys from the reference's own trial generator (Xoshiro256++ seeds, "
                    "exactly floor(n*QBER) errors, libstdc++ draw semantics) run on device, untimed; "
                    + ("reference parity-check matrix file" if fixture else
                       "seeded generated parity-check matrix (the reference's file is absent upstream)"),
            "trial_generation_s": trial_gen_s,
            "trial_generation_first_call_s": trial_gen_first_s,
            "config": {
                "workload": desc, "matrix": fixture or "generated: regular_code(102400, 22001, 4, 777)", "n": n, "m": m, "edges": E, "info_bits_per_frame": k_info,
                "algorithm": Q.ALGORITHM_NAMES[alg], "qber": qber, "max_iterations": args.max_iterations,
                "batch_per_gpu": batch, "global_batch": int(frames_step),
                "parallelism": (f"frames sharded over {world} ranks on ONE GPU (--share-device test run), "
                                "no collectives" if args.share_device else
                                f"frames sharded over {world} GPU(s), no collectives"),
                "kernel_variant": plan["variant"], "lanes_per_frame": plan["lanes"], "streams": nst,
                "edges_per_lane": plan["edges_per_lane"], "workgroups": plan["workgroups"],
            },
            "fer": 1.0 - ok_total / frames_step,
            "key_mismatch_rate": 1.0 - keys_total / frames_step,
            "mean_iterations": it_total / frames_step,
            "decode_kernel_ms": kernel_ms,
            "decode_kernel_ms_max_rank": kernel_ms_max,
            "step_ms_per_stream_pipelined": step_ms_stream,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "bytes_per_frame_iteration": B,
            },
            "cpu_baseline": None,
        }
        if valu_per_launch:
            # The decode kernel keeps messages on chip: it is bound by FP64 VALU
            # issue, not HBM.  VALU issue cycles per launch from the PMC pass
            # (profiles/pmc_<workload>.json: SQ_ACTIVE_INST_VALU, where a
            # v_rcp_f64 counts 4 like its issue time; SQ_INSTS_VALU if absent)
            # over this run's kernel time, against the whole-chip rate of
            # VALU issue slots tools/valu_bench.hip measures
            # (profiles/r04/valu_microbench_r04.json).
            busy = valu_busy or valu_per_launch
            ach = busy / (kms * 1e-3)
            res["compute_roofline"] = {"bound": "fp64-valu-issue", "achieved": ach, "peak": VALU_PEAK_WAVE_INSTR,
                                       "unit": "VALU issue cycles (full-rate wave-instruction slots)/s",
                                       "frac": ach / VALU_PEAK_WAVE_INSTR,
                                       "valu_wave_instructions_per_launch": valu_per_launch,
                                       "valu_busy_cycles_per_launch": valu_busy}
            if alg >= 2:
                # Min-sum: the (2E + 2n) * 8 B streaming model runs at or above
                # 8 TB/s (C3: 1.05) because the kernel never streams messages,
                # so it is no bound; the line's roofline is the binding one,
                # VALU issue, and the byte model is kept beside it.
                res["hbm_model_roofline"] = res["roofline"]
                res["roofline"] = dict(res["compute_roofline"], traffic=traffic)
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(H, alg, prim, sec, qber, args.max_iterations,
                                               args.cpu_baseline_seconds, k_info,
                                               SIMULATION_SEEDS.get(args.workload, 1022025) + 1,
                                               (punct, short) if ra else None)
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def check_devices(have: int, need: int, shared: bool) -> None:
    """Refuse a run that would measure fewer GPUs than asked for."""
    if have < (1 if shared else need):
        raise SystemExit(f"bench.py: --gpus {need} needs {need} GPUs, this node has {have}")


def rank_env(base: dict, world: int, rank: int, port: int) -> dict:
    """The environment torch.distributed.run gives rank `rank` of a one-node job."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(world: int, cmd: list, base_env=None) -> int:
    """Run `cmd` as ranks 0..world-1 (child processes, one per GPU) and wait
    for all of them.  If one fails, the others are terminated (they would wait
    at the barrier forever).  Returns the first non-zero exit code, else 0."""
    import signal

    port = free_port()
    base = dict(os.environ if base_env is None else base_env)
    procs = []
    # a launcher that stops this process (its time limit: SIGTERM) stops the
    # ranks too, so no rank is left holding a GPU
    def _stop(signum, _frame):
        raise SystemExit(128 + signum)

    prev = {sig: signal.signal(sig, _stop) for sig in (signal.SIGTERM, signal.SIGHUP)}
    try:
        procs = [subprocess.Popen(cmd, env=rank_env(base, world, r, port)) for r in range(world)]
        rc = 0
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in pending:
                        q.terminate()
            time.sleep(0.05)
        return rc
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        for sig, h in prev.items():
            signal.signal(sig, h)


def rank_trial_seeds(Q, sim_seed: int, batch: int, world: int, rank: int):
    """The per-trial seeds a rank decodes: the reference's seed list for
    batch * world trials (src/simulation.cpp:713-719), cut into contiguous
    slices of `batch`, slice `rank` per rank (weak scaling, disjoint trials)."""
    return Q.trial_seeds(sim_seed, batch * world)[rank * batch:(rank + 1) * batch]


def combine_ranks(dist, elapsed, it_sum, n_ok, n_keys, frames, kernel_ms, device):
    """Max over ranks of the timed region, sums of the per-rank counters: the
    only collectives of the run, after the timed region (no data-path
    exchange; frames are independent)."""
    import torch

    stats = torch.tensor([elapsed, it_sum, n_ok, n_keys, frames, kernel_ms], dtype=torch.float64, device=device)
    mx = stats.clone()
    if dist is not None:
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(stats, op=dist.ReduceOp.SUM)
    return {"elapsed_max": float(mx[0]), "kernel_ms_max": float(mx[5]), "iters": float(stats[1]),
            "ok": float(stats[2]), "keys": float(stats[3]), "frames": float(stats[4])}


def host_cpus():
    """The host CPUs this job may use: nproc (os.cpu_count), the affinity mask,
    the cgroup CPU quota, and the CPU model (/proc/cpuinfo)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):  # cgroup v2: "<quota> <period>" or "max <period>"
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "usable": usable, "model": model}


def cpu_baseline(H, alg, prim, sec, qber, max_it, seconds, k_info, seed, rate_adapt=None):
    """The CPU oracle (a port of the reference decoder, glibc math, one frame per
    task on a thread pool like src/simulation.cpp:721,740-746) on a bounded
    sample of the same workload: chunks of frames until `seconds` elapse, on
    every host CPU this job may use (value), then on one thread (value_1thread,
    a third of the time budget).  rate_adapt = (punctured, shortened): the
    frames are QKD_LDPC_RATE_ADAPT's extended frames, as on the GPU."""
    from oracle import pyoracle as P
    from oracle.pyoracle import Oracle

    cpus = host_cpus()
    O = Oracle(H)
    p = O.params(alg, max_it, True, 100.0, prim, sec)
    seeds = P.trial_seeds(seed, 1 << 16)

    def sample(threads, budget, start):
        chunk = threads * 4
        frames, t_dec = 0, 0.0
        while t_dec < budget and start + frames + chunk <= seeds.size:
            sds = seeds[start + frames:start + frames + chunk]
            if rate_adapt is None:
                tr = [P.trial(H.n, qber, int(sd)) for sd in sds]  # untimed
                a = np.stack([t[0] for t in tr])
                b = np.stack([t[1] for t in tr])
                q = tr[0][2]
                t0 = time.perf_counter()
                lp = math.log((1.0 - q) / q)
                llr = np.where(b != 0, -lp, lp)
            else:  # the extended frame (its LLRs come with the draws; the build is O(n) either way)
                tr = [P.trial_rate_adapt(H.n, qber, int(sd), rate_adapt[0], rate_adapt[1]) for sd in sds]
                a = np.stack([t[0] for t in tr])
                llr = np.stack([t[1] for t in tr])
                t0 = time.perf_counter()
            s = H.syndrome(a)
            bits, it, ok, _ = O.decode_batch(p, llr, s, threads=threads)
            (bits == a).all(axis=1)
            t_dec += time.perf_counter() - t0
            frames += chunk
        return frames, t_dec

    threads = cpus["usable"]
    frames, t_all = sample(threads, seconds, 0)
    f1, t1 = sample(1, seconds / 3.0, frames)
    return {"value": frames * k_info / t_all, "unit": "info-bits/s", "cores": threads, "kind": "port",
            "value_1thread": f1 * k_info / t1 if t1 > 0 else None,
            "host": cpus,
            "sample": f"{frames} frames of the same workload (chunks of {threads * 4}), {t_all:.1f} s, "
                      f"oracle/ldpc_oracle.c on {threads} host threads (all CPUs this job may use: nproc "
                      f"{cpus['nproc']}, affinity {cpus['affinity']}, cgroup quota {cpus['cgroup_quota']}; "
                      f"{cpus['model']}); 1 thread: {f1} frames in {t1:.1f} s"}


if __name__ == "__main__":
    main()
