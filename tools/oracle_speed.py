#!/usr/bin/env python3
"""Single-thread speed of the CPU oracle (the cpu_baseline "port") in ms per
frame-iteration, on the inputs of SURVEY.md §6's probe of the compiled
reference: C2 (n=10k R=0.79) SPA at QBER 2.15% and C3 (n=10k R=0.82) OMSA
beta=0.77 at QBER 1.5%, 50 iterations, threshold 100, trials from the
reference's own generator.  Prints one JSON object; DESIGN.md §5 records it.

  python tools/oracle_speed.py [--frames 48] [--reps 3]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import load_fixture  # noqa: E402
from oracle import pyoracle as P  # noqa: E402

CASES = {  # name: fixture, algorithm, primary, qber, seed, survey ms/frame-iteration (compiled reference, -O3)
    "c2_spa": ("c2_n10240_m2201.alist", 0, 0.0, 0.0215, 1022025, (1.65, 1.9)),
    "c3_omsa": ("c3_n10240_m1801.alist", 3, 0.77, 0.015, 10022025, (0.51, 0.53)),
}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def no_math_split(frames):
    """The C2 SPA loop without its two C-library calls per edge (a copy of the
    oracle built with QLO_TIMING_NO_MATH, run in a child process): ms per
    frame-iteration of everything but tanh / atanh, on 50-iteration frames."""
    import subprocess
    import tempfile

    d = tempfile.mkdtemp()
    so = os.path.join(d, "libqlo_nomath.so")
    od = os.path.join(ROOT, "oracle")
    subprocess.run(["gcc", "-O3", "-std=c11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-DQLO_TIMING_NO_MATH",
                    "-c", os.path.join(od, "ldpc_oracle.c"), "-o", os.path.join(d, "o.o")], check=True)
    subprocess.run(["g++", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-c", os.path.join(od, "trials_oracle.cpp"),
                    "-o", os.path.join(d, "t.o")], check=True)
    subprocess.run(["g++", "-shared", os.path.join(d, "o.o"), os.path.join(d, "t.o"), "-lm", "-lpthread", "-o", so],
                   check=True)
    code = f"""
import sys, time, numpy as np
sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tests')!r})
from conftest import load_fixture
from oracle import pyoracle as P
H = load_fixture("c2_n10240_m2201.alist"); O = P.Oracle(H); p = O.params(0, 50, True, 100.0, 0, 0)
tr = [P.trial(H.n, 0.0215, int(s)) for s in P.trial_seeds(1022025, {frames})]
a = np.stack([t[0] for t in tr]); b = np.stack([t[1] for t in tr]); q = tr[0][2]
lp = np.log((1 - q) / q); llr = np.where(b != 0, -lp, lp); s = H.syndrome(a)
best = 1e9
for _ in range(3):
    t0 = time.perf_counter(); _, it, _, _ = O.decode_batch(p, llr, s, threads=1); dt = time.perf_counter() - t0
    best = min(best, 1e3 * dt / float(it.sum()))
print(best)
"""
    env = dict(os.environ, QLO_LIB_PATH=so)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, check=True)
    return float(r.stdout.split()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=48)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    out = {"host": cpu_model(), "threads": 1, "frames": args.frames, "cases": {}}
    for name, (fx, alg, prim, qber, seed, ref) in CASES.items():
        H = load_fixture(fx)
        O = P.Oracle(H)
        p = O.params(alg, 50, True, 100.0, prim, 0.0)
        seeds = P.trial_seeds(seed, args.frames)
        tr = [P.trial(H.n, qber, int(s)) for s in seeds]
        a = np.stack([t[0] for t in tr])
        b = np.stack([t[1] for t in tr])
        q = tr[0][2]
        lp = np.log((1.0 - q) / q)
        llr = np.where(b != 0, -lp, lp)
        s = H.syndrome(a)
        best = None
        for _ in range(args.reps):
            t0 = time.perf_counter()
            _, it, _, _ = O.decode_batch(p, llr, s, threads=1)
            dt = time.perf_counter() - t0
            ms = 1e3 * dt / float(it.sum())
            best = ms if best is None else min(best, ms)
        rec = {"ms_per_frame_iteration": best, "mean_iterations": float(it.mean()),
               "survey_reference_ms": list(ref), "ratio_to_reference_mid": best / (0.5 * (ref[0] + ref[1]))}
        out["cases"][name] = rec
    # SPA: the loop without the C library's tanh / atanh, in the same session —
    # what the port spends besides the math the reference calls identically
    nm = no_math_split(max(8, args.frames // 3))
    c2 = out["cases"]["c2_spa"]
    c2["ms_per_frame_iteration_without_libm"] = nm
    c2["libm_tanh_atanh_ms_per_frame_iteration"] = c2["ms_per_frame_iteration"] - nm
    print(json.dumps(out))


if __name__ == "__main__":
    main()
