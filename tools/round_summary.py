#!/usr/bin/env python3
"""Summaries of a tools/profile_round.sh run for profiles/.

usage: tools/round_summary.py <round_prof_dir> <tag> [round_dir, default r02]
Writes profiles/<round_dir>/<tag>_{c2,c3}_pmc.json (per-launch means of every PMC
pass), copies the kernel-trace stats CSVs, and refreshes profiles/pmc_<wl>.json
(the HBM traffic bench.py reports: FETCH_SIZE doubled for gfx950 + WRITE_SIZE,
per MI355X_MICROARCH.md's HBM section)."""
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarize  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(prof, tag, rnd="r02"):
    out_dir = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(out_dir, exist_ok=True)
    for src, dst in (("default_trace", "default_bench"), ("c2_trace", "c2_serial"), ("c3_trace", "c3_serial")):
        f = os.path.join(prof, src, "run_kernel_stats.csv")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(out_dir, f"{tag}_{dst}_kernel_stats.csv"))
    for wl in ("c2", "c3"):
        pmc = {}
        for p in ("fetch", "write", "sq", "sq2", "valu"):
            pmc.update(summarize(prof, "decode_v2", prefix=f"{wl}_{p}"))
        if not pmc:
            continue
        with open(os.path.join(out_dir, f"{tag}_{wl}_pmc.json"), "w") as fh:
            json.dump(pmc, fh, indent=1)
        fetch, write = pmc.get("FETCH_SIZE"), pmc.get("WRITE_SIZE")
        if fetch is None or write is None:
            continue
        summ = {
            "workload": wl,
            "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_* passes (separate runs, --kernel-trace only) "
                      f"of `python bench.py --workload {wl} --steps 5 --warmup 1 --no-cpu-baseline --streams 1 "
                      "--roofline-launches 0` (tools/profile_round.sh); mean over decode launches; "
                      f"profiles/{rnd}/{tag}_{wl}_pmc.json",
            "correction": "FETCH_SIZE (KB) doubled for gfx950 (MI355X_MICROARCH.md HBM section); WRITE_SIZE (KB) as reported",
            "FETCH_SIZE_KB": fetch,
            "WRITE_SIZE_KB": write,
            "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
            "valu_wave_instructions_per_launch": pmc.get("SQ_INSTS_VALU"),
        }
        with open(os.path.join(ROOT, "profiles", f"pmc_{wl}.json"), "w") as fh:
            json.dump(summ, fh, indent=1)
        print(wl, json.dumps(summ))


if __name__ == "__main__":
    main(*sys.argv[1:4])
