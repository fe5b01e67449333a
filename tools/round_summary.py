#!/usr/bin/env python3
"""Summaries of a tools/profile_round.sh run for profiles/.

usage: tools/round_summary.py <round_prof_dir> <tag> [round_dir, default r03]
For every workload with passes in <round_prof_dir>: writes
profiles/<round_dir>/<tag>_<wl>_pmc.json (per-launch means of every PMC pass of
the decode kernel), copies the kernel-trace stats CSVs, and refreshes
profiles/pmc_<wl>.json (the HBM traffic bench.py reports: FETCH_SIZE doubled
for gfx950 + WRITE_SIZE, per MI355X_MICROARCH.md's HBM section; the L2 hit
rate TCC_HIT / (TCC_HIT + TCC_MISS) when the tcc pass ran)."""
import glob
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarize  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = ("fetch", "write", "sq", "sq2", "valu", "tcc", "ea", "lds", "stall")


def main(prof, tag, rnd="r03"):
    out_dir = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(out_dir, exist_ok=True)
    f = os.path.join(prof, "default_trace", "run_kernel_stats.csv")
    if os.path.exists(f):
        shutil.copy(f, os.path.join(out_dir, f"{tag}_default_bench_kernel_stats.csv"))
    wls = sorted({os.path.basename(d).rsplit("_", 1)[0] for d in glob.glob(os.path.join(prof, "*_*"))
                  if os.path.isdir(d) and not os.path.basename(d).startswith("default")})
    for wl in wls:
        f = os.path.join(prof, f"{wl}_trace", "run_kernel_stats.csv")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(out_dir, f"{tag}_{wl}_serial_kernel_stats.csv"))
        pmc = {}
        for p in PASSES:
            pmc.update(summarize(prof, "decode_v2", prefix=f"{wl}_{p}"))
        if not pmc:
            continue
        with open(os.path.join(out_dir, f"{tag}_{wl}_pmc.json"), "w") as fh:
            json.dump(pmc, fh, indent=1)
        fetch, write = pmc.get("FETCH_SIZE"), pmc.get("WRITE_SIZE")
        if fetch is None or write is None:
            continue
        path = os.path.join(ROOT, "profiles", f"pmc_{wl}.json")
        cmd = f"python bench.py --workload {wl} ..."
        try:  # the command line rocprofv3 logged for the fetch pass
            for line in open(os.path.join(prof, f"{wl}_fetch.log")):
                if "'python bench.py" in line:
                    cmd = line.split("'")[1]
                    break
        except OSError:
            pass
        summ = {
            "workload": wl,
            "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_* / TCC_* passes (separate runs, --kernel-trace "
                      f"only) of `{cmd}` (tools/profile_round.sh); mean over decode launches; "
                      f"profiles/{rnd}/{tag}_{wl}_pmc.json",
            "correction": "FETCH_SIZE (KB) doubled for gfx950 (MI355X_MICROARCH.md HBM section); WRITE_SIZE (KB) as reported",
            "FETCH_SIZE_KB": fetch,
            "WRITE_SIZE_KB": write,
            "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
            "valu_wave_instructions_per_launch": pmc.get("SQ_INSTS_VALU"),
            # VALU issue cycles (SQ_ACTIVE_INST_VALU, quad-cycles): a
            # transcendental FP64 op (v_rcp_f64) occupies the SIMD 4x as long
            # as a full-rate op (= SQ_INSTS_VALU + 3 * SQ_INSTS_VALU_TRANS_F64)
            "valu_busy_cycles_per_launch": pmc.get("SQ_ACTIVE_INST_VALU"),
        }
        if pmc.get("TCC_HIT_sum") is not None and pmc.get("TCC_MISS_sum") is not None:
            summ["l2_hit_rate"] = pmc["TCC_HIT_sum"] / max(1.0, pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"])
        if pmc.get("SQ_LDS_BANK_CONFLICT") is not None and pmc.get("SQ_ACTIVE_INST_LDS"):
            summ["lds_bank_conflict_per_active_lds"] = pmc["SQ_LDS_BANK_CONFLICT"] / pmc["SQ_ACTIVE_INST_LDS"]
        for k in ("valu_wave_instructions_per_launch", "valu_busy_cycles_per_launch"):
            if summ[k] is None:
                summ.pop(k)
        with open(path, "w") as fh:
            json.dump(summ, fh, indent=1)
        print(wl, json.dumps(summ))


if __name__ == "__main__":
    main(*sys.argv[1:4])
