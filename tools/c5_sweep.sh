#!/bin/bash
# The 26-point C5 sweep (bench.py --workload c5ra --c5-point i), one bench line
# per point under gpurun_out/c5sweep[_b$BATCH]/, then a summary JSON.
# BATCH=512 runs the BASELINE C5 shape per GPU (4096 frames over 8 GPUs).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
B=${BATCH:-4096}
O=gpurun_out/c5sweep${BATCH:+_b$BATCH}; mkdir -p $O
for i in $(seq 0 25); do
  timeout -k 10 120 python bench.py --workload c5ra --c5-point $i --batch $B --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline \
      --roofline-launches 1 > $O/point_$i.json 2> $O/point_$i.err || { tail -5 $O/point_$i.err; exit 3; }
  echo "point $i done"
done
python - "$O" "$B" <<'PY'
import json, sys
pts = [json.load(open(f"{sys.argv[1]}/point_{i}.json")) for i in range(26)]
rows = [{"point": i, "workload": p["config"]["workload"], "gbit_s": p["value"] / 1e9, "ms_per_step": p["ms_per_step"],
         "fer": p["fer"], "mean_iterations": p["mean_iterations"], "info_bits_per_frame": p["config"]["info_bits_per_frame"],
         "kernel_variant": p["config"]["kernel_variant"],
         # the line's own algorithmic-byte model ((2E + 2n) * 8 B per frame-iteration / 8 TB/s)
         "hbm_model_frac": p.get("hbm_model_roofline", p["roofline"])["frac"],
         # VALU issue fraction only where a PMC pass of THIS point exists (profiles/pmc_c5ra_p<i>.json)
         "valu_issue_frac": p["compute_roofline"]["frac"] if "compute_roofline" in p else None}
        for i, p in enumerate(pts)]
tot_bits = sum(r["gbit_s"] * r["ms_per_step"] for r in rows)
tot_ms = sum(r["ms_per_step"] for r in rows)
out = {"sweep": "configs/ADAPTIVE T.json, 26 points, AOMSA, rate-adapted, batch " + sys.argv[2] + "/GPU, 1 GPU", "points": rows,
       "aggregate_gbit_s": tot_bits / tot_ms}
json.dump(out, open(f"{sys.argv[1]}/summary.json", "w"), indent=1)
for r in rows:
    print(r["point"], round(r["gbit_s"], 3), round(r["ms_per_step"], 1), r["fer"], round(r["mean_iterations"], 2), r["kernel_variant"])
print("aggregate Gbit/s", round(out["aggregate_gbit_s"], 3))
PY
