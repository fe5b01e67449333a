#!/bin/bash
# Round 6: every split plan shape the planner chooses between, under the
# product's two-in-flight rule (same box, 2 reps alternating): part size
# (QLDPC_SPLIT_WP 8 / 16) x scratch slots (QLDPC_SPLIT_SCRATCH 0 / 1), C4
# stand-in and C4 (ii).  Knobs under QLDPC_DIAG=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export QLDPC_DIAG=1
O=gpurun_out/r06_split_plans; mkdir -p $O
run() {  # name, workload, env...
  local name=$1 wl=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $wl --steps 8 --warmup 2 --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/$name.json'))
print('$name', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), 'lanes', d['config']['lanes_per_frame'], 'epl', d['config']['edges_per_lane'])"
}
for rep in 1 2; do
  for wl in c4 c4g; do
    for wp in 8 16; do
      for sc in 0 1; do
        run ${wl}_wp${wp}_s${sc}_$rep $wl QLDPC_SPLIT_WP=$wp QLDPC_SPLIT_SCRATCH=$sc
      done
    done
  done
done
