#!/bin/bash
# Round 6: 16-wave split parts with the scratch slots (fewer parts per frame at
# the same frames per XCD): C4 (ii) K = 8 x 16 waves vs the planner's 16 x 8;
# the stand-in K = 6 x 16 waves (5 frames per XCD) vs its 15 x 8 without
# scratch slots.  Knobs under QLDPC_DIAG=1, same box, 2 reps alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export QLDPC_DIAG=1
O=gpurun_out/r06_wp16rg; mkdir -p $O
run() {  # name, workload, env...
  local name=$1 wl=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $wl --steps 8 --warmup 2 --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/$name.json'))
print('$name', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), d['config']['lanes_per_frame'], d['config']['edges_per_lane'])"
}
for rep in 1 2; do
  run c4g_default_$rep c4g QLDPC_DIAG=1
  run c4g_wp16_$rep c4g QLDPC_SPLIT_WP=16
  run c4_default_$rep c4 QLDPC_DIAG=1
  run c4_wp16rg_$rep c4 QLDPC_SPLIT_WP=16 QLDPC_SPLIT_SCRATCH=1
done
