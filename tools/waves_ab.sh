#!/bin/bash
# C2/C3 decode time at the planner's default waves per frame vs a forced count
# (QLDPC_V2_WAVES), alternating runs.  usage: tools/waves_ab.sh [waves]
W=${1:-12}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for rep in 1 2; do for wl in c2 c3; do for w in 0 $W; do
  if [ $w = 0 ]; then unset QLDPC_V2_WAVES; else export QLDPC_V2_WAVES=$w; fi
  timeout -k 10 200 python bench.py --workload $wl --steps 6 --warmup 2 --no-cpu-baseline \
    > gpurun_out/wv_${wl}_$w.json 2>gpurun_out/wv_${wl}_$w.err || exit 13
  python -c "import json; d=json.load(open('gpurun_out/wv_${wl}_$w.json')); print('$wl waves=$w', d['config']['lanes_per_frame'], d['config']['edges_per_lane'], 'dec ms', round(d['decode_kernel_ms'],3))"
done; done; done
