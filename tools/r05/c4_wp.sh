#!/bin/bash
# C4 stand-in after the deferred exit test: 16-wave parts (planner) vs forced
# 8-wave parts (QLDPC_SPLIT_WP=8), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_c4wp; mkdir -p $O
for rep in 1 2; do
for wp in 0 8; do
  QLDPC_SPLIT_WP=$wp timeout -k 10 300 python bench.py --workload c4 --steps 6 --warmup 1 --no-cpu-baseline > $O/wp${wp}_$rep.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/wp${wp}_$rep.json'))
print('wp $wp', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), 'lanes', d['config']['lanes_per_frame'], 'epl', d['config']['edges_per_lane'])"
done
done
