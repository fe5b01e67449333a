#!/bin/bash
# C4 stand-in, 8-wave parts: planner K = 15 (EPL 40, 60 of an XCD's 64
# workgroups) vs K = 16 (EPL 38, all 64), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_c4k; mkdir -p $O
for rep in 1 2; do
for k in 0 16; do
  QLDPC_SPLIT_K=$k timeout -k 10 300 python bench.py --workload c4 --steps 6 --warmup 1 --no-cpu-baseline > $O/k${k}_$rep.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/k${k}_$rep.json'))
print('k $k', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), 'lanes', d['config']['lanes_per_frame'], 'epl', d['config']['edges_per_lane'])"
done
done
