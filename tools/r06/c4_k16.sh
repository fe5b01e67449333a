#!/bin/bash
# Round 6: with split decodes serialised per device (no next-batch overlap in
# a launch's tail), does the stand-in prefer K = 16 parts (EPL 38, every
# workgroup of an XCD busy, 4 frames) over the planner's smallest K = 15?
# Same box, 3 reps alternating (QLDPC_SPLIT_K under QLDPC_DIAG=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export QLDPC_DIAG=1
O=gpurun_out/r06_c4_k16; mkdir -p $O
for rep in 1 2 3; do
for k in 0 16; do
  if [ $k = 0 ]; then unset QLDPC_SPLIT_K; else export QLDPC_SPLIT_K=$k; fi
  timeout -k 10 300 python bench.py --workload c4 --steps 6 --warmup 1 --no-cpu-baseline > $O/k${k}_$rep.json 2> $O/k$k.err || { tail -5 $O/k$k.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/k${k}_$rep.json'))
print('K=$k', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), d['config']['lanes_per_frame'])"
done
done
