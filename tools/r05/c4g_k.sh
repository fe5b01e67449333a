#!/bin/bash
# C4 (ii): part count K vs frames in flight per XCD (32 CUs): K = 11 (default,
# 2 frames + 10 waiting CUs), 12, 16 (2 frames, no waiting CU).  Decode ms and
# phase stamps per K.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_c4gk; mkdir -p $O
for K in 11 16 12; do
  QLDPC_SPLIT_K=$K timeout -k 10 300 python bench.py --workload c4g --steps 4 --warmup 1 --no-cpu-baseline > $O/k$K.json 2> $O/k$K.err || { tail -5 $O/k$K.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/k$K.json'))
print('K=$K decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), 'iters', round(d['mean_iterations'],3), 'lanes', d['config']['lanes_per_frame'])"
  QLDPC_SPLIT_K=$K QLDPC_DIAG_STAMPS=1 timeout -k 10 300 python bench.py --workload c4g --steps 1 --warmup 0 --no-cpu-baseline --streams 1 --roofline-launches 0 > $O/st$K.json 2> $O/st$K.err || { tail -5 $O/st$K.err; exit 4; }
  echo "K=$K $(grep phase_stamps $O/st$K.err | tail -1)"
done
