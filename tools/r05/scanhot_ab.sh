#!/bin/bash
# Diagnostic A/B: the split scan's totals from 256 L1-hot entries (QL_DIAG_SCAN_HOT,
# wrong decodes) vs the product — how much of the C4 decode is the scan's
# total[col] latency.  ms per frame-iteration of the decode kernel, plus stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_scanhot; mkdir -p $O
for rep in 1 2; do
for arm in prod scanhot; do
  for wl in c4 c4g; do
    if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
    timeout -k 10 300 python bench.py --workload $wl --steps 4 --warmup 1 --no-cpu-baseline --streams 1 > $O/${arm}_${wl}_$rep.json 2> $O/${arm}_${wl}_$rep.err || { tail -5 $O/${arm}_${wl}_$rep.err; exit 3; }
    python3 -c "
import json; d=json.load(open('$O/${arm}_${wl}_$rep.json'))
it=d['mean_iterations']*d['config']['batch_per_gpu']
print('$arm $wl rep$rep', 'decode', round(d['decode_kernel_ms'],2), 'ms iters', round(d['mean_iterations'],2), 'us/frame-iter', round(1e3*d['decode_kernel_ms']/it,3))"
  done
done
done
