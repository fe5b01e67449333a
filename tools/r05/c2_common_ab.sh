#!/bin/bash
# Diagnostic A/B (C2 SPA): QL_COUNT_COMMON drops the rare-path bodies (and their
# divergent branches) from tanh / atanh — an upper bound of what straight-line
# slot code buys.  Decode kernel ms, 2 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_common; mkdir -p $O
for rep in 1 2; do
for arm in prod common; do
  if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
  timeout -k 10 300 python bench.py --workload c2 --steps 8 --warmup 1 --no-cpu-baseline > $O/${arm}_$rep.json 2> $O/${arm}_$rep.err || { tail -5 $O/${arm}_$rep.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${arm}_$rep.json'))
print('$arm c2 rep$rep', 'decode', round(d['decode_kernel_ms'],3), 'ms step', round(d['ms_per_step'],3), 'iters', round(d['mean_iterations'],3))"
done
done
