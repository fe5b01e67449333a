#!/bin/bash
# 8-wave split parts after the deferred exit test: exchange-gather depth 2
# (xg2: fewer spills) and 14 LDS message slots (rl14: fewer spills, smaller
# exchange chunks) vs the product; split parity per arm, then C4 / C4 (ii)
# alternating, 2 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_sknobs; mkdir -p $O
for arm in xg2 rl14; do
  QLDPC_AB_BUILD=$arm timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "c4 or split" > $O/pytest_$arm.log 2>&1 || { tail -30 $O/pytest_$arm.log; exit 10; }
  echo "$arm $(tail -1 $O/pytest_$arm.log)"
done
for rep in 1 2; do
for arm in prod xg2 rl14; do
for wl in c4g c4; do
  if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
  timeout -k 10 300 python bench.py --workload $wl --steps 6 --warmup 1 --no-cpu-baseline > $O/${arm}_${wl}_$rep.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${arm}_${wl}_$rep.json'))
print('$arm $wl', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2))"
done
done
done
