#!/bin/bash
# Split frames with 44 slots per lane (A/B build r44: make ab AB=r44
# AB_FLAGS=-DQL_SPLIT_R=44 AB_CAPI=1 — fewer, larger parts: C4 14 x 8 waves,
# C4 (ii) 19) vs the product's 40; split parity of the arm, then C4 / C4 (ii)
# alternating, 2 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_r44; mkdir -p $O
for arm in r44; do
  QLDPC_AB_BUILD=$arm timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "c4 or split" > $O/pytest_$arm.log 2>&1; grep -E "^FAILED" $O/pytest_$arm.log | cut -c1-120
  echo "$arm $(tail -1 $O/pytest_$arm.log)"
done
for rep in 1 2; do
for arm in prod r44; do
for wl in c4g c4; do
  if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
  timeout -k 10 300 python bench.py --workload $wl --steps 6 --warmup 1 --no-cpu-baseline > $O/${arm}_${wl}_$rep.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${arm}_${wl}_$rep.json'))
print('$arm $wl', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2))"
done
done
done
