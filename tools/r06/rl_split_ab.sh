#!/bin/bash
# Round 6 A/B: LDS message slots of the split SPA kernel (QL_RL_SPLIT 8 / 16
# vs the product's 12) on the 16-wave + scratch-slot plan of C4 (ii) and the
# 8-wave stand-in: split parity of each arm, then 2 reps alternating.
# Builds: make ab AB=rl8 AB_FLAGS=-DQL_RL_SPLIT=8; make ab AB=rl16 AB_FLAGS=-DQL_RL_SPLIT=16
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export QLDPC_DIAG=1
O=gpurun_out/r06_rl; mkdir -p $O
for arm in rl8 rl16; do
  QLDPC_AB_BUILD=$arm timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "c4_100k_split_variant or c4_generated or c4_split_deferred" > $O/pytest_$arm.log 2>&1
  rc=$?; echo "$arm pytest rc=$rc $(tail -1 $O/pytest_$arm.log)"; [ $rc -le 1 ] || exit $rc
done
for rep in 1 2; do
for arm in prod rl8 rl16; do
for wl in c4g c4; do
  if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
  timeout -k 10 300 python bench.py --workload $wl --steps 8 --warmup 2 --no-cpu-baseline > $O/${arm}_${wl}_$rep.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${arm}_${wl}_$rep.json'))
print('$arm $wl', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2))"
done
done
done
