#!/bin/bash
# Round 6 A/B: split parts with 12 scratch message slots per lane (build rg12:
# make ab AB=rg12 AB_CAPI=1 AB_FLAGS=-DQL_SPLIT_RG=12 — C4 (ii) 16 x 8-wave
# parts, 4 frames per XCD; stand-in 12 parts, 5 frames) vs the product.
# Split parity of the arm, then C4 (ii) / C4 alternating, 2 reps, then one
# FETCH_SIZE / WRITE_SIZE / SQ pass per arm on C4 (ii).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export QLDPC_DIAG=1 TMPDIR=/tmp
ARM=${ARM:-rg12}
O=gpurun_out/r06_$ARM; mkdir -p $O
QLDPC_AB_BUILD=$ARM timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "c4 or split" > $O/pytest_$ARM.log 2>&1
prc=$?
grep -E "^FAILED" $O/pytest_$ARM.log | cut -c1-150
echo "$ARM pytest rc=$prc $(tail -1 $O/pytest_$ARM.log)"
if [ $prc -gt 1 ]; then exit $prc; fi
for rep in 1 2; do
for arm in prod $ARM; do
for wl in c4g c4; do
  if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
  timeout -k 10 300 python bench.py --workload $wl --steps 6 --warmup 1 --no-cpu-baseline > $O/${arm}_${wl}_$rep.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${arm}_${wl}_$rep.json'))
print('$arm $wl', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), 'it', d['mean_iterations'], d['config']['lanes_per_frame'])"
done
done
done
unset QLDPC_AB_BUILD
B="--workload c4g --steps 2 --warmup 1 --no-cpu-baseline --streams 1 --roofline-launches 0"
for arm in prod $ARM; do
  if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $O/pmc_${arm}_p$i -o run --output-format csv -- python bench.py $B > $O/pmc_${arm}_p$i.log 2>&1 || { tail -5 $O/pmc_${arm}_p$i.log; exit 4; }
  done
  python3 tools/pmc_summary.py $O decode_v2 --prefix pmc_${arm}_ --json $O/pmc_${arm}.json | tail -12
done
