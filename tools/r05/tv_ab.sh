#!/bin/bash
# Same-box A/B of the split scan's totals loads (C4 stand-in and C4 (ii)):
# product vs QL_TV_NOPRIO (no priority rotation in the split scan), QL_TV_HALF
# (next group's totals half a group early), both.  Decode kernel ms (serial
# launches) and the 2-stream step.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_tv; mkdir -p $O
for rep in 1 2; do
for arm in prod tvnoprio tvhalf tvhalfnp; do
  for wl in c4 c4g; do
    if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
    timeout -k 10 300 python bench.py --workload $wl --steps 6 --warmup 1 --no-cpu-baseline > $O/${arm}_${wl}_$rep.json 2> $O/${arm}_${wl}_$rep.err || { tail -5 $O/${arm}_${wl}_$rep.err; exit 3; }
    python3 -c "
import json; d=json.load(open('$O/${arm}_${wl}_$rep.json'))
print('$arm $wl rep$rep', 'decode', round(d['decode_kernel_ms'],2), 'ms step', round(d['ms_per_step'],2), 'fer', d['fer'], 'iters', round(d['mean_iterations'],3))"
  done
done
done
