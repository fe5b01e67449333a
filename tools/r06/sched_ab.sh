#!/bin/bash
# scheduler-option A/B: bench lines per arm, 2 reps alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/sched_ab; mkdir -p $O
for rep in 1 2; do
  for wl in c2 c5; do
    for arm in product trk bias0 maxilp; do
      if [ $arm = product ]; then E=""; else E="QLDPC_DIAG=1 QLDPC_AB_BUILD=$arm"; fi
      env $E timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 2 --no-cpu-baseline > $O/${wl}_${arm}_$rep.json 2> $O/${wl}_${arm}_$rep.err || exit 11
      python -c "import json;d=json.load(open('$O/${wl}_${arm}_$rep.json'));print('$wl $arm $rep', round(d['ms_per_step'],3), round(d['decode_kernel_ms'],3), d['mean_iterations'])" | tee -a $O/summary.txt
    done
  done
done
