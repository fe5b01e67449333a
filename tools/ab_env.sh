#!/bin/bash
# Same-build A/B over environment settings: for each workload in WLS and each
# setting in ENVS ("NAME=v1 NAME=v2" ...; "-" = none), REPS alternating runs of
# bench.py; one summary line per run.  usage: WLS="c2 c3" ENVS="QLDPC_RELABEL=0 -" tools/ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do for wl in ${WLS:-c2}; do for e in ${ENVS:--}; do
  tag=$(echo "$e" | tr '=' '_')
  if [ "$e" = "-" ]; then envset=""; else envset="$e"; fi
  env $envset timeout -k 10 300 python bench.py --workload $wl --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline \
    > gpurun_out/abe_${tag}_$wl.json 2>gpurun_out/abe_${tag}_$wl.err || { tail -5 gpurun_out/abe_${tag}_$wl.err; exit 13; }
  python -c "import json; d=json.load(open('gpurun_out/abe_${tag}_$wl.json')); print('$e $wl', 'Gbit/s', round(d['value']/1e9,3), 'dec ms', round(d['decode_kernel_ms'],3), 'iters', round(d['mean_iterations'],3))"
done; done; done
