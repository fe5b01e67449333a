#!/bin/bash
# the library and its loader read QLDPC_* knobs / alternative builds only under QLDPC_DIAG=1
export QLDPC_DIAG=1
# Same-build A/B of an environment knob: ENVS="QLDPC_X=0 QLDPC_X=1" over
# workloads (WLS) and C5 sweep points (POINTS), REPS times, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/envab; mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for e in ${ENVS}; do
    for wl in ${WLS:-}; do
      env $e timeout -k 10 120 python bench.py --workload $wl --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline \
          > $O/r.json 2> $O/r.err || { tail -5 $O/r.err; exit 3; }
      python -c "import json; d=json.load(open('$O/r.json')); print('$e', '$wl', round(d['value']/1e9,4), 'dec ms', round(d['decode_kernel_ms'],3))"
    done
    for i in ${POINTS:-}; do
      env $e timeout -k 10 120 python bench.py --workload c5ra --c5-point $i --steps 3 --warmup 1 --no-cpu-baseline \
          --roofline-launches 1 > $O/r.json 2> $O/r.err || { tail -5 $O/r.err; exit 3; }
      python -c "import json; d=json.load(open('$O/r.json')); print('$e', 'point $i', round(d['value']/1e9,4), 'dec ms', round(d['decode_kernel_ms'],3))"
    done
  done
done
