#!/bin/bash
# the library and its loader read QLDPC_* knobs / alternative builds only under QLDPC_DIAG=1
export QLDPC_DIAG=1
# Decode-kernel A/B over in-tree builds: "cur" is the product library, any other
# name an A/B build under qkd_ldpc_v_amd/ab/<name>/ (QLDPC_AB_BUILD).  Runs
# alternate between builds, REPS times.  usage: VARS="cur x" WLS="c2 c3" REPS=2 tools/ab_builds.sh
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do for wl in ${WLS:-c2}; do for v in ${VARS:-cur}; do
  if [ $v = cur ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$v; fi
  timeout -k 10 300 python bench.py --workload $wl --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline \
    > gpurun_out/abb_${v}_$wl.json 2>gpurun_out/abb_${v}_$wl.err || { tail -5 gpurun_out/abb_${v}_$wl.err; exit 13; }
  python -c "import json; d=json.load(open('gpurun_out/abb_${v}_$wl.json')); print('$v $wl', 'Gbit/s', round(d['value']/1e9,3), 'dec ms', round(d['decode_kernel_ms'],3), 'iters', round(d['mean_iterations'],3))"
done; done; done
