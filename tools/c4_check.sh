#!/bin/bash
# C4 (split frames) parity tests + bench lines.  usage: tools/c4_check.sh [tag]
TAG=${1:-c4}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "${KSEL:-c4 or host_threads}" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1 || { tail -30 gpurun_out/t_$TAG.log; exit 12; }
tail -2 gpurun_out/t_$TAG.log
for wl in ${WLS:-c4 c4g}; do
  timeout -k 10 300 python bench.py --workload $wl --steps 6 --warmup 2 --no-cpu-baseline \
    > gpurun_out/b_${TAG}_${wl}.json 2>gpurun_out/b_${TAG}_${wl}.err || exit 13
  python -c "import json; d=json.load(open('gpurun_out/b_${TAG}_${wl}.json')); print('$wl', 'Gbit/s', round(d['value']/1e9,3), 'dec ms', round(d['decode_kernel_ms'],3), 'ms/step', round(d['ms_per_step'],3), 'iters', round(d['mean_iterations'],3), 'frac', round(d['roofline']['frac'],4), 'fer', d['fer'])"
done
