#!/bin/bash
# GPU parity suite, then an A/B of the frame claim order (QLDPC_ORDER=0: index
# order) on the bench workloads.  usage: tools/order_ab.sh [tag]
TAG=${1:-ord}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/t_$TAG.log 2>&1 || { tail -30 gpurun_out/t_$TAG.log; exit 12; }
tail -2 gpurun_out/t_$TAG.log
for wl in ${WLS:-c2 c3 c5 c5ra c4}; do for o in 0 1; do
  QLDPC_ORDER=$o timeout -k 10 200 python bench.py --workload $wl --steps 6 --warmup 2 --no-cpu-baseline \
    > gpurun_out/ab_${TAG}_${wl}_o$o.json 2>gpurun_out/ab_${TAG}_${wl}_o$o.err || exit 13
  python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${wl}_o$o.json')); print('$wl order=$o', 'Gbit/s', round(d['value']/1e9,3), 'dec ms', round(d['decode_kernel_ms'],3), 'ms/step', round(d['ms_per_step'],3), 'iters', round(d['mean_iterations'],3), 'frac', round(d['roofline']['frac'],4))"
done; done
