cd $GRAFT_REPO_ROOT
for v in ${VARS:-base common}; do for wl in ${WLS:-c2}; do
  if [ $v = base ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$v; fi
  timeout -k 10 200 python bench.py --workload $wl --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${v}_${wl}.json 2>/dev/null || exit 3
  python -c "import json; d=json.load(open('gpurun_out/ab_${v}_${wl}.json')); print('$v $wl', 'dec', round(d['decode_kernel_ms'],3), 'iters', round(d['mean_iterations'],3), 'ms/iter', round(d['decode_kernel_ms']/d['mean_iterations'],4))"
done; done
