# usage: bash /tmp/ab.sh "variants" "workloads" reps
V="$1"; W="$2"; N=${3:-2}
cd $GRAFT_REPO_ROOT
for r in $(seq $N); do for v in $V; do for wl in $W; do
  if [ $v = base ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$v; fi
  timeout -k 10 200 python bench.py --workload $wl --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${v}_${wl}_$r.json 2>/dev/null || exit 3
  python -c "import json; d=json.load(open('gpurun_out/ab_${v}_${wl}_$r.json')); print('$v $wl $r', round(d['decode_kernel_ms'],3), round(d['value']/1e9,4))"
done; done; done
