set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_c2_v2.json 2> gpurun_out/b_c2_v2.err || exit 11
timeout -k 10 1200 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/t_gpu.log 2>&1 ; rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit 12
QLDPC_VARIANT=v1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_c2_v1.json 2> gpurun_out/b_c2_v1.err || exit 13
timeout -k 10 300 python bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_c3_v2.json 2> gpurun_out/b_c3_v2.err || exit 14
QLDPC_V2_WAVES=12 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_c2_v2w12.json 2> gpurun_out/b_c2_v2w12.err || exit 15
exit $rc
