cd $GRAFT_REPO_ROOT
for v in g s p; do
  QLDPC_AB_BUILD=$v timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 -p no:cacheprovider -k "c4" > gpurun_out/bis_$v.log 2>&1; echo "$v rc=$? $(tail -n 1 gpurun_out/bis_$v.log)"
done
