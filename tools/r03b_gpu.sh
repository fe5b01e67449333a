set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03b_pytest_gpu.log; exit 11; }
tail -3 gpurun_out/r03b_pytest_gpu.log
WLS="c2 c3" ENVS="QLDPC_RELABEL=0 -" REPS=2 bash tools/ab_env.sh || exit 12
DEFAULT=0 WLS="c2 c3" PASSES="lds sq2" bash tools/profile_round.sh || exit 13
