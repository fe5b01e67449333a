#!/bin/bash
# Round-4 close on one GPU box: the GPU parity suite, rocprofv3 kernel-trace +
# PMC passes of every workload (summarised into profiles/pmc_*.json here, so
# the bench lines below price traffic and VALU issue from this same build),
# then every bench line with its cpu_baseline.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r04k}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread --maxfail=5 \
  > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
tail -n 3 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || exit 11
CLEAN=1 DEFAULT=1 WLS="c2 c3 c5 c5ra c4 c4g" PASSES="trace fetch write sq sq2 valu tcc ea stall" \
  timeout -k 10 700 tools/profile_round.sh || exit 12
python tools/round_summary.py gpurun_out/round_prof $TAG r04 > gpurun_out/${TAG}_summary.log 2>&1 || exit 13
TAG=$TAG DEFAULT=1 WLS="c3 c5 c5ra c4 c4g" CPU_S=8 timeout -k 10 700 tools/round_bench.sh || exit 14
echo done
