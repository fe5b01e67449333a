#!/bin/bash
# Round-4 close: GPU parity suite, then every bench line (with its
# cpu_baseline) at HEAD (tools/round_bench.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
TAG=${TAG:-r04h}
timeout -k 10 500 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread --maxfail=5 \
  > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
tail -n 3 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || exit 11
TAG=$TAG DEFAULT=1 WLS="c3 c5 c5ra c4 c4g" CPU_S=8 timeout -k 10 900 tools/round_bench.sh || exit 12
echo done
