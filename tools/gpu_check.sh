#!/bin/bash
# One GPU-box session: the GPU parity suite, then (unless it crashed or timed
# out: a fault, an abort or a limit ends the session there) the default bench.
#   TAG=r04a tools/gpu_check.sh [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
TAG=${TAG:-r04}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread --maxfail=8 \
  > "gpurun_out/${TAG}_pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a "gpurun_out/${TAG}_pytest_gpu.log"
tail -15 "gpurun_out/${TAG}_pytest_gpu.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py "$@" > "gpurun_out/${TAG}_bench_default.json" 2> "gpurun_out/${TAG}_bench_default.err"
brc=$?
echo "bench rc=$brc"
cat "gpurun_out/${TAG}_bench_default.json"
exit $brc
