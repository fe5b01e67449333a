#!/bin/bash
# One GPU call: GPU parity suite on the product library, then a decode A/B
# between builds (tools/ab_builds.sh).  usage: VARS="cur prev" WLS="c2 c3" REPS=2 tools/gpu_ab.sh TAG
set -u
TAG=${1:-ab}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 12; }
tail -1 $O/pytest_gpu.log
bash tools/ab_builds.sh
