#!/bin/bash
# Round-4: split frames over a whole XCD with each part's totals in LDS
# (K = 32, QLDPC_SPLIT_LOCAL=1 default) — split parity first, then A/B against
# the 16-wave parts (QLDPC_SPLIT_LOCAL=0) on C4 / C4 (ii), the whole suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r04_local; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -v -m gpu -k "c4 or split" --timeout 120 --timeout-method thread -x \
  > $O/pytest_split.log 2>&1; rc=$?
tail -n 25 $O/pytest_split.log
[ $rc -eq 0 ] || exit 11
ENVS="QLDPC_SPLIT_LOCAL=1 QLDPC_SPLIT_LOCAL=0" WLS="c4 c4g" REPS=2 timeout -k 10 500 tools/env_ab.sh || exit 12
timeout -k 10 500 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread --maxfail=5 \
  > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 3 $O/pytest_gpu.log
exit $rc
