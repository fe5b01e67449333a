#!/bin/bash
# Round-4: exchange gather unrolled 8 deep (QL_XG_UNROLL) — split parity, A/B
# against 4 deep (ab/xu4), C4 phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r04_z; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "c4 or split" --timeout 200 --timeout-method thread -x \
  > $O/pytest_split.log 2>&1; rc=$?
tail -n 3 $O/pytest_split.log
[ $rc -eq 0 ] || exit 11
VARS="cur xu4" WLS="c4 c4g" REPS=2 STEPS=5 timeout -k 10 500 tools/ab_builds.sh || exit 12
WLS=c4 timeout -k 10 200 tools/stamps.sh || exit 14
echo done
