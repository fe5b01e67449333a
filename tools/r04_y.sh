#!/bin/bash
# Round-4: split-frame SPA with tanh's word-form table (QL_SPLIT_TANH_W) —
# split parity, A/B against the trimmed form (ab/trim), C4 counters and phase
# stamps with the exchange layout, then the seam timeline and C2 stall pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r04_y; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "c4 or split or self_test" --timeout 200 --timeout-method thread -x \
  > $O/pytest_split.log 2>&1; rc=$?
tail -n 3 $O/pytest_split.log
[ $rc -eq 0 ] || exit 11
VARS="cur trim" WLS="c4 c4g" REPS=2 STEPS=5 timeout -k 10 500 tools/ab_builds.sh || exit 12
WLS=c4 PASSES="trace fetch write ea tcc" DEFAULT=0 timeout -k 10 400 tools/profile_round.sh || exit 13
WLS=c4 timeout -k 10 200 tools/stamps.sh || exit 14
timeout -k 10 600 tools/r04_seamprof.sh || exit 15
echo done
