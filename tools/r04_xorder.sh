#!/bin/bash
# Round-4: exchange-stage order within a region grouped by slot group across a
# part's waves (QLDPC_SPLIT_XORDER=1, default) vs one run per wave (0): split
# parity, A/B, then C4 / C4 (ii) traffic passes at the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r04_xorder; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "c4 or split" --timeout 200 --timeout-method thread -x \
  > $O/pytest_split.log 2>&1; rc=$?
tail -n 3 $O/pytest_split.log
[ $rc -eq 0 ] || exit 11
ENVS="QLDPC_SPLIT_XORDER=1 QLDPC_SPLIT_XORDER=0" WLS="c4 c4g" REPS=2 timeout -k 10 500 tools/env_ab.sh || exit 12
WLS="c4 c4g" PASSES="fetch write ea" DEFAULT=0 timeout -k 10 300 tools/profile_round.sh || exit 13
echo done
