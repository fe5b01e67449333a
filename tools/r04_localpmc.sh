#!/bin/bash
# Round-4: counters of the K = 32 local-totals split (QLDPC_SPLIT_LOCAL=1) on C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
rm -rf gpurun_out/round_prof
QLDPC_SPLIT_LOCAL=1 WLS=c4 PASSES="sq sq2 stall fetch write tcc" DEFAULT=0 timeout -k 10 400 tools/profile_round.sh || exit 11
echo done
