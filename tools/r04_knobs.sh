#!/bin/bash
# Round-4: C4 knobs with the exchange layout (fewer frames per XCD, K = 10)
# and C5 phase stamps at R = 0.8 (point 2) and R = 0.5 (point 20).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
ENVS="QLDPC_SPLIT_WGS=0 QLDPC_SPLIT_WGS=192" WLS="c4 c4g" REPS=2 timeout -k 10 500 tools/env_ab.sh || exit 11
ENVS="QLDPC_SPLIT_K=8 QLDPC_SPLIT_K=10" WLS="c4" REPS=2 timeout -k 10 300 tools/env_ab.sh || exit 12
POINTS="2 20" timeout -k 10 300 tools/stamps_c5.sh || exit 13
echo done
