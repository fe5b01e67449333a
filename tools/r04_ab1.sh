#!/bin/bash
# Round-4 A/B session 1: C2 shape / LDS-slot A/B and the batch seam's chunking.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r04_ab1; mkdir -p $O
M=tests/golden/matrices/c2_n10240_m2201.alist.gz
for c in 4096 2048 1024 512; do
  QLDPC_TRIAL_CHUNK=$c timeout -k 10 120 tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 8192 1022025 0 > $O/seam_c$c.txt 2>&1 || { cat $O/seam_c$c.txt; exit 11; }
  echo "chunk $c: $(cat $O/seam_c$c.txt)"
done
ENVS="QLDPC_V2_WAVES=16 QLDPC_V2_WAVES=12" WLS=c2 REPS=2 STEPS=6 timeout -k 10 400 tools/env_ab.sh || exit 12
VARS="cur rl5" WLS=c2 REPS=2 STEPS=6 timeout -k 10 400 tools/ab_builds.sh || exit 13
echo done
