#!/bin/bash
# Round-4: split-frame SPA with 14 / 10 of its message slots in LDS (ab/rl14,
# ab/rl10) against the product's 12: C4 parity of each arm, then the A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for v in rl14 rl10; do
  QLDPC_AB_BUILD=$v timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "c4_100k_split_variant or c4_100k_split_full or c4_generated" \
    --timeout 120 --timeout-method thread -x > gpurun_out/rl_$v.log 2>&1 || { tail -n 5 gpurun_out/rl_$v.log; exit 11; }
  tail -n 1 gpurun_out/rl_$v.log
done
VARS="cur rl14 rl10" WLS="c4 c4g" REPS=2 STEPS=5 timeout -k 10 600 tools/ab_builds.sh || exit 12
echo done
