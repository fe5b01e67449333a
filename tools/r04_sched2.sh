#!/bin/bash
# Round-4: two more machine-scheduler strategies (ab/mclause: max-memory-clause,
# ab/maxocc: iterative-maxocc) against the product's iterative-ilp, then the
# 26-point C5 sweep at HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
VARS="cur mclause maxocc" WLS="c2 c5 c4" REPS=2 STEPS=6 timeout -k 10 700 tools/ab_builds.sh || exit 12
timeout -k 10 800 tools/c5_sweep.sh || exit 13
echo done
