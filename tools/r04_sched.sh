#!/bin/bash
# Round-4: decoder built with other AMDGPU machine-scheduler strategies
# (ab/ilp: max-ilp, ab/iter: iterative-ilp) against the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
VARS="cur ilp iter" WLS="c2 c3 c5 c4" REPS=2 STEPS=6 timeout -k 10 900 tools/ab_builds.sh || exit 12
timeout -k 10 300 tools/r04_localpmc.sh || exit 13
echo done
