#!/bin/bash
# Round-4: decoder compiled without memory-op clustering in the machine
# scheduler (ab/nocl) against the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
VARS="cur nocl" WLS="c2 c5 c4" REPS=2 STEPS=6 timeout -k 10 600 tools/ab_builds.sh || exit 12
echo done
