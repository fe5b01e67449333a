#!/bin/bash
# Round-3 baseline measurement at HEAD: counter list, then PMC / trace passes of
# C4 (split frames), C5 (hybrid shape), C3 and C2 (LDS counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 90 rocprofv3 --list-avail > gpurun_out/rocprof_avail.txt 2>&1 || echo "list-avail rc=$?"
DEFAULT=0 WLS="c4" PASSES="trace fetch write sq sq2 tcc ea" STEPS=3 tools/profile_round.sh || exit 21
DEFAULT=0 WLS="c5" PASSES="trace fetch write sq2 tcc" tools/profile_round.sh || exit 22
DEFAULT=0 WLS="c3" PASSES="trace fetch write sq sq2 valu lds" tools/profile_round.sh || exit 23
DEFAULT=0 WLS="c2" PASSES="lds" tools/profile_round.sh || exit 24
