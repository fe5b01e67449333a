#!/bin/bash
# Round-4: kernel timeline of the C2 batch seam (qldpc_run_trials through the
# C++ drop-in, 4096 trials after a warm-up call), and the C2 stall / clock PMC
# pass (tools/profile_round.sh "stall") plus the FP64 microbenchmark's clock.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r04_seamprof; mkdir -p $O
M=tests/golden/matrices/c2_n10240_m2201.alist.gz
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/seam -o run --output-format csv -- \
  tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 4096 1022025 0 > $O/seam.txt 2>&1 || { tail -5 $O/seam.txt; exit 11; }
grep seam $O/seam.txt
WLS=c2 PASSES="stall" DEFAULT=0 timeout -k 10 300 tools/profile_round.sh || exit 12
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace \
  -d $O/vb -o run --output-format csv -- tools/valu_bench > $O/vb.log 2>&1 || { tail -5 $O/vb.log; exit 13; }
echo done
