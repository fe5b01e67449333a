#!/bin/bash
# Round-4 diagnostics 2: the FP64 microbenchmark's clock and VALU occupancy
# (is a dense FP64 stream power-limited?), C5 phase stamps at R=0.8 / R=0.5,
# and the C2 kpos-0 LLR hoist A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r04_diag2; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace \
  -d $O/vb -o run --output-format csv -- tools/valu_bench > $O/vb.log 2>&1 || { tail -5 $O/vb.log; exit 11; }
POINTS="2 20" timeout -k 10 400 tools/stamps_c5.sh || exit 12
VARS="cur hoist" WLS=c2 REPS=2 STEPS=6 timeout -k 10 400 tools/ab_builds.sh || exit 13
QLDPC_SPLIT_K=16 WLS=c4 timeout -k 10 300 tools/stamps.sh || exit 14
echo done
