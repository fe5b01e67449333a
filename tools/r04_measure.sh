#!/bin/bash
# Round-4 measurements on the GPU box (each GPU step under its own limit; the
# session ends at the first failure):
#   1. the C2 batch seam vs the per-trial drop-in (tests/dropin/batch_check time)
#   2. C2 PMC: wait / LDS / clock counters (tools/profile_round.sh passes sq2, lds)
#   3. split-frame phase stamps of C4 (diagnostic build)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r04_measure; mkdir -p $O
M=tests/golden/matrices/c2_n10240_m2201.alist.gz
for cfg in "4096 16" "4096 8" "1024 1"; do
  set -- $cfg
  echo "[$(date +%T)] batch_check time trials=$1 threads=$2"
  timeout -k 10 240 tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 $1 1022025 $2 > $O/seam_t$2.txt 2>&1 || { cat $O/seam_t$2.txt; exit 11; }
  cat $O/seam_t$2.txt
done
WLS=c2 DEFAULT=0 PASSES="sq2 lds" STEPS=3 timeout -k 10 600 tools/profile_round.sh || exit 12
WLS="c4" timeout -k 10 400 tools/stamps.sh || exit 13
echo done
