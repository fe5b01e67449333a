#!/bin/bash
# The C2 batch seam (qldpc_run_trials through the C++ drop-in) and the per-trial
# drop-in from T threads: tests/dropin/batch_check time, one line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r04_seam; mkdir -p $O
M=tests/golden/matrices/c2_n10240_m2201.alist.gz
for cfg in "8192 0" "4096 0" "4096 16" "4096 8" "1024 1"; do
  set -- $cfg
  timeout -k 10 240 tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 $1 1022025 $2 > $O/t_$1_$2.txt 2>&1 || { cat $O/t_$1_$2.txt; exit 11; }
  echo "trials=$1 threads=$2: $(tr '\n' ' ' < $O/t_$1_$2.txt)"
done
