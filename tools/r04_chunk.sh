#!/bin/bash
# Round-4: batch-seam chunking A/B (QLDPC_TRIAL_CHUNK) on C2 through the C++
# drop-in (tests/dropin/batch_check time), 4096 and 8192 trials.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r04_chunk; mkdir -p $O
M=tests/golden/matrices/c2_n10240_m2201.alist.gz
for rep in 1 2; do
  for ch in 0 4096 8192; do
    for tr in 4096 8192; do
      QLDPC_TRIAL_CHUNK=$ch timeout -k 10 120 tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 $tr 1022025 0 > $O/t_${ch}_${tr}_$rep.txt 2>&1 || { cat $O/t_${ch}_${tr}_$rep.txt; exit 11; }
      echo "chunk=$ch trials=$tr: $(tr '\n' ' ' < $O/t_${ch}_${tr}_$rep.txt)"
    done
  done
done
