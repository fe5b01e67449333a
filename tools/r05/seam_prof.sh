#!/bin/bash
# Kernel timeline of the pipelined C2 seam sweep (8 combinations) and the
# trial generator's kernels: rocprofv3 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r05_seamprof; mkdir -p $O
M=tests/golden/matrices/c2_n10240_m2201.alist.gz
printf '0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n' > $O/q_c2.txt
timeout -k 10 240 tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 4096 1022025 0 > $O/seam_c2.txt 2>&1 || { cat $O/seam_c2.txt; exit 12; }
echo "seam c2: $(cat $O/seam_c2.txt)"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o sweep -- tests/dropin/batch_check sweep $M 1 0 0 0 $O/q_c2.txt 50 4096 1022025 > $O/sweep_c2.txt 2>&1 || { tail -20 $O/sweep_c2.txt; exit 13; }
tail -2 $O/sweep_c2.txt
find $O/trace -name "*.csv" | head
