#!/bin/bash
# C4 (n=100k split frames) probe: batch sweep, phase stamps, C2 reference.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/c4p; mkdir -p $O
for b in 32 128 512; do
  timeout -k 10 200 python bench.py --workload c4 --batch $b --steps 4 --warmup 1 --no-cpu-baseline > $O/c4_b$b.json 2> $O/c4_b$b.err || exit 11
done
QLDPC_DIAG_STAMPS=1 timeout -k 10 200 python bench.py --workload c4 --steps 2 --warmup 1 --streams 1 --no-cpu-baseline > $O/c4_st.json 2> $O/c4_st.err || exit 12
QLDPC_DIAG_STAMPS=1 timeout -k 10 200 python bench.py --workload c2 --steps 2 --warmup 1 --streams 1 --no-cpu-baseline > $O/c2_st.json 2> $O/c2_st.err || exit 13
