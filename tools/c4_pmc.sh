#!/bin/bash
# C4 split-frame PMC passes (L2 hit/miss, fabric requests, VALU/wait).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/c4pmc/${WL:-c4}; mkdir -p $O
B="--workload ${WL:-c4} --steps 2 --warmup 1 --no-cpu-baseline --streams 1 --roofline-launches 0"
i=0
for ctr in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $O/p$i -o run --output-format csv -- python bench.py $B > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1$i; }
done
for i in 1 2 3; do python tools/pmc_summary.py $O decode_v2 --prefix p$i; done
