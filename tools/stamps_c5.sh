#!/bin/bash
# the library and its loader read QLDPC_* knobs / alternative builds only under QLDPC_DIAG=1
export QLDPC_DIAG=1
# Phase shares (diagnostic stamp build) on C5 sweep points and C3.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/stamps; mkdir -p $O
for i in ${POINTS:-2 9 20}; do
  QLDPC_DIAG_STAMPS=1 timeout -k 10 120 python bench.py --workload c5ra --c5-point $i --steps 1 --warmup 0 --no-cpu-baseline \
    --streams 1 --roofline-launches 0 > $O/p$i.json 2> $O/p$i.err || { tail -5 $O/p$i.err; exit 13; }
  echo "p$i $(grep phase_stamps $O/p$i.err | tail -1)"
done
QLDPC_DIAG_STAMPS=1 timeout -k 10 120 python bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline \
    --streams 1 --roofline-launches 0 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 13; }
echo "c3 $(grep phase_stamps $O/c3.err | tail -1)"
