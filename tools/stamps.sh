#!/bin/bash
# the library and its loader read QLDPC_* knobs / alternative builds only under QLDPC_DIAG=1
export QLDPC_DIAG=1
# Per-phase share of wave time (diagnostic phase-stamp build, `make stamps`) for
# the given workloads, one serial step each.  usage: WLS="c2 c4" tools/stamps.sh
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for wl in ${WLS:-c2}; do
  QLDPC_DIAG_STAMPS=1 timeout -k 10 300 python bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline --streams 1 \
    --roofline-launches 0 > gpurun_out/st_$wl.json 2> gpurun_out/st_$wl.err || { tail -5 gpurun_out/st_$wl.err; exit 13; }
  echo "$wl $(grep phase_stamps gpurun_out/st_$wl.err | tail -1)"
done
