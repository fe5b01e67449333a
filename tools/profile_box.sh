#!/bin/bash
# Run on the GPU box (via gpurun): kernel trace + PMC passes for one workload.
# usage: tools/profile_box.sh <tag> <workload> [steps]
# Writes gpurun_out/prof_<tag>/...  Each rocprofv3 pass has its own time limit;
# the script stops at the first failing pass.
set -u
TAG=$1; WL=$2; STEPS=${3:-5}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
BENCH="bench.py --workload $WL --steps $STEPS --warmup 1 --no-cpu-baseline"
run() {  # name, extra rocprofv3 args...
  local name=$1; shift
  echo "[$(date +%T)] pass $name" >&2
  timeout -k 10 400 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python $BENCH > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pass $name failed rc=$rc" >&2; tail -20 "$OUT/$name.log" >&2; exit $rc; fi
}
run trace --kernel-trace --stats
run pmc_fetch --pmc FETCH_SIZE --kernel-trace
run pmc_write --pmc WRITE_SIZE --kernel-trace
run pmc_sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM --kernel-trace
run pmc_sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace
echo "[$(date +%T)] done" >&2
