#!/bin/bash
# Instruction-cache and issue-stall counters for one workload (separate PMC
# passes, --kernel-trace only).  usage: tools/profile_icache.sh <tag> <workload>
set -u
TAG=$1; WL=$2
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/icache_${TAG}
mkdir -p "$OUT"
BENCH="bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --streams 1 --roofline-launches 0"
run() {
  local name=$1; shift
  echo "[$(date +%T)] pass $name" >&2
  timeout -k 10 400 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python $BENCH > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pass $name failed rc=$rc" >&2; tail -20 "$OUT/$name.log" >&2; exit $rc; fi
}
run ic1 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-trace
run ic2 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_VALU --kernel-trace
run ic3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --kernel-trace
echo "[$(date +%T)] done" >&2
