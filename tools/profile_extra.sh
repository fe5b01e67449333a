#!/bin/bash
# Extra PMC passes (instruction cache, VALU mix) for one workload, on the GPU box.
# usage: tools/profile_extra.sh <tag> <workload> [steps]
set -u
TAG=$1; WL=$2; STEPS=${3:-3}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
BENCH="bench.py --workload $WL --steps $STEPS --warmup 1 --no-cpu-baseline"
run() {
  local name=$1; shift
  echo "[$(date +%T)] pass $name" >&2
  timeout -k 10 400 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python $BENCH > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pass $name failed rc=$rc" >&2; tail -20 "$OUT/$name.log" >&2; exit $rc; fi
}
run pmc_icache --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH --kernel-trace
run pmc_valu --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_FLAT SQ_INSTS_BRANCH --kernel-trace
run pmc_valu2 --pmc SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU --kernel-trace
echo "[$(date +%T)] done" >&2
