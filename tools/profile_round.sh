#!/bin/bash
# Round profile on the GPU box: the default bench command under
# rocprofv3 --kernel-trace --stats, then separate PMC passes (HBM bytes, VALU,
# instruction cache) for the C2 and C3 workloads.  Writes gpurun_out/round_prof/.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/round_prof
mkdir -p "$OUT"
pass() {  # name, workload-args, rocprof args...
  local name=$1; local bargs=$2; shift 2
  echo "[$(date +%T)] pass $name" >&2
  timeout -k 10 500 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python bench.py $bargs \
      > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pass $name failed rc=$rc" >&2; tail -20 "$OUT/$name.log" >&2; exit $rc; fi
}
pass default_trace "" --kernel-trace --stats
for wl in c2 c3; do
  B="--workload $wl --steps 5 --warmup 1 --no-cpu-baseline --streams 1 --roofline-launches 0"
  pass ${wl}_trace "$B" --kernel-trace --stats
  pass ${wl}_fetch "$B" --pmc FETCH_SIZE --kernel-trace
  pass ${wl}_write "$B" --pmc WRITE_SIZE --kernel-trace
  pass ${wl}_sq "$B" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace
  pass ${wl}_sq2 "$B" --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace
  pass ${wl}_valu "$B" --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 --kernel-trace
done
echo "[$(date +%T)] done" >&2
