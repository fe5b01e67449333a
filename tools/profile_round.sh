#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel-trace summaries and separate
# PMC passes (one counter group per run, --kernel-trace only, as
# MI355X_MICROARCH.md prescribes) of `bench.py --workload <wl>` for each
# workload in WLS.  Writes gpurun_out/round_prof/<wl>_<pass>/;
# tools/round_summary.py turns them into profiles/<round>/ + profiles/pmc_<wl>.json.
#   WLS="c2 c3" PASSES="trace fetch write sq sq2 valu tcc ea lds" DEFAULT=1 tools/profile_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/round_prof
if [ "${CLEAN:-0}" = 1 ]; then rm -rf "$OUT"; fi  # (a round's first call: no passes of an older build mix in)
mkdir -p "$OUT"
pass() {  # name, bench args, rocprof args...
  local name=$1; local bargs=$2; shift 2
  echo "[$(date +%T)] pass $name" >&2
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python bench.py $bargs \
      > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pass $name failed rc=$rc" >&2; tail -20 "$OUT/$name.log" >&2; exit $rc; fi
}
if [ "${DEFAULT:-1}" = 1 ]; then
  pass default_trace "" --kernel-trace --stats
fi
for wl in ${WLS:-c2 c3}; do
  B="--workload $wl --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --streams 1 --roofline-launches 0"
  for p in ${PASSES:-trace fetch write sq sq2 valu}; do
    case $p in
      trace) pass ${wl}_trace "$B" --kernel-trace --stats ;;
      fetch) pass ${wl}_fetch "$B" --pmc FETCH_SIZE --kernel-trace ;;
      write) pass ${wl}_write "$B" --pmc WRITE_SIZE --kernel-trace ;;
      sq)    pass ${wl}_sq "$B" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace ;;
      sq2)   pass ${wl}_sq2 "$B" --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace ;;
      valu)  pass ${wl}_valu "$B" --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 --kernel-trace ;;
      tcc)   pass ${wl}_tcc "$B" --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace ;;
      ea)    pass ${wl}_ea "$B" --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace ;;
      stall) pass ${wl}_stall "$B" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace ;;
      lds)   pass ${wl}_lds "$B" --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL --kernel-trace ;;
      *) echo "unknown pass $p" >&2; exit 2 ;;
    esac
  done
done
echo "[$(date +%T)] done" >&2
