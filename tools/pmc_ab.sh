#!/bin/bash
# VALU / LDS / wait counters of the decode kernel for A/B builds (product = "cur",
# others qkd_ldpc_v_amd/ab/<name>): usage VARS="cur x" WL=c2 tools/pmc_ab.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
WL=${WL:-c2}
B="--workload $WL --steps 2 --warmup 1 --no-cpu-baseline --streams 1 --roofline-launches 0"
for v in ${VARS:-cur}; do
  if [ $v = cur ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$v; fi
  O=gpurun_out/pmcab/${1:-q}_${v}_$WL; mkdir -p $O
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace -d $O/p1 -o run --output-format csv -- python bench.py $B > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 11; }
  python - "$O" "$v" <<'PY'
import sys, json
sys.path.insert(0, "tools")
from pmc_summary import summarize
o = summarize(sys.argv[1], "decode_v2", prefix="p1")
print(sys.argv[2], json.dumps({k: round(v) for k, v in sorted(o.items())}))
PY
done
