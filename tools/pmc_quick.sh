#!/bin/bash
# Two PMC passes (instruction mix, LDS/wait) for one workload: WL=c3 tools/pmc_quick.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
WL=${WL:-c3}; O=gpurun_out/pmcq/${1:-q}_$WL; mkdir -p $O
B="--workload $WL --steps 2 --warmup 1 --no-cpu-baseline --streams 1 --roofline-launches 0"
i=0
for ctr in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $O/p$i -o run --output-format csv -- python bench.py $B > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1$i; }
done
python - "$O" <<'PY'
import sys, json
sys.path.insert(0, "tools")
from pmc_summary import summarize
o = {}
for p in ("p1", "p2"):
    o.update(summarize(sys.argv[1], "decode_v2", prefix=p))
print(json.dumps({k: round(v) for k, v in sorted(o.items())}))
PY
