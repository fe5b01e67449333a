#!/bin/bash
# Instruction-fetch counters of the C2 SPA decode (is the unrolled slot code
# streamed from L2 every iteration?).  Lists the SQ/SQC fetch counters first.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r05_icache; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o -E "\b(SQC?_[A-Z0-9_]*(IFETCH|ICACHE|INST_LEVEL|WAIT_INST|IC_)[A-Z0-9_]*)\b" $O/avail.txt | sort -u > $O/fetch_counters.txt || true
cat $O/fetch_counters.txt | tr '\n' ' '; echo
C=""
for c in SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQC_ICACHE_MISSES_DUPLICATE; do
  if grep -q -w "$c" $O/avail.txt; then C="$C $c"; fi
done
echo "pmc:$C"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p -o p -- python3 bench.py --workload c2 --steps 2 --warmup 0 --no-cpu-baseline --streams 1 --roofline-launches 0 > $O/run.txt 2>&1 || { tail -5 $O/run.txt; exit 3; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/p/*counter_collection.csv")[0]
agg = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if "decode_v2" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Dispatch_Id"]] += 1
print("dispatches", len(n), {k: round(v / max(1, len(n))) for k, v in agg.items()})
PY
