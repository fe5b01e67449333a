#!/bin/bash
# PMC counters of the trial generator's kernels (tools/r05/gen_micro.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r05_genpmc; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $O/p1 -o p1 -- python3 tools/r05/gen_micro.py > $O/p1.txt 2>&1 || { tail -5 $O/p1.txt; exit 3; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o p2 -- python3 tools/r05/gen_micro.py > $O/p2.txt 2>&1 || { tail -5 $O/p2.txt; exit 4; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
for p in ("p1", "p2"):
    f = glob.glob(f"{sys.argv[1]}/{p}/*counter_collection.csv")[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "trials_draw" not in r["Kernel_Name"]:
            continue
        key = (r["Grid_Size"] if "Grid_Size" in r else r.get("Grid_Size_X", ""), r["Dispatch_Id"])
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    seen = {}
    for key, d in agg.items():
        g = key[0]
        if g in seen:
            continue
        seen[g] = 1
        print(p, g, {k: round(v) for k, v in d.items()})
PY
