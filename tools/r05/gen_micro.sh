#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r05_genmicro; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o gm -- python3 tools/r05/gen_micro.py > $O/out.txt 2>&1 || { tail -20 $O/out.txt; exit 3; }
grep "n=" $O/out.txt
python3 - "$O" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/prof/*kernel_trace.csv")[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    if "trials" in r["Kernel_Name"]:
        print(r["Kernel_Name"][:40], r["Grid_Size_X"], r["Grid_Size_Y"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
PY
