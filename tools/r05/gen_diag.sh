#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r05_gendiag; mkdir -p $O
for d in 0 1 2 4 7; do
  QLDPC_GEN_DIAG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$d -o d -- python3 tools/r05/gen_micro.py > $O/d$d.txt 2>&1 || { tail -5 $O/d$d.txt; exit 3; }
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/d$d/*kernel_stats.csv')[0])):
    if 'trials' in r['Name']: print('diag $d', r['Name'][30:52], r['Calls'], round(float(r['AverageNs'])/1e3,1), round(float(r['MinNs'])/1e3,1))
"
done
