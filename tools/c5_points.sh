#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/c5pts; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "c5" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 12; }
tail -1 $O/pytest.log
for i in 0 7 16; do
  timeout -k 10 120 python bench.py --workload c5ra --c5-point $i --steps 3 --warmup 1 --no-cpu-baseline --roofline-launches 1 > $O/p$i.json 2> $O/p$i.err || { tail -5 $O/p$i.err; exit 3; }
  python -c "import json; d=json.load(open('$O/p$i.json')); print($i, round(d['value']/1e9,3), round(d['ms_per_step'],1))"
done
