#!/bin/bash
# C5 quick check: hybrid-shape parity tests, then bench sweep points (POINTS)
# and the c5 / c5ra workloads, one line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/c5q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "${TESTS:-c5 or rate_adapt}" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 12; }
tail -1 $O/pytest.log
for i in ${POINTS:-2 9 20}; do
  timeout -k 10 120 python bench.py --workload c5ra --c5-point $i --steps 3 --warmup 1 --no-cpu-baseline \
      --roofline-launches 1 > $O/p$i.json 2> $O/p$i.err || { tail -5 $O/p$i.err; exit 3; }
  python -c "import json; d=json.load(open('$O/p$i.json')); print('point', $i, round(d['value']/1e9,3), round(d['ms_per_step'],2), round(d['decode_kernel_ms'],2))"
done
for wl in ${WLS:-c5 c5ra}; do
  timeout -k 10 120 python bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 4; }
  python -c "import json; d=json.load(open('$O/$wl.json')); print('$wl', round(d['value']/1e9,3), round(d['ms_per_step'],2), round(d['decode_kernel_ms'],2))"
done
