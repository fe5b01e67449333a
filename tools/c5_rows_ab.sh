#!/bin/bash
# C5 R=0.5 hybrid: min-sum rows of the leading waves in LDS (default) vs all
# rows in global scratch (QLDPC_ROWS_LDS=0): parity tests then bench points.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/c5rows; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "c5 or rate_adapt" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 12; }
tail -1 $O/pytest.log
for v in 1 0; do
  for i in ${POINTS:-16 20 25}; do
    QLDPC_ROWS_LDS=$v timeout -k 10 120 python bench.py --workload c5ra --c5-point $i --steps 3 --warmup 1 \
        --no-cpu-baseline --roofline-launches 1 > $O/p${i}_r$v.json 2> $O/p${i}_r$v.err || { tail -5 $O/p${i}_r$v.err; exit 3; }
    python -c "import json; d=json.load(open('$O/p${i}_r$v.json')); print('rows_lds=$v', $i, round(d['value']/1e9,3), round(d['ms_per_step'],1), d['mean_iterations'])"
  done
done
