#!/bin/bash
# R=0.5 hybrid: edge share of the waves whose rows live in global scratch
# (QLDPC_RGLB_SHARE, percent) — parity at SHARE_TEST, then sweep points per share.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/c5share; mkdir -p $O
QLDPC_RGLB_SHARE=${SHARE_TEST:-75} timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "c5_other or rate_adapted_other" > $O/pytest.log 2>&1 \
    || { tail -30 $O/pytest.log; exit 12; }
tail -1 $O/pytest.log
for rep in 1 2; do for sh in ${SHARES:-100 85 75 65}; do for i in ${POINTS:-20}; do
  QLDPC_RGLB_SHARE=$sh timeout -k 10 120 python bench.py --workload c5ra --c5-point $i --steps 3 --warmup 1 \
      --no-cpu-baseline --roofline-launches 1 > $O/p${i}_$sh.json 2> $O/p${i}_$sh.err || { tail -5 $O/p${i}_$sh.err; exit 3; }
  python -c "import json; d=json.load(open('$O/p${i}_$sh.json')); print('share', $sh, 'point', $i, round(d['value']/1e9,4), round(d['ms_per_step'],2), round(d['decode_kernel_ms'],2))"
done; done; done
