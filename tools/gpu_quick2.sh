#!/bin/bash
# Quick check: SPA/SPA-lin parity subset + C2/C3 bench.  usage: tools/gpu_quick2.sh TAG [pytest -k expr]
set -u
TAG=${1:-q}; K=${2:-}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 12; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 12; }
fi
tail -1 $O/pytest.log
for wl in ${WLS:-c2 c3}; do
  timeout -k 10 300 python bench.py --workload $wl --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 13; }
  python -c "import json; d=json.load(open('$O/bench_$wl.json')); print('$wl', round(d['value']/1e9,4), 'Gbit/s dec', round(d['decode_kernel_ms'],3), 'ms frac', round(d['roofline']['frac'],4))"
done
