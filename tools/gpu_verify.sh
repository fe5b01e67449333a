#!/bin/bash
# One GPU call: parity suite + smoke() + default bench (and optional extra workloads).
# usage: WLS="c3 c5" tools/gpu_verify.sh TAG
set -u
TAG=${1:-v}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 12; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 13; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 14; }
python -c "import json; d=json.load(open('$O/bench_default.json')); print('default', round(d['value']/1e9,3), 'Gbit/s dec', round(d['decode_kernel_ms'],3), 'frac', round(d['roofline']['frac'],3))"
for wl in ${WLS:-}; do
  timeout -k 10 300 python bench.py --workload $wl --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 15; }
  python -c "import json; d=json.load(open('$O/bench_$wl.json')); print('$wl', round(d['value']/1e9,3), 'Gbit/s dec', round(d['decode_kernel_ms'],3))"
done
