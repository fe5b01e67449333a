#!/bin/bash
# Round 6 GPU check: the GPU suite, smoke, then short bench lines of the
# default workload and the split-frame workloads (the per-device split-decode
# serialisation changes their 2-stream step).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
TAG=${TAG:-r06a}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --maxfail=8 \
  > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -12 $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 3; }
cat $O/smoke.txt
for wl in ${WLS:-c2 c4 c4g}; do
  timeout -k 10 240 python bench.py --workload $wl --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail $O/bench_$wl.err; exit 3; }
  python -c "import json; d=json.load(open('$O/bench_$wl.json')); print('$wl', d['value']/1e9, d['ms_per_step'], d['decode_kernel_ms'], d['roofline']['frac'])"
done
exit $rc
