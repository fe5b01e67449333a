#!/bin/bash
# One GPU call: parity suite, bench lines for every workload, and the default
# bench command under rocprofv3 --kernel-trace --stats.  usage: tools/gpu_check.sh TAG
set -u
TAG=${1:-q}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
echo "[$(date +%T)] pytest" >&2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 12; }
tail -2 $O/pytest_gpu.log
for wl in c2 c3 c4 c5 c5ra; do
  echo "[$(date +%T)] bench $wl" >&2
  timeout -k 10 300 python bench.py --workload $wl --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 13; }
done
echo "[$(date +%T)] default bench under rocprof" >&2
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 14; }
echo "[$(date +%T)] done" >&2
