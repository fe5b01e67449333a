#!/bin/bash
# Bench lines of a round on the GPU box: `bench.py` (the default command, with
# its cpu_baseline) and `bench.py --workload <wl>` for each workload in WLS,
# one JSON line each under gpurun_out/round_bench/<tag>_bench_<wl>.json.
#   TAG=r03d WLS="c3 c5" DEFAULT=1 tools/round_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/round_bench
TAG=${TAG:-r03}
mkdir -p "$OUT"
run() {  # name, bench args
  local name=$1; shift
  echo "[$(date +%T)] bench $name" >&2
  timeout -k 10 300 python bench.py "$@" > "$OUT/${TAG}_bench_$name.json" 2> "$OUT/${TAG}_bench_$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "bench $name failed rc=$rc" >&2; tail -20 "$OUT/${TAG}_bench_$name.err" >&2; exit $rc; fi
}
if [ "${DEFAULT:-1}" = 1 ]; then run default; fi
for wl in ${WLS:-c3 c5}; do run "$wl" --workload "$wl" --cpu-baseline-seconds ${CPU_S:-8}; done
echo "[$(date +%T)] done" >&2
