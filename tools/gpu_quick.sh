#!/bin/bash
# Quick GPU check: parity suite + C2/C3 bench lines.  usage: tools/gpu_quick.sh [tag]
TAG=${1:-q}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1 || { tail -30 gpurun_out/t_$TAG.log; exit 12; }
tail -2 gpurun_out/t_$TAG.log
for wl in c2 c3 c5 c5ra; do
  timeout -k 10 300 python bench.py --workload $wl --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/b_${wl}_$TAG.json 2> gpurun_out/b_${wl}_$TAG.err || exit 13
done
timeout -k 10 300 python bench.py --workload c2 --steps 8 --warmup 2 --streams 1 --no-cpu-baseline > gpurun_out/b_c2s1_$TAG.json 2> gpurun_out/b_c2s1_$TAG.err || exit 14
