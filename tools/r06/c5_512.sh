#!/bin/bash
# Round 6, verdict item 3: the C5 workload at BASELINE's per-GPU shape (batch
# 4096 over 8 GPUs = 512 frames per GPU) against the 4096-per-GPU line on the
# same box; serial (1 stream) and pipelined (2 streams) steps, rocprof kernel
# stats of the 512 serial run, then the 26-point sweep at 512 per GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r06_c5_512; mkdir -p $O
T="timeout -k 10 180"
export TMPDIR=/tmp
$T python bench.py --workload c5ra --batch 512 --steps 40 --warmup 3 > $O/bench_c5ra_b512.json 2> $O/bench_c5ra_b512.err || exit 3
$T python bench.py --workload c5ra --batch 512 --steps 40 --warmup 3 --streams 1 --no-cpu-baseline > $O/bench_c5ra_b512_s1.json 2> $O/bench_c5ra_b512_s1.err || exit 3
$T python bench.py --workload c5ra --batch 4096 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5ra_b4096.json 2> $O/bench_c5ra_b4096.err || exit 3
$T python bench.py --workload c5ra --batch 4096 --steps 10 --warmup 2 --streams 1 --no-cpu-baseline > $O/bench_c5ra_b4096_s1.json 2> $O/bench_c5ra_b4096_s1.err || exit 3
$T rocprofv3 --kernel-trace --stats -d $O/prof512 -o run -- python bench.py --workload c5ra --batch 512 --steps 20 --warmup 2 --streams 1 --no-cpu-baseline > $O/prof512.log 2>&1 || exit 3
find $O/prof512 -name '*kernel_stats.csv' -exec cp {} $O/c5ra_b512_serial_kernel_stats.csv \;
echo "c5ra 512 lines done"
BATCH=512 STEPS=10 bash tools/c5_sweep.sh > $O/sweep512.log 2>&1 || { tail -5 $O/sweep512.log; exit 3; }
tail -3 $O/sweep512.log
