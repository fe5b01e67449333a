#!/bin/bash
# Batch-seam repeatability: three reps each of the C2 one-call seam and the
# C2 / C5 / C4 multi-combination sweeps (same inputs as gen_seam.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r06_seamreps; mkdir -p $O
M=tests/golden/matrices/c2_n10240_m2201.alist.gz
M5=tests/golden/matrices/c5_n10240_m2048.sp2.gz
M4=tests/golden/matrices/c4s_n102400_m32001.alist.gz
printf '0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n' > $O/q_c2.txt
printf '0.0156\n0.0156\n0.0156\n0.0156\n0.0156\n0.0156\n0.0156\n0.0156\n' > $O/q_c5.txt
printf '0.038\n0.038\n0.038\n0.038\n' > $O/q_c4.txt
for rep in 1 2 3; do
  timeout -k 10 240 tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 4096 1022025 0 >> $O/seam_c2.txt 2>&1 || exit 12
  timeout -k 10 240 tests/dropin/batch_check sweep $M 1 0 0 0 $O/q_c2.txt 50 4096 1022025 >> $O/sweep_c2.txt 2>&1 || exit 13
  timeout -k 10 240 tests/dropin/batch_check sweep $M5 3 5 0.7 0.99 $O/q_c5.txt 50 4096 5555 >> $O/sweep_c5.txt 2>&1 || exit 14
  timeout -k 10 240 tests/dropin/batch_check sweep $M4 1 0 0 0 $O/q_c4.txt 50 128 1022025 >> $O/sweep_c4.txt 2>&1 || exit 15
done
for w in c2 c5 c4; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || exit 11
  python -c "import json;d=json.load(open('$O/bench_$w.json'));print('bench $w', round(d['ms_per_step'],2), 'ms/step')"
done
cat $O/seam_c2.txt $O/sweep_c2.txt $O/sweep_c5.txt $O/sweep_c4.txt
