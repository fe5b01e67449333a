#!/bin/bash
# Round 5: the segment-parallel trial generator and the pipelined batch seam.
# GPU parity of the generator / seam / drop-in / driver tests, then generation
# times (bench.py's trial_generation_s), the C2 seam call, and multi-combination
# seam sweeps (ms per combination vs the bench step).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_gen; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 10; }
tail -3 $O/pytest.log
fi
for w in c2 c4 c4g c5 c5ra; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 11; }
  python -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w', round(d['value']/1e9,3), 'Gbit/s', round(d['ms_per_step'],2), 'ms/step gen', round(d['trial_generation_s']*1e3,3), 'ms first', round(d['trial_generation_first_call_s']*1e3,1))"
done
M=tests/golden/matrices/c2_n10240_m2201.alist.gz
timeout -k 10 240 tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 4096 1022025 0 > $O/seam_c2.txt 2>&1 || { cat $O/seam_c2.txt; exit 12; }
echo "seam c2: $(cat $O/seam_c2.txt)"
printf '0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n0.0215\n' > $O/q_c2.txt
timeout -k 10 240 tests/dropin/batch_check sweep $M 1 0 0 0 $O/q_c2.txt 50 4096 1022025 > $O/sweep_c2.txt 2>&1 || { cat $O/sweep_c2.txt; exit 13; }
echo "sweep c2: $(cat $O/sweep_c2.txt)"
M5=tests/golden/matrices/c5_n10240_m2048.sp2.gz
printf '0.0156\n0.0156\n0.0156\n0.0156\n0.0156\n0.0156\n0.0156\n0.0156\n' > $O/q_c5.txt  # the bench's c5 point
timeout -k 10 240 tests/dropin/batch_check sweep $M5 3 5 0.7 0.99 $O/q_c5.txt 50 4096 5555 > $O/sweep_c5.txt 2>&1 || { cat $O/sweep_c5.txt; exit 14; }
echo "sweep c5: $(cat $O/sweep_c5.txt)"
M4=tests/golden/matrices/c4s_n102400_m32001.alist.gz
printf '0.038\n0.038\n0.038\n0.038\n' > $O/q_c4.txt
timeout -k 10 240 tests/dropin/batch_check sweep $M4 1 0 0 0 $O/q_c4.txt 50 128 1022025 > $O/sweep_c4.txt 2>&1 || { cat $O/sweep_c4.txt; exit 15; }
echo "sweep c4: $(cat $O/sweep_c4.txt)"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o seam -- tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 4096 1022025 0 > $O/seam_prof.txt 2>&1 || { tail -20 $O/seam_prof.txt; exit 16; }
find $O/prof -name "*stats*"
