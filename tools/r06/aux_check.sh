#!/bin/bash
# Round 6: the frame builders / claim weight / key compare with 1024 threads per
# frame for n >= 32768 and 16-byte key compares: the pipeline and generator GPU
# tests, then rocprof kernel stats of one serial C4 (ii) / C4 / C2 run each and
# the 2-stream bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r06_aux; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_rate_adapt.py tests/test_run_trials.py tests/test_trial_generator.py -k "pipeline or frames or keys or run_trials or rate or c4_100k_split_variant or claim" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -le 1 ] || exit $rc
for wl in c4g c4 c2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$wl -o run --output-format csv -- python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --streams 1 --roofline-launches 0 > $O/prof_$wl.log 2>&1 || { tail -5 $O/prof_$wl.log; exit 4; }
  python3 - $O/prof_$wl/run_kernel_stats.csv $wl <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r['AverageNs']) > 5000: print(sys.argv[2], r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
done
for rep in 1 2; do
for wl in c4g c4 c2; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $O/${wl}_$rep.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${wl}_$rep.json'))
print('$wl', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2))"
done
done
exit $rc
