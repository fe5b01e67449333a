#!/bin/bash
# Round 6: split launches may overlap (two in flight per device when
# 2 (K - 1) < S, same shape) — the split and seam GPU tests, then C4 / C4 (ii)
# bench lines (2-stream step vs decode alone), 2 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r06_split_overlap; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_run_trials.py -k "c4 or split or run_trials" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
for wl in c4 c4g; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $O/${wl}_$rep.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${wl}_$rep.json'))
print('$wl', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2))"
done
done
exit $rc
