#!/bin/bash
# Trial generator: GPU parity of the generator-dependent tests, then kernel times.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_gencheck; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_trial_generator.py tests/test_run_trials.py tests/test_dropin.py tests/test_simulation.py tests/test_rate_adapt.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 10; }
tail -2 $O/pytest.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o p -- python3 tools/r05/gen_micro.py > $O/micro.txt 2>&1 || { tail -5 $O/micro.txt; exit 3; }
grep "n=" $O/micro.txt
python3 - "$O" <<'PY'
import csv, glob, sys, itertools
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/p/*kernel_trace.csv")[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
seen = [((r["Kernel_Name"][30:50], r["Grid_Size_X"], r["Grid_Size_Y"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows if "trials" in r["Kernel_Name"]]
for k, g in itertools.groupby(seen, key=lambda t: t[0]):
    v = [x[1] for x in g]
    print(k, len(v), round(min(v), 1), "us")
PY
M=tests/golden/matrices/c2_n10240_m2201.alist.gz
timeout -k 10 240 tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 4096 1022025 0 > $O/seam_c2.txt 2>&1 || { cat $O/seam_c2.txt; exit 12; }
echo "seam c2: $(cat $O/seam_c2.txt)"
timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 11; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', round(d['value']/1e9,3), 'Gbit/s', round(d['ms_per_step'],2), 'ms/step gen', round(d['trial_generation_s']*1e3,3))"
