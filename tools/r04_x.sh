#!/bin/bash
# Round-4: split-frame exchange gather — C4 parity (split tests), then the C4 /
# C4 (ii) bench lines with the exchange layout (QLDPC_SPLIT_X=1, default) and
# the term-major stage (0), alternating, then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r04_x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "c4 or split" --timeout 200 --timeout-method thread -x \
  > $O/pytest_split.log 2>&1; rc=$?
tail -3 $O/pytest_split.log
[ $rc -eq 0 ] || exit 11
for rep in 1 2; do
  for x in 1 0; do
    for wl in c4 c4g; do
      QLDPC_SPLIT_X=$x timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 5 > $O/b_${wl}_x${x}_$rep.json 2> $O/b_${wl}_x${x}_$rep.err || exit 12
      python - $O/b_${wl}_x${x}_$rep.json $x <<'PY'
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], "Gbit/s", round(d["value"]/1e9,4), "dec ms", round(d["decode_kernel_ms"],3), "iters", d["mean_iterations"], "fer", d["fer"])
PY
    done
  done
done
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread --maxfail=5 > $O/pytest_all.log 2>&1; rc=$?
tail -3 $O/pytest_all.log
exit $rc
