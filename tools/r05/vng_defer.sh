#!/bin/bash
# Bit-gather frames' deferred exit test: GPU parity (whole file), then C3 / C5 /
# rate-adapted C5 / sweep points 2 and 20, product (deferred) vs vd0 (test
# first), alternating, + stamps of sweep point 20.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_vdefer; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 10; }
tail -1 $O/pytest.log
run() {  # arm label args...
  local arm=$1 lab=$2; shift 2
  if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
  timeout -k 10 300 python bench.py "$@" --steps 4 --warmup 1 --no-cpu-baseline > $O/${arm}_${lab}.json 2> $O/${lab}.err || { tail -5 $O/${lab}.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${arm}_${lab}.json'))
print('$arm $lab', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), 'iters', round(d['mean_iterations'],3), 'fer', d['fer'])"
}
for arm in prod vd0 prod vd0; do
  run $arm c3 --workload c3
  run $arm c5 --workload c5
  run $arm c5ra --workload c5ra
  run $arm p2 --workload c5ra --c5-point 2
  run $arm p20 --workload c5ra --c5-point 20
done
unset QLDPC_AB_BUILD
QLDPC_DIAG_STAMPS=1 timeout -k 10 300 python bench.py --workload c5ra --c5-point 20 --steps 1 --warmup 0 --no-cpu-baseline --streams 1 --roofline-launches 0 > $O/st.json 2> $O/st.err || { tail -5 $O/st.err; exit 4; }
echo "p20 $(grep phase_stamps $O/st.err | tail -1)"
