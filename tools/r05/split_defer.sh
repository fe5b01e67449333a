#!/bin/bash
# Split frames' deferred exit test: split parity (product + wave-fence arm), then
# C4 / C4 (ii) bench of the product (defer, workgroup barrier), d0 (test first,
# three group barriers) and d2 (defer, wave-local fence) + C4 (ii) stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_defer; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "c4 or split" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 10; }
tail -1 $O/pytest.log
QLDPC_AB_BUILD=d2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "c4 or split" > $O/pytest_d2.log 2>&1 || { tail -40 $O/pytest_d2.log; exit 11; }
tail -1 $O/pytest_d2.log
for arm in prod d0 d2 prod; do
for wl in c4g c4; do
  if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
  timeout -k 10 300 python bench.py --workload $wl --steps 6 --warmup 1 --no-cpu-baseline > $O/${arm}_${wl}.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${arm}_${wl}.json'))
print('$arm $wl', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), 'iters', round(d['mean_iterations'],3), 'fer', d['fer'])"
done
done
unset QLDPC_AB_BUILD
QLDPC_DIAG_STAMPS=1 timeout -k 10 300 python bench.py --workload c4g --steps 1 --warmup 0 --no-cpu-baseline --streams 1 --roofline-launches 0 > $O/st.json 2> $O/st.err || { tail -5 $O/st.err; exit 4; }
echo "c4g $(grep phase_stamps $O/st.err | tail -1)"
