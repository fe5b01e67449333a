#!/bin/bash
# 8-wave split parts: split parity tests, then C4 / C4 (ii) bench + C4 (ii) stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_half; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "c4 or split" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 10; }
tail -2 $O/pytest.log
for wl in c4g c4; do
  timeout -k 10 300 python bench.py --workload $wl --steps 6 --warmup 1 --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/$wl.json'))
print('$wl', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), 'iters', round(d['mean_iterations'],3), 'fer', d['fer'], 'lanes', d['config']['lanes_per_frame'], 'wgs', d['config']['workgroups'])"
done
QLDPC_DIAG_STAMPS=1 timeout -k 10 300 python bench.py --workload c4g --steps 1 --warmup 0 --no-cpu-baseline --streams 1 --roofline-launches 0 > $O/st.json 2> $O/st.err || { tail -5 $O/st.err; exit 4; }
echo "c4g $(grep phase_stamps $O/st.err | tail -1)"
