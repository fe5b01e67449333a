#!/bin/bash
# A/B of the min-sum bit gather (QLDPC_VNG=1, default) against the VN phases (0).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/vng
for wl in ${WLS:-c3}; do for v in 1 0; do
  QLDPC_VNG=$v timeout -k 10 200 python bench.py --workload $wl --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/vng/${wl}_$v.json 2> gpurun_out/vng/${wl}_$v.err || { tail -5 gpurun_out/vng/${wl}_$v.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/vng/${wl}_$v.json')); print('$wl vng=$v', round(d['value']/1e9,4), 'Gbit/s dec', round(d['decode_kernel_ms'],3), 'iters', round(d['mean_iterations'],3))"
done; done
