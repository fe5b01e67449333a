#!/bin/bash
# Load-cost probe for a stage-summing split scan (QL_FUSE_PROBE: the scan also
# issues the column's two 16-byte stage loads and its code byte): C4 / C4 (ii)
# product vs probe, alternating, + probe stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r05_fprobe; mkdir -p $O
for arm in prod fp prod fp; do
for wl in c4g c4; do
  if [ $arm = prod ]; then unset QLDPC_AB_BUILD; else export QLDPC_AB_BUILD=$arm; fi
  timeout -k 10 300 python bench.py --workload $wl --steps 6 --warmup 1 --no-cpu-baseline > $O/${arm}_${wl}.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$O/${arm}_${wl}.json'))
print('$arm $wl', round(d['value']/1e9,4), 'Gbit/s decode', round(d['decode_kernel_ms'],2), 'step', round(d['ms_per_step'],2), 'iters', round(d['mean_iterations'],3), 'fer', d['fer'])"
done
done
