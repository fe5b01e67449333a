#!/bin/bash
# Round-6 measurements on one GPU box, in stages that each fit one gpurun call:
#   STAGE=test   the GPU parity suite
#   STAGE=prof   rocprofv3 kernel-trace + PMC passes of WLS (profile_round.sh),
#                summarised into profiles/r06/ + profiles/pmc_<wl>.json
#   STAGE=bench  bench lines of WLS (DEFAULT=1: the default command too), each
#                priced by the pmc_<wl>.json of the same box/build when present
# Everything the stage writes under profiles/ is copied to gpurun_out/r06_sync/
# (gpurun brings back gpurun_out/ only).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${TAG:-r06a}
mkdir -p gpurun_out/r06_sync/r06
case ${STAGE:-test} in
  test)
    timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread --maxfail=5 \
      > gpurun_out/r06_sync/r06/${TAG}_pytest_gpu.log 2>&1; rc=$?
    tail -n 3 gpurun_out/r06_sync/r06/${TAG}_pytest_gpu.log
    [ $rc -eq 0 ] || exit 11 ;;
  prof)
    CLEAN=1 DEFAULT=${DEFAULT:-0} WLS="$WLS" PASSES="${PASSES:-trace fetch write sq sq2 valu tcc ea stall}" \
      timeout -k 10 1000 tools/profile_round.sh || exit 12
    python tools/round_summary.py gpurun_out/round_prof $TAG r06 > gpurun_out/r06_sync/${TAG}_summary.log 2>&1 || exit 13
    cp -r profiles/r06/. gpurun_out/r06_sync/r06/
    for wl in $WLS; do cp profiles/pmc_$wl.json gpurun_out/r06_sync/ 2>/dev/null || true; done ;;
  bench)
    TAG=$TAG DEFAULT=${DEFAULT:-1} WLS="$WLS" CPU_S=${CPU_S:-8} timeout -k 10 1000 tools/round_bench.sh || exit 14
    cp gpurun_out/round_bench/${TAG}_bench_*.json gpurun_out/r06_sync/r06/ ;;
esac
echo done
