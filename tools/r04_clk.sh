#!/bin/bash
# Round-4: the claim timestamp stored at claim time instead of held in a
# register through the decode (4-9 fewer VGPR spills per instantiation): GPU
# parity, then A/B against the held form (ab/clk) on C2 / C3 / C5 / C5ra.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r04_clk; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread --maxfail=5 \
  > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 11
VARS="cur clk" WLS="c2 c3 c5 c5ra" REPS=2 STEPS=6 timeout -k 10 600 tools/ab_builds.sh || exit 12
echo done
