#!/bin/bash
# Round-4: split message passes read the stage-position word alone (flags
# packed in it); the hybrid bit gather requests the next bit's entry one bit
# ahead; the trial generator runs two waves per 64 trials (GF(2) jump) —
# the whole GPU suite, A/B against the previous build (ab/m2old: C4), the
# gather without the prefetch (ab/ghpf0: C5), the generator with one wave
# (QLDPC_TRIAL_SPLIT=0: C2 seam), C4 / C4 (ii) traffic passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r04_m2; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread --maxfail=5 \
  > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 11
M=tests/golden/matrices/c2_n10240_m2201.alist.gz
for rep in 1 2; do for sp in 1 0; do
  QLDPC_TRIAL_SPLIT=$sp timeout -k 10 120 tests/dropin/batch_check time $M 1 0 0 0 0.0215 50 4096 1022025 0 > $O/seam_$sp.txt 2>&1 || { cat $O/seam_$sp.txt; exit 12; }
  echo "trial_split=$sp: $(cat $O/seam_$sp.txt)"
done; done
VARS="cur m2old" WLS="c4 c4g" REPS=2 STEPS=5 timeout -k 10 500 tools/ab_builds.sh || exit 13
VARS="cur ghpf0" WLS="c5 c5ra" REPS=2 STEPS=5 timeout -k 10 500 tools/ab_builds.sh || exit 14
WLS="c4 c4g" PASSES="fetch write ea tcc" DEFAULT=0 timeout -k 10 300 tools/profile_round.sh || exit 15
echo done
