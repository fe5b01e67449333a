#!/bin/bash
# Round-4 close: rocprofv3 kernel-trace + PMC passes of every bench workload at
# HEAD (tools/profile_round.sh), summarised here by tools/round_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
CLEAN=1 DEFAULT=1 WLS="c2 c3 c5 c5ra c4 c4g" PASSES="trace fetch write sq sq2 valu tcc ea stall" \
  timeout -k 10 1000 tools/profile_round.sh || exit 11
timeout -k 10 400 tools/r04_chunk.sh || exit 12
echo done
