#!/bin/bash
# Round-4: phase stamps of the K = 32 local-totals split (QLDPC_SPLIT_LOCAL=1)
# against the default 16-wave parts, C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for L in 1 0; do
  QLDPC_SPLIT_LOCAL=$L WLS=c4 timeout -k 10 200 tools/stamps.sh || exit 11
done
echo done
