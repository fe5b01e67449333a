#!/bin/bash
# Build the committed HEAD's product library as an A/B build: qkd_ldpc_v_amd/ab/<name>/
# (compare with tools/ab_builds.sh VARS="cur <name>").  usage: tools/build_ab_head.sh [name] [rev]
set -e
NAME=${1:-prev}; REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
cd "$ROOT"
for f in $(git ls-files qkd_ldpc_v_amd/csrc include Makefile); do mkdir -p "$TMP/$(dirname $f)"; git show $REV:$f > "$TMP/$f"; done
make -C "$TMP" -j8 qkd_ldpc_v_amd/libqkdldpc_hip.so > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
mkdir -p "$ROOT/qkd_ldpc_v_amd/ab/$NAME"
cp "$TMP/qkd_ldpc_v_amd/libqkdldpc_hip.so" "$ROOT/qkd_ldpc_v_amd/ab/$NAME/"
rm -rf "$TMP"
echo "built $REV -> qkd_ldpc_v_amd/ab/$NAME"
