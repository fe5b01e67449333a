#!/bin/bash
# A/B build of the working tree with extra compile flags on decoder_v2.hip:
# qkd_ldpc_v_amd/ab/<name>/.  usage: tools/build_ab_flag.sh <name> -DFLAG ...
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
HIPFLAGS=$(make -s -f Makefile -f - print-hipflags <<'MK'
print-hipflags:
	@echo $(HIPFLAGS) $(V2FLAGS)
MK
)
C=qkd_ldpc_v_amd/csrc
mkdir -p qkd_ldpc_v_amd/ab/$NAME
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c $C/decoder_v2.hip -o qkd_ldpc_v_amd/ab/$NAME/decoder_v2.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $C/decoder.o qkd_ldpc_v_amd/ab/$NAME/decoder_v2.o $C/trials.o \
    $C/order.o $C/capi.o $C/loaders.o $C/relabel.o -lz -o qkd_ldpc_v_amd/ab/$NAME/libqkdldpc_hip.so
rm qkd_ldpc_v_amd/ab/$NAME/decoder_v2.o
echo "built qkd_ldpc_v_amd/ab/$NAME ($*)"
