#!/bin/bash
# Static VALU / SALU / LDS instruction counts per 4-slot group of the V2
# decoder, per pass, for one instantiation.  usage: tools/slot_cost.sh [ALG] [R]
ALG=${1:-0}; R=${2:-44}
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S \
  -o /tmp/v2_cost.s qkd_ldpc_v_amd/csrc/decoder_v2.hip 2>/dev/null || exit 1
RG=${3:-0}
SYM="_ZN5qldpc12_GLOBAL__N_116decode_v2_kernelILi${ALG}ELi${R}ELi${RG}EEEvNS_10DecodeArgsE"
awk -v sym="$SYM:" '$1==sym{on=1} on&&/s_endpgm/{on=0} on' /tmp/v2_cost.s > /tmp/v2_kern.s
awk '/buffer_load_dwordx4/{ if (n) printf "%d:%d/%d/%d ", n, v, s, d; n++; v=0; s=0; d=0; next}
     /^[ \t]+v_/{v++} /^[ \t]+s_/{s++} /^[ \t]+ds_/{d++}
     END{printf "tail:%d/%d/%d\n", v, s, d}' /tmp/v2_kern.s
grep -E "^[ \t]+v_" /tmp/v2_kern.s | wc -l | sed 's/^/total VALU static: /'
grep -A30 "^    .name:           $SYM" /tmp/v2_cost.s | grep -E "vgpr_count|vgpr_spill|sgpr_spill" | tr -s ' ' | tr '\n' ' '; echo
