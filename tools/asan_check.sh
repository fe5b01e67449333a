#!/bin/bash
# the library and its loader read QLDPC_* knobs / alternative builds only under QLDPC_DIAG=1
export QLDPC_DIAG=1
# The CPU test suite and the C++ drivers' host-only modes against the
# ASan + UBSan build of `make asan` (SURVEY.md §5 "race detection /
# sanitizers"): the product library's host code (C ABI, planner, bank
# relabelling, loaders), the CPU oracle and both C++ drivers.  Python and
# torch are not instrumented; clang's ASan runtime is preloaded for them.
set -euo pipefail
cd "$(dirname "$0")/.."
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export LD_LIBRARY_PATH="$(dirname "$RT")${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:alloc_dealloc_mismatch=0:detect_odr_violation=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
M=tests/golden/matrices
echo "== C++ drivers (host-only modes)"
for f in "c1_n1024_m220.alist 1" "c2_n10240_m2201.alist 1" "c5_n10240_m2048.sp2 3" "s1_n10_m5.sp1 2"; do
  name=${f% *}; fmt=${f#* }
  build/asan/host_mirror_check load $M/$name.gz $fmt
  build/asan/run_trial_check load $M/$name.gz $fmt
done
echo "== drop-in graph-cache keys and the syndrome check (host-only)"
build/asan/run_trial_check keycost $M/c2_n10240_m2201.alist.gz 1 50
if build/asan/run_trial_check badsyndrome $M/c1_n1024_m220.alist.gz 1; then echo "bad syndrome accepted" >&2; exit 1; fi
echo "== pytest -m 'not gpu' on the ASan libraries"
LD_PRELOAD=$RT QLDPC_ASAN=1 python -m pytest tests -q -m "not gpu" -p no:cacheprovider -x "$@"
