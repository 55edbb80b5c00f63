#!/bin/bash
# SURVEY 5 sanitizer run (host code only; GPU sanitizers are not available
# on the pool): the library's host code and the C oracles built with
# AddressSanitizer + UndefinedBehaviorSanitizer (clang), then the CPU test
# suite (-m "not gpu") against them with clang's ASan runtime preloaded.
# Any ASan / UBSan report aborts the run (halt_on_error).
#   scripts/sanitize.sh [pytest args...]   ->  log in gpurun_out/sanitize.log
set -euo pipefail
cd "$(dirname "$0")/.."
make -C ska-sdp-func_amd SAN=1 -j"${JOBS:-8}" >/dev/null
LLVM=/opt/rocm/lib/llvm
RT=$(ls "$LLVM"/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -n1)
export SDP_SANITIZE=1
export SKA_SDP_FUNC_LIB_DIR="$PWD/ska-sdp-func_amd/san"
# Python and torch keep memory to exit and mix allocators across their own
# libraries: leak and mismatch checks off; every error in our code halts.
export ASAN_OPTIONS=detect_leaks=0:alloc_dealloc_mismatch=0:detect_odr_violation=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
mkdir -p gpurun_out
LD_PRELOAD="$RT" python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider \
    "$@" 2>&1 | tee gpurun_out/sanitize.log
