#!/bin/bash
# The CPU test suite (pytest -m "not gpu") with every host translation unit of
# libfitoct (fitoct_amd/build_san/libfitoct.so: argument checks, basis, layout, Stan
# CSV, diagnostics, L-BFGS / ADVI drivers), the C oracle and the oracle-backed
# drivers (oracle/build_san/) under AddressSanitizer + UndefinedBehaviorSanitizer
# (SURVEY.md §5).  Device code is not instrumented (GPU sanitizers are not available
# on this pool).  Leak checking is off: the Python interpreter itself is not
# instrumented and holds its allocations until exit.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
python -m fitoct_amd.build --sanitize > /dev/null && make -s -C oracle sanitize || exit 1
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
export LD_LIBRARY_PATH=/opt/rocm/lib/llvm/lib:${LD_LIBRARY_PATH}
export FITOCT_SANITIZE=1 FITOCT_LIB_PATH=$PWD/fitoct_amd/build_san/libfitoct.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:symbolize=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD=$RT python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
