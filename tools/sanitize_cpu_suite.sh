#!/bin/bash
# The CPU test suite under AddressSanitizer + UndefinedBehaviorSanitizer: the oracle (including the ack JSON parser,
# the health FSM and the message printer, which read untrusted bytes) and libowgs.so's host code (C-ABI argument
# checks, state mirror) built with clang's sanitizers, loaded into the unchanged tests.
#   bash tools/sanitize_cpu_suite.sh [pytest args]      (GPU box: PYTEST_MARK=gpu runs the GPU suite the same way)
set -e
cd "$(dirname "$0")/.."
make -s -C oracle sanitize
make -s -C openwhisk_amd san 2>&1 | grep -v warning || true
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export OWO_LIB=$PWD/oracle/build-san/libowsched_oracle.so
export OWGS_LIB=$PWD/openwhisk_amd/libowgs_san.so
# leaks: python and the ROCm runtime keep allocations until exit; everything else aborts the run
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD=$RT python -m pytest tests -q -x -m "${PYTEST_MARK:-not gpu}" -p no:cacheprovider "$@"
