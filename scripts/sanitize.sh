#!/bin/bash
# Host-code sanitizer builds of the native tests (csrc/tests/native_tests.cpp):
#   asan  = AddressSanitizer + UndefinedBehaviorSanitizer over ring kernels, parser,
#           graph passes, scheduler, mailbox and TCP networking;
#   tsan  = ThreadSanitizer over the concurrent parts (mailbox, dataflow, networking).
# CPU only (GPU ASAN / XNACK are not available on the GPU pool).
# Usage: scripts/sanitize.sh [asan|tsan|all]   (default all)
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=build/sanitize
mkdir -p "$OUT"
CXX=${CXX:-g++}
SRC="csrc/tests/native_tests.cpp csrc/runtime/graph.cpp csrc/runtime/scheduler.cpp
     csrc/runtime/textual.cpp csrc/runtime/net.cpp csrc/ring_cpu.cpp csrc/rss_fused_cpu.cpp
     csrc/rss_party_cpu.cpp"
# device entry points (mxh_*) are only reached with dev != 0, which the tests never use
LINK="-Wl,--unresolved-symbols=ignore-all -lssl -lcrypto -pthread"
COMMON="-std=c++17 -g -O1 -fno-omit-frame-pointer -msse4.1 -maes -pthread"
WHAT=${1:-all}
if [[ $WHAT == asan || $WHAT == all ]]; then
  $CXX $COMMON -fsanitize=address,undefined -fno-sanitize-recover=undefined $SRC $LINK \
    -o $OUT/native_tests_asan
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
    $OUT/native_tests_asan
fi
TSAN_CXX=${TSAN_CXX:-$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.tsan-x86_64.a >/dev/null 2>&1 && echo /opt/rocm/lib/llvm/bin/clang++ || echo $CXX)}
if [[ $WHAT == tsan || $WHAT == all ]]; then
  # clang: its TSAN runtime intercepts pthread_cond_clockwait (condition_variable::wait_for)
  $TSAN_CXX $COMMON -fsanitize=thread $SRC $LINK -o $OUT/native_tests_tsan
  TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 $OUT/native_tests_tsan conc
fi
echo "sanitizers: ok"
