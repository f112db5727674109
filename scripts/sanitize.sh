#!/bin/bash
# Host sanitizer runs of the C++ test-suite: ThreadSanitizer and
# AddressSanitizer+UBSan builds in build-tsan/ and build-asan/ (CPU only; no GPU code involved).
# Built with the ROCm LLVM clang++ (compiler-rt runtimes): gcc-11's libtsan does not intercept
# pthread_cond_clockwait and reports false "double lock" races on condition_variable::wait_for.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
JOBS="${JOBS:-8}"
CXX="${SAN_CXX:-/opt/rocm/llvm/bin/clang++}"
for san in "thread" "address,undefined"; do
  dir="$ROOT/build-$( [ "$san" = thread ] && echo tsan || echo asan )"
  cmake -S "$ROOT" -B "$dir" -G Ninja -DCMAKE_BUILD_TYPE=RelWithDebInfo -DCMAKE_CXX_COMPILER="$CXX" \
    -DDEVSPACE_SANITIZE="$san" > /dev/null
  ninja -C "$dir" -j "$JOBS" devspace_tests devspace > /dev/null
  cp -f "$ROOT/bin/devspace-helper" "$dir/bin/devspace-helper"
  echo "== $san"
  TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" \
  ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:detect_odr_violation=0" UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1" \
    "$dir/bin/devspace_tests" "${@}"
done
