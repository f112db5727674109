#!/bin/bash
# Host sanitizer runs of the C++ test-suite: ThreadSanitizer and
# AddressSanitizer+UBSan builds in build-tsan/ and build-asan/ (CPU only; no GPU code involved).
# TSan uses the ROCm LLVM clang++ (compiler-rt): gcc-11's libtsan does not intercept
# pthread_cond_clockwait and reports false "double lock" on condition_variable::wait_for.
# ASan+UBSan uses g++ (compiler-rt's ASan double-registers string-literal globals here).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
JOBS="${JOBS:-8}"
build_and_run() {
  local san="$1" dir="$2" cxx="$3"
  cmake -S "$ROOT" -B "$dir" -G Ninja -DCMAKE_BUILD_TYPE=RelWithDebInfo -DCMAKE_CXX_COMPILER="$cxx" \
    -DDEVSPACE_SANITIZE="$san" > /dev/null
  ninja -C "$dir" -j "$JOBS" devspace_tests devspace > /dev/null
  cp -f "$ROOT/bin/devspace-helper" "$dir/bin/devspace-helper"
  echo "== $san ($cxx)"
  TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" \
  ASAN_OPTIONS="detect_leaks=1:halt_on_error=1" UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1" \
    "$dir/bin/devspace_tests" "${@:4}"
}
build_and_run thread "$ROOT/build/tsan" "${TSAN_CXX:-/opt/rocm/llvm/bin/clang++}" "$@"
build_and_run address,undefined "$ROOT/build/asan" "${ASAN_CXX:-g++}" "$@"
# The CLI itself under both sanitizers, driven by the end-to-end suite (local cluster).
for b in tsan asan; do
  echo "== e2e with build/$b/bin/devspace"
  DEVSPACE_BIN="$ROOT/build/$b/bin/devspace" TSAN_OPTIONS="halt_on_error=1" ASAN_OPTIONS="detect_leaks=0:halt_on_error=1" \
    python3 -m pytest -q -x "$ROOT/tests/test_e2e_cli.py" "$ROOT/tests/test_e2e_services.py" \
      "$ROOT/tests/test_e2e_tls.py" "$ROOT/tests/test_cloud_cli.py" "$ROOT/tests/test_e2e_helm.py" \
      "$ROOT/tests/test_e2e_apply.py" "$ROOT/tests/test_e2e_auth.py" "$ROOT/tests/test_e2e_recovery.py" \
      "$ROOT/tests/test_hostile_server.py" "$ROOT/tests/test_e2e_gpu_sched.py" "$ROOT/tests/test_e2e_throttle.py" \
      "$ROOT/tests/test_e2e_pull_wait.py" "$ROOT/tests/test_e2e_rbac.py" "$ROOT/tests/test_e2e_portforward_wan.py" 2>&1 | tail -1
done
