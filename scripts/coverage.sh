#!/bin/bash
# Line coverage of the C++ CLI (the counterpart of the reference's scripts/coverage.bash, which
# runs `go test -race -coverprofile` per package): a gcov build in build/coverage, the C++ test
# suite, then the end-to-end suites driving that build's `devspace` against the bundled local
# cluster, then the same for the portable client (-DDEVSPACE_PORTABLE=ON: the POSIX platform
# layer and the stat-scan watcher; C++ suite, platform and sync-matrix tests), then a per-module
# summary of executed lines over both builds (scripts/coverage_summary.py).
#
#   scripts/coverage.sh [out.txt]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
B="$ROOT/build/coverage"
OUT="${1:-$B/coverage.txt}"
cmake -S "$ROOT" -B "$B" -G Ninja -DCMAKE_BUILD_TYPE=Debug -DDEVSPACE_COVERAGE=ON > /dev/null
ninja -C "$B" -j "${JOBS:-8}" devspace_tests devspace > /dev/null
find "$B" -name '*.gcda' -delete
cp -f "$ROOT/bin/devspace-helper" "$B/bin/devspace-helper"
echo "== C++ suite"
"$B/bin/devspace_tests" | tail -1
echo "== e2e suites with $B/bin/devspace"
# a failing test is reported (-rf) but does not stop the summary: coverage is what is measured here
DEVSPACE_BIN="$B/bin/devspace" python3 -m pytest -q -rf -p no:cacheprovider \
  "$ROOT/tests/test_e2e_cli.py" "$ROOT/tests/test_e2e_services.py" "$ROOT/tests/test_e2e_tls.py" \
  "$ROOT/tests/test_cloud_cli.py" "$ROOT/tests/test_e2e_helm.py" "$ROOT/tests/test_e2e_apply.py" \
  "$ROOT/tests/test_e2e_auth.py" "$ROOT/tests/test_e2e_recovery.py" "$ROOT/tests/test_hostile_server.py" \
  "$ROOT/tests/test_e2e_gpu_sched.py" "$ROOT/tests/test_cli_surface.py" "$ROOT/tests/test_e2e_throttle.py" \
  "$ROOT/tests/test_e2e_pull_wait.py" "$ROOT/tests/test_e2e_rbac.py" "$ROOT/tests/test_e2e_gpu_partitions.py" \
  "$ROOT/tests/test_e2e_image_layers.py" "$ROOT/tests/test_e2e_portforward_wan.py" \
  "$ROOT/tests/test_e2e_noninteractive.py" "$ROOT/tests/test_platform.py" 2>&1 | grep -E "^FAILED|passed|failed" || true
P="$ROOT/build/coverage-portable"
cmake -S "$ROOT" -B "$P" -G Ninja -DCMAKE_BUILD_TYPE=Debug -DDEVSPACE_COVERAGE=ON -DDEVSPACE_PORTABLE=ON \
  -DDEVSPACE_PYTHON=OFF "-DDEVSPACE_OUTPUT_DIR=$P/bin" > /dev/null
ninja -C "$P" -j "${JOBS:-8}" devspace_tests devspace > /dev/null
find "$P" -name '*.gcda' -delete
cp -f "$ROOT/bin/devspace-helper" "$P/bin/devspace-helper"
echo "== portable build: C++ suite"
"$P/bin/devspace_tests" | tail -1
echo "== portable build: platform, non-interactive and sync-matrix tests"
DEVSPACE_BIN="$P/bin/devspace" DEVSPACE_TESTS_BIN="$P/bin/devspace_tests" python3 -m pytest -q -rf -p no:cacheprovider \
  "$ROOT/tests/test_platform.py" "$ROOT/tests/test_e2e_noninteractive.py" "$ROOT/tests/test_sync_matrix_kube.py" 2>&1 \
  | grep -E "^FAILED|passed|failed" || true
python3 "$ROOT/scripts/coverage_summary.py" "$B" "$P" "$ROOT/src" | tee "$OUT"
