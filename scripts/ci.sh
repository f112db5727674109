#!/bin/bash
# The pipeline every change runs (.github/workflows/ci.yml calls it; it runs the same by hand).
# The reference's CI builds and runs `go test -race` on every package
# (/root/reference/.travis.yml:7-20, /root/reference/scripts/coverage.bash:12-21); here:
#   build     the default (Linux platform layer) build, then `ctest` (C++ suite + platform seam)
#   portable  -DDEVSPACE_PORTABLE=ON in build-portable/: its `ctest`, the sync matrix over all
#             three protocols and the e2e suite against its binary (POSIX platform layer,
#             stat-scan watcher: the darwin client's code path, run on Linux)
#   pytest    the CPU suite (pytest -m "not gpu")
#   sanitize  TSan and ASan+UBSan over the C++ suite and the e2e suite (scripts/sanitize.sh)
# Usage: scripts/ci.sh [stage...]   (default: build portable pytest; `all` adds sanitize)
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
JOBS="${JOBS:-$(nproc)}"
stages=("$@")
[ ${#stages[@]} -eq 0 ] && stages=(build portable pytest)
[ "${stages[0]}" = all ] && stages=(build portable pytest sanitize)

E2E=(tests/test_e2e_cli.py tests/test_e2e_services.py tests/test_e2e_tls.py tests/test_e2e_noninteractive.py
     tests/test_e2e_recovery.py tests/test_e2e_portforward_wan.py tests/test_platform.py)

for s in "${stages[@]}"; do
  echo "== ci: $s"
  case "$s" in
    build)
      cmake -S . -B build -G Ninja > /dev/null
      ninja -C build -j "$JOBS"
      (cd build && ctest --output-on-failure)
      ;;
    portable)
      cmake -S . -B build-portable -G Ninja -DDEVSPACE_PORTABLE=ON -DDEVSPACE_PYTHON=OFF \
        "-DDEVSPACE_OUTPUT_DIR=$ROOT/build-portable/bin" > /dev/null
      ninja -C build-portable -j "$JOBS"
      (cd build-portable && ctest --output-on-failure)
      DEVSPACE_TESTS_BIN="$ROOT/build-portable/bin/devspace_tests" python3 -m pytest -q -x tests/test_sync_matrix_kube.py
      DEVSPACE_BIN="$ROOT/build-portable/bin/devspace" python3 -m pytest -q -x "${E2E[@]}"
      ;;
    pytest)
      python3 -m pytest -q -x -m "not gpu" tests/
      ;;
    sanitize)
      bash scripts/sanitize.sh
      ;;
    *)
      echo "ci: unknown stage $s" >&2
      exit 2
      ;;
  esac
done
echo "== ci: ok (${stages[*]})"
