#!/bin/bash
# Runner GPU tests (hot reload, preemption drain) + the 1-GPU bench with the default runner.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== runner tests (gpu)" && \
timeout -k 10 300 python -u -m pytest tests/test_runner.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_runner.log" 2>&1 && tail -4 "$OUT/pytest_runner.log" && \
echo "== bench" && \
timeout -k 10 500 python -u bench.py --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" && \
echo "== done"
