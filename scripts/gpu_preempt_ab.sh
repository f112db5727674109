#!/bin/bash
# A/B of runner preemption points on the 1-GPU hot-reload bench (same box, back to back).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== runner gpu test" && \
timeout -k 10 300 python -u -m pytest tests/test_runner.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_runner.log" 2>&1 && tail -3 "$OUT/pytest_runner.log" && \
echo "== bench preempt on" && \
timeout -k 10 400 python -u bench.py --steps 40 --warmup 3 --ref-steps 0 --no-deploy-bench > "$OUT/bench_preempt_on.json" 2> "$OUT/bench_preempt_on.err" && cat "$OUT/bench_preempt_on.json" && \
echo "== bench preempt off" && \
DEVSPACE_PREEMPT=0 timeout -k 10 400 python -u bench.py --steps 40 --warmup 3 --ref-steps 0 --no-deploy-bench > "$OUT/bench_preempt_off.json" 2> "$OUT/bench_preempt_off.err" && cat "$OUT/bench_preempt_off.json" && \
echo "== bench preempt on (again)" && \
timeout -k 10 400 python -u bench.py --steps 40 --warmup 3 --ref-steps 0 --no-deploy-bench > "$OUT/bench_preempt_on2.json" 2> "$OUT/bench_preempt_on2.err" && cat "$OUT/bench_preempt_on2.json" && \
echo "== done"
