#!/bin/bash
# Fused-ops session: numerics tests on the GPU, interleaved A/B microbench, rocprofv3 kernel
# stats of the hot-reload workload, then the 1-GPU bench. First failure ends the script.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== pytest fused (gpu)" && \
timeout -k 10 300 python -u -m pytest tests/test_fused_ops.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_fused.log" 2>&1 && tail -3 "$OUT/pytest_fused.log" && \
echo "== A/B fused vs eager" && \
timeout -k 10 300 python -u scripts/bench_fused_ops.py --json "$OUT/fused_ab.json" > "$OUT/fused_ab.txt" 2>&1 && cat "$OUT/fused_ab.txt" && \
echo "== rocprofv3 workload" && \
(cd /tmp && export TMPDIR=/tmp PYTHONPATH="$ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o train -- \
  python -m devspace_amd.runner --max-steps 60 --log-every 20 "$ROOT/examples/rocm-pytorch/train.py" > "$OUT/prof_train.log" 2>&1) && \
python scripts/prof_summary.py "$(ls "$OUT"/prof/*/train_results.db "$OUT"/prof/train_results.db 2>/dev/null | head -1)" 30 > "$OUT/train_kernels.txt" && head -40 "$OUT/train_kernels.txt" && \
echo "== bench" && \
timeout -k 10 500 python -u bench.py --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" && \
echo "== done"
