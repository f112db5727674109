#!/bin/bash
# One GPU-box session: gpu tests, graft smoke, copy-kernel sweep, 1-GPU bench (verbose, with
# the runner's per-reload breakdown), rocprofv3 kernel stats of the probe kernels and of the
# hot-reload training workload. Every GPU step has its own time limit; the first failure ends
# the script (no retries).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== pytest -m gpu" && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 && tail -3 "$OUT/pytest_gpu.log" && \
echo "== smoke" && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" && \
echo "== gpucheck + copy sweep" && \
timeout -k 10 300 python -m devspace_amd.gpucheck > "$OUT/gpucheck.log" 2>&1 && cat "$OUT/gpucheck.log" && \
timeout -k 10 300 python -m devspace_amd.gpucheck --sweep-copy > "$OUT/copy_sweep.log" 2>&1 && head -5 "$OUT/copy_sweep.log" && \
echo "== bench N=1" && \
BENCH_VERBOSE=1 timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" && \
echo "== rocprofv3 probe + workload" && \
cd /tmp && export TMPDIR=/tmp && export PYTHONPATH="$ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o probe -- \
  python -m devspace_amd.gpucheck > "$OUT/prof_probe.log" 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o train -- \
  python -m devspace_amd.runner --max-steps 60 --log-every 20 "$ROOT/examples/rocm-pytorch/train.py" \
  > "$OUT/prof_train.log" 2>&1 && \
echo "== done"
