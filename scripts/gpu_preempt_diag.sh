#!/bin/bash
# Per-reload lines of the 1-GPU bench (BENCH_VERBOSE) for preempt/watch-mode variants.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 BENCH_VERBOSE=1
for v in "on 1 1" "preempt_off 0 1" "on_b 1 1" "preempt_off_b 0 1"; do
  set -- $v
  echo "== $1"
  DEVSPACE_PREEMPT=$2 DEVSPACE_WATCH_SETTLED=$3 timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --ref-steps 0 --no-deploy-bench > "$OUT/diag_$1.json" 2> "$OUT/diag_$1.err" || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['p50_ms'], d['p90_ms'], d['ms_per_step'], d['breakdown_p50'])" "$OUT/diag_$1.json"
done
echo "== done"
