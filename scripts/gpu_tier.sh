#!/usr/bin/env bash
# The GPU tier on one MI355X (the driver's round-end checks, and the profiles committed under
# profiles/), run on a gpurun box from the repo root:
#
#   gpurun --timeout 1200 -- bash scripts/gpu_tier.sh [tests] [smoke] [bench] [prof] [rescue]
#
#   tests   python -m pytest tests -m gpu (every HIP op against fp32 PyTorch, the runner on the GPU)
#   smoke   __graft_entry__.smoke(): one forward+backward of the flagship TinyLM on cuda:0
#   bench   bench.py --steps $BENCH_STEPS --warmup $BENCH_WARMUP (the headline JSON line)
#   prof    rocprofv3 --kernel-trace --stats of the hot-reload runner training the rocm-pytorch example
#   rescue  the runner's snapshot cost on the flagship example (scripts/rescue_cost.py)
#   kernels the gfx950 fused ops against the eager op chains they replace (scripts/bench_fused_ops.py)
#   layers  the rocm-pytorch image built with RUN executed, then rebuilt after an edit (scripts/image_rebuild_cost.py)
#   via     port-forward on a remote cluster: retries from the laptop vs the hold in the pod (scripts/ab_portforward_via.py)
#   digest  the rescue snapshots' content digest: gfx950 state_digest kernel vs torch ops (scripts/digest_cost.py)
#
# Output: gpurun_out/$GPU_TIER_TAG/ (default "tier"). Every GPU step has its own time limit and
# the script stops at the first failing step: no GPU step runs after a fault or a timeout.
set -o pipefail
cd "$(dirname "$0")/.."
OUT="$PWD/gpurun_out/${GPU_TIER_TAG:-tier}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(tests smoke bench)

fail() {
  echo "step $1 failed (exit $2); log tail:"
  tail -40 "$3"
  exit 1
}

for s in "${steps[@]}"; do
  case "$s" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || fail tests $? "$OUT/pytest_gpu.log"
      tail -2 "$OUT/pytest_gpu.log"
      ;;
    smoke)
      timeout -k 10 300 python -u __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || fail smoke $? "$OUT/smoke.log"
      tail -2 "$OUT/smoke.log"
      ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps "${BENCH_STEPS:-20}" --warmup "${BENCH_WARMUP:-3}" \
        > "$OUT/bench.json" 2> "$OUT/bench.err" || fail bench $? "$OUT/bench.err"
      tail -1 "$OUT/bench.json"
      ;;
    prof)
      # the hot-reload runner on the flagship example for a bounded number of steps: a clean exit
      # lets every profiled process write its trace. (rocprofv3's SIGTERM handler waits for the
      # process's children before it chains to the program's handler, so a supervisor stopped
      # with SIGTERM never forwards it to its ranks, which run in sessions of their own: a
      # profile of a pod stopped that way, as `devspace dev` under the bench ends it, is empty.)
      R=$PWD
      (cd /tmp && export TMPDIR=/tmp PYTHONPATH="$R" && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        -d "$OUT/prof" -o runner -- python3 -m devspace_amd.runner --max-steps "${PROF_STEPS:-40}" --no-warm-standby \
        "$R/examples/rocm-pytorch/train.py" > "$OUT/prof_runner.log" 2>&1) || fail prof $? "$OUT/prof_runner.log"
      db=$(find "$OUT/prof" -name '*.db' | head -1)
      [ -n "$db" ] && python3 scripts/prof_summary.py "$db" > "$OUT/prof_kernels.txt" && head -12 "$OUT/prof_kernels.txt"
      ;;
    kernels)
      timeout -k 10 600 python -u scripts/bench_fused_ops.py --json "$OUT/kernels.json" > "$OUT/kernels.txt" \
        2> "$OUT/kernels.err" || fail kernels $? "$OUT/kernels.err"
      cat "$OUT/kernels.txt"
      ;;
    rescue)
      timeout -k 10 600 python -u scripts/rescue_cost.py > "$OUT/rescue.json" 2> "$OUT/rescue.err" \
        || fail rescue $? "$OUT/rescue.err"
      tail -1 "$OUT/rescue.json"
      ;;
    via)
      timeout -k 10 600 python -u scripts/ab_portforward_via.py > "$OUT/via.json" 2> "$OUT/via.err" \
        || fail via $? "$OUT/via.err"
      tail -1 "$OUT/via.json"
      ;;
    digest)
      timeout -k 10 300 python -u scripts/digest_cost.py > "$OUT/digest.json" 2> "$OUT/digest.err" \
        || fail digest $? "$OUT/digest.err"
      tail -1 "$OUT/digest.json"
      ;;
    layers)
      timeout -k 10 900 python -u scripts/image_rebuild_cost.py > "$OUT/layers.json" 2> "$OUT/layers.err" \
        || fail layers $? "$OUT/layers.err"
      tail -1 "$OUT/layers.json"
      ;;
    *)
      echo "unknown step $s" >&2
      exit 2
      ;;
  esac
done
