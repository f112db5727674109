#!/bin/bash
# A/B of the runner's change feed on MI355X: post-then-compile (default) vs compile-then-post
# (DEVSPACE_FEED_COMPILE_FIRST=1), alternating runs on one box, 60 timed reloads each.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
: > gpurun_out/feed_ab.jsonl
for round in 1 2; do
  for v in 1 0; do
    echo "round $round compile_first=$v"
    DEVSPACE_FEED_COMPILE_FIRST=$v timeout -k 10 300 python bench.py --steps 60 --warmup 5 --qs-steps 0 --ref-steps 0 \
      --no-deploy-bench > gpurun_out/feed_ab_${round}_${v}.json 2> gpurun_out/feed_ab_${round}_$v.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/feed_ab_${round}_${v}.json')); print(json.dumps({'compile_first': $v, 'round': $round, 'p50': d['p50_ms'], 'p90': d['p90_ms'], 'parts': d.get('breakdown_p50')}))" | tee -a gpurun_out/feed_ab.jsonl
  done
done
