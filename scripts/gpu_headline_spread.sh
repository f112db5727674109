#!/bin/bash
# Run-to-run spread of the bench headline on one MI355X box: five headline-only runs
# (quickstart loop, 30 timed steps each), one JSON summary line per run.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/headline_spread.txt
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --ref-steps 0 --gpu-steps 0 --example-steps 0 \
    --no-deploy-bench > gpurun_out/hs_run.json 2> gpurun_out/hs_run.err || { tail -20 gpurun_out/hs_run.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/hs_run.json').read().strip().splitlines()[-1]); print('run $i: p50', d['p50_ms'], 'p90', d['p90_ms'], 'sync', d['sync_p50_ms'], 'dev_start_s', d['dev_start_s'])" >> gpurun_out/headline_spread.txt
  tail -1 gpurun_out/headline_spread.txt
done
