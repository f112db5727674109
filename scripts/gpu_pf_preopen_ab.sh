#!/bin/bash
# A/B of the port-forward hold's pre-opened next attempt (DEVSPACE_PORTFORWARD_PREOPEN) on the
# bench headline loop (quickstart only), alternating the arms.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/pf_preopen_ab.txt
: > $out
for rep in 1 2 3; do
  for arm in 1 0; do
    DEVSPACE_PORTFORWARD_PREOPEN=$arm timeout -k 10 240 python bench.py --steps 40 --warmup 3 --ref-steps 0 \
      --gpu-steps 0 --example-steps 0 --no-deploy-bench > gpurun_out/pf_ab_run.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/pf_ab_run.json').read().strip().splitlines()[-1]); print('preopen=$arm p50', d['p50_ms'], 'p90', d['p90_ms'])" >> $out || exit 1
  done
done
cat $out
