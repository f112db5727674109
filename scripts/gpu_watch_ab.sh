#!/bin/bash
# A/B of the quickstart watcher's standby hand-off on one MI355X box: IPC message (the previous
# watch.js, saved as scripts/.watch_ipc_ab.js) against the signal + pipe hand-off, alternating
# headline-only bench runs, then one instrumented breakdown of each. Save the IPC version first:
#   git show 39e469f:examples/quickstart/watch.js > scripts/.watch_ipc_ab.js
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/watch_ab.txt
: > $OUT
cp examples/quickstart/watch.js gpurun_out/.watch_sig.js
use() { if [ "$1" = ipc ]; then cp scripts/.watch_ipc_ab.js examples/quickstart/watch.js; else cp gpurun_out/.watch_sig.js examples/quickstart/watch.js; fi; }
for i in 1 2 3; do
  for v in ipc sig; do
    use $v
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --ref-steps 0 --gpu-steps 0 --example-steps 0 \
      --no-deploy-bench > gpurun_out/ab_run.json 2> gpurun_out/ab_run.err || { tail -20 gpurun_out/ab_run.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_run.json').read().strip().splitlines()[-1]); print('$v run $i: p50', d['p50_ms'], 'p90', d['p90_ms'], 'sync', d['sync_p50_ms'])" >> $OUT
    tail -1 $OUT
  done
done
for v in ipc sig; do
  use $v
  echo "== breakdown $v" >> $OUT
  TMPDIR=/tmp timeout -k 10 200 python -u scripts/qs_breakdown.py --steps 30 --warmup 4 >> $OUT 2> gpurun_out/ab_bd.err || { tail -20 gpurun_out/ab_bd.err; exit 1; }
  tail -4 $OUT
done
use sig
