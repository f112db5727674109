#!/bin/bash
# A/B of the GPU inner loop over plain ws vs TLS wss on one box (same code, back to back).
set -o pipefail
mkdir -p gpurun_out
for t in plain tls plain tls; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --qs-steps 0 --ref-steps 0 --no-deploy-bench \
    --transport $t >> gpurun_out/r2_transport_ab.jsonl 2>> gpurun_out/r2_transport_ab.err || exit 1
  echo "done $t"
done
