#!/bin/bash
# Round-3 MI355X check: GPU test tier and the driver's bench command on the current tree.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_pytest_gpu.txt 2>&1 && echo PYTEST_OK && \
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err && echo BENCH_OK && cat gpurun_out/r3_bench.json
