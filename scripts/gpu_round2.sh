#!/bin/bash
# Round-2 MI355X evidence: GPU test tier, the driver's bench command, and a rocprofv3 kernel
# profile of smoke() (ROCm 7 writes a rocpd database; scripts/rocpd_summary.py summarises it).
set -o pipefail
R=$PWD
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_pytest_gpu.txt 2>&1 && echo PYTEST_OK && \
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err && echo BENCH_OK && cat gpurun_out/r2_bench.json && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_smoke -o smoke -- python3 $R/__graft_entry__.py smoke > $R/gpurun_out/r2_prof_smoke.log 2>&1 && echo PROF_OK
