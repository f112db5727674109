#!/bin/bash
# Round-3 MI355X validation of HEAD: the GPU test tier, smoke(), and the driver's bench command.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3f_pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/r3f_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r3f_pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3f_smoke.txt 2>&1 || { tail -20 gpurun_out/r3f_smoke.txt; exit 1; }
tail -1 gpurun_out/r3f_smoke.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3f_bench.json 2> gpurun_out/r3f_bench.err || { tail -20 gpurun_out/r3f_bench.err; exit 1; }
tail -c 1200 gpurun_out/r3f_bench.json
