#!/bin/bash
# Round-3 MI355X evidence: the GPU test tier, the driver's bench command, and a rocprofv3 kernel
# trace taken INSIDE the GPU pod of the e2e test (the pod runs the vendored workload kit, no
# checkout on its Python path: the trace must show the fused gfx950 kernels, attn_fwd_kernel
# included).
set -o pipefail
R=$PWD
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_pytest_gpu.txt 2>&1 && echo PYTEST_OK && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err && echo BENCH_OK && cat gpurun_out/r3_bench.json && \
rm -rf gpurun_out/prof_pod && \
DEVSPACE_E2E_POD_PROFILE=$R/gpurun_out/prof_pod timeout -k 10 400 python -u -m pytest tests/test_gpu_e2e.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_prof_pod.log 2>&1 && echo PROF_OK && \
for db in $(find gpurun_out/prof_pod -name '*.db'); do python3 scripts/rocpd_summary.py $db --top 40; done > gpurun_out/r3_pod_kernels.txt 2>&1; echo SUMMARY_DONE
