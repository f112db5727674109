#!/bin/bash
# GPU probe tests (incl. the xGMI peer check) and a rocprofv3 kernel trace taken inside the GPU
# pod of the e2e test (the pod runs the vendored kit; the trace shows the fused gfx950 kernels).
set -o pipefail
R=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpucheck.py tests/test_gpu_probe_fallback.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3p_probe.txt 2>&1 || { tail -30 gpurun_out/r3p_probe.txt; exit 1; }
tail -2 gpurun_out/r3p_probe.txt
timeout -k 10 120 python -m devspace_amd.gpucheck --quick >> gpurun_out/r3p_probe.txt 2>&1; tail -3 gpurun_out/r3p_probe.txt
rm -rf gpurun_out/prof_pod
DEVSPACE_E2E_POD_PROFILE=$R/gpurun_out/prof_pod timeout -k 10 400 python -u -m pytest tests/test_gpu_e2e.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3p_prof_pod.log 2>&1 || { tail -30 gpurun_out/r3p_prof_pod.log; exit 1; }
for db in $(find gpurun_out/prof_pod -name '*.db'); do python3 scripts/rocpd_summary.py $db --top 40; done > gpurun_out/r3p_pod_kernels.txt 2>&1
head -25 gpurun_out/r3p_pod_kernels.txt
