#!/bin/bash
# Two pod ranks on one GPU through the gloo process group (see gpu_rehearse_multi.sh): the
# runner alone, output unbuffered, so a stall shows where it is.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DEVSPACE_DIST_BACKEND=gloo PYTHONUNBUFFERED=1 TORCH_DISTRIBUTED_DEBUG=DETAIL
timeout -k 10 150 python -u -m devspace_amd.runner --nproc 2 --max-steps 30 --log-every 5 examples/rocm-pytorch/train.py 2>&1 | tee gpurun_out/runner_n2.log
