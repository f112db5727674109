#!/bin/bash
# Rehearsal of the driver's N>1 bench invocation on a 1-GPU box: two bench ranks under
# torch.distributed.run, the pod runs two training ranks on the one GPU. RCCL refuses two ranks
# on one device, so the pod's process group uses gloo (DEVSPACE_DIST_BACKEND); RCCL itself is
# covered by tests/test_rccl.py. Everything else is the 8-GPU path: gloo timing barriers between
# bench ranks, MAX over ranks, the pod's N-rank generation agreement, JSON on rank 0 only.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DEVSPACE_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/rehearse_n2.json 2> gpurun_out/rehearse_n2.err
rc=$?
echo "rc=$rc"
cat gpurun_out/rehearse_n2.json
tail -20 gpurun_out/rehearse_n2.err
exit $rc
