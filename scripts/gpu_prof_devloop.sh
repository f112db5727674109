#!/bin/bash
# rocprofv3 kernel trace of the whole inner loop on one MI355X: bench.py drives `devspace dev` of
# the rocm-pytorch pod; the profiler follows the pod's runner process (environment inherited
# through the local kubelet), so the stats are the training steps run during hot reloads.
set -o pipefail
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_devloop -o devloop -- \
  python3 $R/bench.py --steps 10 --warmup 2 --qs-steps 0 --ref-steps 0 --no-deploy-bench \
  > $R/gpurun_out/r2_prof_devloop.json 2> $R/gpurun_out/r2_prof_devloop.err && echo PROF_OK
ls -R $R/gpurun_out/prof_devloop | head -20
