"""Single-rank RCCL check (world_size=1: one GPU box, one rank): torch.distributed backend "nccl"
(RCCL on ROCm) as the rocm-pytorch pod uses it: a communicator
per process, collectives on HIP streams, and the example's DDP training step (32 MB gradient
buckets all-reduced during backward). One GPU box -> one rank; the multi-rank path of the same
code runs on CPU/gloo in test_runner.py and on 8 GPUs in the driver's scaling bench."""

import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

SCRIPT = r"""
import os, sys, time
sys.path.insert(0, os.environ["ROOT"])
import torch
import torch.distributed as dist
from devspace_amd import runner

assert torch.cuda.is_available()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1)
assert dist.get_backend() == "nccl"
# collectives the runner and DDP use, on a 64 MiB bf16 buffer
x = torch.full((32 << 20,), 2.0, dtype=torch.bfloat16, device=dev)
dist.all_reduce(x, op=dist.ReduceOp.SUM)
dist.broadcast(x, src=0)
out = torch.empty_like(x)
dist.all_gather_into_tensor(out, x)
rs = torch.empty_like(x)
dist.reduce_scatter_tensor(rs, x)
ctl = torch.tensor([7], dtype=torch.int64, device=dev)
dist.all_reduce(ctl, op=dist.ReduceOp.MAX)
torch.cuda.synchronize()
assert float(out[0]) == 2.0 and float(rs[-1]) == 2.0 and int(ctl.item()) == 7
# timed all-reduce (single rank: the communicator's local path, no xGMI traffic)
t0 = time.perf_counter()
for _ in range(10):
    dist.all_reduce(x)
torch.cuda.synchronize()
ar_ms = (time.perf_counter() - t0) * 100.0
# the example's DDP step through the runner's context
mod = runner.load_module(os.path.join(os.environ["ROOT"], "examples", "rocm-pytorch", "train.py"), 1)
for k, v in (("LAYERS", 2), ("SEQ", 256), ("BATCH", 2)):
    setattr(mod, k, v)
ctx = runner.Context(0, 1, 0, dev)
ctx.distributed = True
state = mod.setup(ctx)
assert isinstance(state["model"], torch.nn.parallel.DistributedDataParallel)
losses = [mod.step(ctx, state)["loss"] for _ in range(3)]
torch.cuda.synchronize()
assert all(l == l and l > 0 for l in losses), losses
dist.destroy_process_group()
print(f"RCCL OK allreduce_64MiB_ms={ar_ms:.3f} ddp_losses={[round(l, 4) for l in losses]}")
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_rccl_collectives_and_ddp_step_on_gpu():
    env = dict(os.environ, ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-c", SCRIPT], capture_output=True, text=True, env=env, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "RCCL OK" in p.stdout, p.stdout
    print(p.stdout.strip().splitlines()[-1])
