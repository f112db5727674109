# Hot-reloadable training loop for a rocm/pytorch dev pod (run by devspace_amd.runner).
#
# Edit anything below `step()` (or MARKER) while `devspace dev` is running: the file is synced
# into the pod and the runner swaps the code at the next step boundary without restarting the
# process — model/optimizer stay resident in HBM and the RCCL process group stays up.
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def _eager_add_rms_norm(x, delta, weight, eps=None):
    s = x + delta
    return s, F.rms_norm(s, (s.shape[-1],), weight, eps)


def _eager_attention(qkv, causal=True):
    q, k, v = qkv.unbind(2)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=causal)
    return o.transpose(1, 2)


def _eager_swiglu(h):
    g, u = h.chunk(2, dim=-1)
    return F.silu(g) * u


def _eager_cross_entropy(logits, target):
    return F.cross_entropy(logits.float(), target)


# gfx950 HIP kernels (attention, RMSNorm, SwiGLU, cross-entropy, AdamW) from devspace_amd.ops,
# which `devspace init` vendors into the project next to this file (built at image build, or
# compiled once on the first pod start). FUSED says which path runs; setup() prints it.
try:
    from devspace_amd.ops import fused as _fused

    FUSED = _fused.backend()
except ImportError as e:  # the kit is not in the image
    _fused, FUSED = None, f"eager (devspace_amd.ops not importable: {e})"
if FUSED == "hip" or (_fused is not None and not torch.cuda.is_available()):
    # (without a GPU the fused module runs its PyTorch formulation: CPU smoke runs and tests)
    AdamW, RMSNorm = _fused.AdamW, _fused.RMSNorm
    add_rms_norm, attention, cross_entropy, swiglu = _fused.add_rms_norm, _fused.attention, _fused.cross_entropy, _fused.swiglu
else:
    AdamW, RMSNorm = None, nn.RMSNorm
    add_rms_norm, attention, cross_entropy, swiglu = _eager_add_rms_norm, _eager_attention, _eager_cross_entropy, _eager_swiglu

MARKER = "v0"
SETUP_VERSION = 1  # bump to rebuild model/optimizer on the next reload

VOCAB = 8192
DIM = 1024
HEADS = 16
LAYERS = 4
SEQ = 512
BATCH = 8


class Block(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.heads = heads
        self.norm1 = RMSNorm(dim)
        self.qkv = nn.Linear(dim, 3 * dim, bias=False)
        self.proj = nn.Linear(dim, dim, bias=False)
        self.norm2 = RMSNorm(dim)
        self.up = nn.Linear(dim, 8 * dim // 3 * 2, bias=False)
        self.down = nn.Linear(8 * dim // 3, dim, bias=False)

    def forward(self, x, pending=None):
        # The residual stream is carried as (x, pending): each residual add is fused into the
        # RMSNorm that reads its result (x += pending; h = norm(x) in one kernel each way).
        b, t, d = x.shape
        if pending is None:
            h = self.norm1(x)
        else:
            x, h = add_rms_norm(x, pending, self.norm1.weight, self.norm1.eps)
        qkv = self.qkv(h).view(b, t, 3, self.heads, d // self.heads)
        a = attention(qkv, causal=True)  # [b, t, heads, head_dim]
        x, h = add_rms_norm(x, self.proj(a.reshape(b, t, d)), self.norm2.weight, self.norm2.eps)
        return x, self.down(swiglu(self.up(h)))


class TinyLM(nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(VOCAB, DIM)
        self.blocks = nn.ModuleList([Block(DIM, HEADS) for _ in range(LAYERS)])
        self.norm = RMSNorm(DIM)
        self.head = nn.Linear(DIM, VOCAB, bias=False)

    def forward(self, idx):
        x, pending = self.emb(idx), None
        for blk in self.blocks:
            x, pending = blk(x, pending)
        _, h = add_rms_norm(x, pending, self.norm.weight, self.norm.eps)
        return self.head(h)


def setup(ctx):
    ctx.log(f"fused={FUSED}")
    torch.manual_seed(1234 + ctx.rank)
    model = TinyLM().to(device=ctx.device, dtype=torch.bfloat16)
    if ctx.distributed:
        # One process per GPU, gradients all-reduced by RCCL over xGMI while backward runs.
        # 32 MB buckets: ~5 all-reduces for the 134 MB of bf16 gradients, so the first starts
        # once the head + last block are done and only the last ~32 MB (≈0.2 ms on an 8-GPU
        # ring) is exposed after backward; one 128 MB bucket would wait for nearly all of it.
        model = nn.parallel.DistributedDataParallel(model, bucket_cap_mb=32, gradient_as_bucket_view=True)
    if AdamW is not None:
        opt = AdamW(model.parameters(), lr=3e-4)  # multi-tensor HIP update
    else:
        opt = torch.optim.AdamW(model.parameters(), lr=3e-4, fused=ctx.device.type == "cuda")
    data = torch.randint(0, VOCAB, (BATCH, SEQ + 1), device=ctx.device)
    return {"model": model, "opt": opt, "data": data}


def step(ctx, state):
    model, opt, data = state["model"], state["opt"], state["data"]
    logits = model(data[:, :-1])
    loss = cross_entropy(logits.view(-1, VOCAB), data[:, 1:].reshape(-1))
    opt.zero_grad(set_to_none=True)
    # Preemption point between forward and backward: when the next edit is already waiting,
    # the runner drops the rest of this step (backward + update) instead of running it.
    ctx.preempt_point()
    loss.backward()
    opt.step()
    loss = loss.item()
    return {"loss": round(loss, 4), "ppl": round(math.exp(min(20.0, loss)), 2)}
