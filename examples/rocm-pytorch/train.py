# Hot-reloadable training loop for a rocm/pytorch dev pod (run by devspace_amd.runner).
#
# Edit anything below `step()` (or MARKER) while `devspace dev` is running: the file is synced
# into the pod and the runner swaps the code at the next step boundary without restarting the
# process — model/optimizer stay resident in HBM and the RCCL process group stays up.
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

try:  # gfx950 HIP kernels shipped with devspace_amd (attention, RMSNorm, SwiGLU, CE, AdamW)
    from devspace_amd.ops.fused import AdamW, RMSNorm, attention, cross_entropy, swiglu
except ImportError:  # plain PyTorch when the package is not in the image
    RMSNorm = nn.RMSNorm
    AdamW = None

    def attention(qkv, causal=True):
        q, k, v = qkv.unbind(2)
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=causal)
        return o.transpose(1, 2)

    def swiglu(h):
        g, u = h.chunk(2, dim=-1)
        return F.silu(g) * u

    def cross_entropy(logits, target):
        return F.cross_entropy(logits.float(), target)

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

    def forward(self, x):
        b, t, d = x.shape
        qkv = self.qkv(self.norm1(x)).view(b, t, 3, self.heads, d // self.heads)
        a = attention(qkv, causal=True)  # [b, t, heads, head_dim]
        x = x + self.proj(a.reshape(b, t, d))
        return x + self.down(swiglu(self.up(self.norm2(x))))


class TinyLM(nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(VOCAB, DIM)
        self.blocks = nn.ModuleList([Block(DIM, HEADS) for _ in range(LAYERS)])
        self.norm = RMSNorm(DIM)
        self.head = nn.Linear(DIM, VOCAB, bias=False)

    def forward(self, idx):
        x = self.emb(idx)
        for blk in self.blocks:
            x = blk(x)
        return self.head(self.norm(x))


def setup(ctx):
    torch.manual_seed(1234 + ctx.rank)
    model = TinyLM().to(device=ctx.device, dtype=torch.bfloat16)
    if ctx.distributed:
        # one process per GPU; big buckets -> few large RCCL all-reduces over xGMI
        model = nn.parallel.DistributedDataParallel(model, bucket_cap_mb=128, gradient_as_bucket_view=True)
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
    loss.backward()
    opt.step()
    return {"loss": round(loss.item(), 4), "ppl": round(math.exp(min(20.0, loss.item())), 2)}
