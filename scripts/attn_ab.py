#!/usr/bin/env python3
"""Times attention fwd+bwd (rocm-pytorch shape: B8 x T512, 16 heads x 64, causal) from the
devspace_amd package under ROOT (argv[1]), so two builds of fused_ops.hip can be compared in one
GPU session: python scripts/attn_ab.py <root> [iters]."""
import sys
import time

root = sys.argv[1]
sys.path.insert(0, root)
import torch  # noqa: E402

from devspace_amd.ops import fused  # noqa: E402


def main():
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(8, 512, 3, 16, 64, device="cuda", generator=g).bfloat16().requires_grad_()
    do = torch.randn(8, 512, 16, 64, device="cuda", generator=g).bfloat16()
    for _ in range(20):
        fused.attention(qkv, causal=True).backward(do)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record()
    for _ in range(iters):
        o = fused.attention(qkv, causal=True)
    ev[1].record()
    for _ in range(iters):
        fused.attention(qkv, causal=True).backward(do)
    ev[2].record()
    torch.cuda.synchronize()
    fwd = ev[0].elapsed_time(ev[1]) / iters * 1000
    both = ev[1].elapsed_time(ev[2]) / iters * 1000
    qkv.grad = None
    fused.attention(qkv, causal=True).backward(do)
    chk = float(qkv.grad.float().abs().sum()) + float(o.float().abs().sum())
    print(f"{fused.ext().__file__}: fwd {fwd:.1f} us, fwd+bwd {both:.1f} us, checksum {chk:.6e}", flush=True)


if __name__ == "__main__":
    main()
