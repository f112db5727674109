#!/usr/bin/env python3
"""Attention fwd+bwd at the rocm-pytorch shape (B8 x T512, 16 heads x 64) in a loop, for
rocprofv3 kernel traces / PMC passes of the attention kernels alone."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from devspace_amd.ops import fused  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    qkv = torch.randn(8, 512, 3, 16, 64, device="cuda").bfloat16().requires_grad_()
    do = torch.randn(8, 512, 16, 64, device="cuda").bfloat16()
    for _ in range(iters):
        fused.attention(qkv, causal=True).backward(do)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
