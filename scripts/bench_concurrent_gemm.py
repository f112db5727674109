#!/usr/bin/env python3
"""Do the TinyLM backward GEMMs fill an MI355X? For every linear layer of the rocm-pytorch
example (tokens = 4096), time dX = dY @ W and dW = dY^T @ X back-to-back on one stream vs.
concurrently on two streams (dW on a side stream, separate HW queue). If the pair runs
faster concurrently, the GEMMs leave CUs idle and the backward can overlap them."""
import statistics

import torch


def main():
    dev = torch.device("cuda")
    T = 4096
    shapes = {"qkv": (1024, 3072), "proj": (1024, 1024), "up": (1024, 5460), "down": (2730, 1024),
              "head": (1024, 8192)}
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()
    print(f"{'layer':6s} {'dX_us':>8} {'dW_us':>8} {'serial_us':>10} {'concurrent_us':>14} {'gain':>6}")
    tot_s = tot_c = 0.0
    for name, (k, n) in shapes.items():
        x = torch.randn(T, k, device=dev).bfloat16()
        w = torch.randn(n, k, device=dev).bfloat16()
        dy = torch.randn(T, n, device=dev).bfloat16()

        def dx():
            return dy @ w

        def dw():
            return dy.t() @ x

        def timed(fn, iters=50):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fn()
            torch.cuda.synchronize()
            s.record()
            for _ in range(iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            return s.elapsed_time(e) * 1000.0 / iters

        def serial():
            dx()
            dw()

        def concurrent():
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                dw()
            dx()
            main_s.wait_stream(side)

        r = {"dx": [], "dw": [], "ser": [], "con": []}
        for _ in range(7):
            r["dx"].append(timed(dx))
            r["dw"].append(timed(dw))
            r["ser"].append(timed(serial))
            r["con"].append(timed(concurrent))
        m = {k: statistics.median(v) for k, v in r.items()}
        tot_s += m["ser"]
        tot_c += m["con"]
        print(f"{name:6s} {m['dx']:8.1f} {m['dw']:8.1f} {m['ser']:10.1f} {m['con']:14.1f} {m['ser'] / m['con']:6.2f}x")
    print(f"{'total':6s} {'':8s} {'':8s} {tot_s:10.1f} {tot_c:14.1f} {tot_s / tot_c:6.2f}x")


if __name__ == "__main__":
    main()
