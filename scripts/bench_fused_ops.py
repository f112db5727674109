#!/usr/bin/env python3
"""A/B of the gfx950 fused ops against the eager PyTorch op chains they replace, in one
process with interleaved rounds (cdna_hip_programming.md §5.4 rule 24), on the shapes of the
rocm-pytorch example (B*T = 4096 rows, D = 1024, H = 2730, V = 8192), plus the whole
TinyLM training step built either way.

Two clocks per case:
  * launched: the calls issued from Python one after another (what an eager training loop
    sees; at these sizes the host's dispatch, autograd included, can be the bound);
  * graph: the same calls captured once into a HIP graph and replayed, so the number is the
    device's time for the kernels alone (cases that cannot be captured print n/a).

    python scripts/bench_fused_ops.py [--rounds 10] [--json out.json]
"""

import argparse
import importlib.util
import json
import os
import statistics
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from devspace_amd.ops import fused  # noqa: E402


def timeit(fn, iters):
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    start.record()
    for _ in range(iters):
        fn()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) * 1000.0 / iters  # us


def timeit_graph(fn, iters):
    """Device time of `iters` calls replayed from one captured HIP graph (us per call); None
    when the case cannot be captured (a host sync or a host-side value inside it)."""
    try:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up off the capture stream, as capture requires
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        g.replay()
        end.record()
        torch.cuda.synchronize()
        return start.elapsed_time(end) * 1000.0 / iters
    except Exception:  # noqa: BLE001 - not capturable: reported as n/a
        torch.cuda.synchronize()
        return None


def op_cases(dev):
    R, D, H, V = 4096, 1024, 2730, 8192
    x = torch.randn(R, D, device=dev).bfloat16().requires_grad_()
    w = torch.ones(D, device=dev).bfloat16().requires_grad_()
    dy = torch.randn(R, D, device=dev).bfloat16()
    h = torch.randn(R, 2 * H, device=dev).bfloat16().requires_grad_()
    dyh = torch.randn(R, H, device=dev).bfloat16()
    logits = torch.randn(R, V, device=dev).bfloat16().requires_grad_()
    t = torch.randint(0, V, (R,), device=dev)
    eps = torch.finfo(torch.bfloat16).eps

    def rms_fused():
        fused.rms_norm(x, w, eps, kernel=True).backward(dy)

    def rms_eager():
        F.rms_norm(x, (D,), w, eps).backward(dy)

    def swiglu_fused():
        fused.swiglu(h).backward(dyh)

    def swiglu_eager():
        g, u = h.chunk(2, -1)
        (F.silu(g) * u).backward(dyh)

    def ce_fused():
        fused.cross_entropy(logits, t).backward()

    def ce_eager():
        F.cross_entropy(logits.float(), t).backward()

    # optimizer: TinyLM-sized parameter set (67M bf16), grads fixed
    shapes = [(8192, 1024), (8192, 1024)] + [(3072, 1024), (1024, 1024), (5460, 1024), (1024, 2730), (1024,),
                                             (1024,)] * 4
    params = [torch.randn(s, device=dev).bfloat16().requires_grad_() for s in shapes]
    for q in params:
        q.grad = torch.randn_like(q) * 1e-3
    params_b = [q.detach().clone().requires_grad_() for q in params]
    for q, r in zip(params, params_b):
        r.grad = q.grad.clone()
    opt_f = fused.AdamW(params, lr=1e-4)
    opt_e = torch.optim.AdamW(params_b, lr=1e-4, fused=True)

    qkv = torch.randn(8, 512, 3, 16, 64, device=dev).bfloat16().requires_grad_()
    dattn = torch.randn(8, 512, 16, 64, device=dev).bfloat16()

    def attn_fused():
        fused.attention(qkv, causal=True).backward(dattn)

    def attn_eager():
        q, k, v = qkv.unbind(2)
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=True)
        o.transpose(1, 2).reshape(8, 512, 1024).backward(dattn.view(8, 512, 1024))

    xd = torch.randn(R, D, device=dev).bfloat16().requires_grad_()

    def addnorm_fused():
        s_, y_ = fused.add_rms_norm(x, xd, w, eps)
        torch.autograd.backward([s_, y_], [dy, dy])

    def addnorm_eager():
        s_ = x + xd
        y_ = F.rms_norm(s_, (D,), w, eps)
        torch.autograd.backward([s_, y_], [dy, dy])

    return {"attention fwd+bwd [8x512, 16 heads x 64]": (attn_fused, attn_eager),
            "residual add + rmsnorm fwd+bwd [4096x1024]": (addnorm_fused, addnorm_eager),
            "adamw step [67M bf16 params]": (opt_f.step, opt_e.step),
            "rmsnorm fwd+bwd [4096x1024]": (rms_fused, rms_eager),
            "swiglu fwd+bwd [4096x2x2730]": (swiglu_fused, swiglu_eager),
            "cross_entropy fwd+bwd [4096x8192]": (ce_fused, ce_eager)}


def load_train():
    spec = importlib.util.spec_from_file_location("tinylm_ab", os.path.join(ROOT, "examples", "rocm-pytorch", "train.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def step_case(dev):
    from devspace_amd.runner import Context  # what the runner hands train.py

    def Ctx():
        return Context(0, 1, 0, dev)

    m_fused = load_train()
    m_eager = load_train()
    m_eager.RMSNorm = nn.RMSNorm

    def sw(hh):
        g, u = hh.chunk(2, dim=-1)
        return F.silu(g) * u

    m_eager.swiglu = sw

    def add_norm(x, d, w, eps=None):
        s = x + d
        return s, F.rms_norm(s, (s.shape[-1],), w, eps)

    m_eager.add_rms_norm = add_norm
    m_eager.AdamW = None  # torch.optim.AdamW(fused=True)
    m_eager.cross_entropy = lambda lg, tg: F.cross_entropy(lg.float(), tg)
    sf, se = m_fused.setup(Ctx()), m_eager.setup(Ctx())
    return ("TinyLM train step (4x1024, B8xT512)", (lambda: m_fused.step(Ctx(), sf), lambda: m_eager.step(Ctx(), se)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    fused.ext()
    cases = op_cases(dev)
    name, fns = step_case(dev)
    cases[name] = fns
    res = {k: {"fused": [], "eager": []} for k in cases}
    for _ in range(a.rounds):
        for k, (f, e) in cases.items():
            iters = 5 if k.startswith("TinyLM") else a.iters
            res[k]["fused"].append(timeit(f, iters))
            res[k]["eager"].append(timeit(e, iters))
    graph = {}
    for k, (f, e) in cases.items():
        if k.startswith("TinyLM") or k.startswith("adamw"):
            continue  # host-side step counters and syncs: not captured
        gf, ge = [], []
        for _ in range(max(1, a.rounds // 2)):
            gf.append(timeit_graph(f, a.iters))
            ge.append(timeit_graph(e, a.iters))
        if None not in gf and None not in ge:
            graph[k] = (statistics.median(gf), statistics.median(ge))
    out = {}
    print(f"{'case':42s} {'fused_us':>10} {'eager_us':>10} {'speedup':>8}   {'graph: fused_us':>15} {'eager_us':>9} "
          f"{'speedup':>8}   (medians, interleaved rounds)")
    for k, v in res.items():
        fm, em = statistics.median(v["fused"]), statistics.median(v["eager"])
        out[k] = {"fused_us": round(fm, 1), "eager_us": round(em, 1), "speedup": round(em / fm, 3),
                  "fused_min_us": round(min(v["fused"]), 1), "eager_min_us": round(min(v["eager"]), 1)}
        line = f"{k:42s} {fm:>10.1f} {em:>10.1f} {em / fm:>8.2f}x"
        if k in graph:
            gfm, gem = graph[k]
            out[k].update({"graph_fused_us": round(gfm, 1), "graph_eager_us": round(gem, 1),
                           "graph_speedup": round(gem / gfm, 3)})
            line += f"   {gfm:>15.1f} {gem:>9.1f} {gem / gfm:>8.2f}x"
        else:
            line += f"   {'n/a':>15}"
        print(line)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0), "results": out}, f, indent=1)


if __name__ == "__main__":
    main()
