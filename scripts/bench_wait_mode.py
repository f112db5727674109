#!/usr/bin/env python3
"""A/B of the HIP host wait mode for the hot-reload workload's step loop.

Each training step of examples/rocm-pytorch ends in a host sync (`loss.item()`); the runner's
loop period (and so the edit->reload latency: in-flight wait + first step) includes the time the
host needs to notice the GPU finished. ROCclr spins for ROC_ACTIVE_WAIT_TIMEOUT us and then
sleeps on an interrupt; a 3.5 ms step always falls into the interrupt path. This script runs the
same step loop in fresh processes with different wait settings, interleaved, and reports the
median step period.

Usage: python scripts/bench_wait_mode.py [--steps 200] [--rounds 4] [--json out.json]
"""

import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import importlib.util, os, sys, time, json
sys.path.insert(0, os.environ["ROOT"])
import torch
spec = importlib.util.spec_from_file_location("train", os.path.join(os.environ["ROOT"], "examples/rocm-pytorch/train.py"))
m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
class Ctx: rank = 0; world_size = 1; distributed = False; device = torch.device("cuda", 0)
st = m.setup(Ctx)
for _ in range(20): m.step(Ctx, st)
torch.cuda.synchronize()
steps = int(os.environ["STEPS"]); dts = []
t = time.perf_counter()
for _ in range(steps):
    m.step(Ctx, st)
    n = time.perf_counter(); dts.append((n - t) * 1e3); t = n
dts.sort()
print(json.dumps({"p50": dts[len(dts) // 2], "p10": dts[len(dts) // 10], "p90": dts[9 * len(dts) // 10]}))
"""

VARIANTS = {
    "default": {},
    "active_wait_50ms": {"ROC_ACTIVE_WAIT_TIMEOUT": "50000"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--json")
    a = ap.parse_args()
    res = {k: [] for k in VARIANTS}
    for r in range(a.rounds):
        for name, extra in VARIANTS.items():
            env = dict(os.environ, ROOT=ROOT, STEPS=str(a.steps), **extra)
            p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
            if p.returncode != 0:
                print(p.stdout, p.stderr, file=sys.stderr)
                return 1
            d = json.loads(p.stdout.strip().splitlines()[-1])
            res[name].append(d)
            print(f"round {r} {name:18s} period p50 {d['p50']:.3f} ms  p10 {d['p10']:.3f}  p90 {d['p90']:.3f}", flush=True)
    summary = {k: round(statistics.median(x["p50"] for x in v), 4) for k, v in res.items()}
    print("median step period (ms):", json.dumps(summary))
    if a.json:
        json.dump({"summary": summary, "rounds": res}, open(a.json, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
