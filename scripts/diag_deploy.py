#!/usr/bin/env python3
"""Where does the quickstart deploy wall-clock go? Runs the deploy benchmark with the local
cluster's object-event trace (LOCALKUBE_TRACE) and prints the cluster-side timeline relative
to the start of `devspace deploy`; `--cuda-first` initialises HIP in this process first (as
bench.py does on a GPU box)."""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cuda-first", action="store_true")
    ap.add_argument("--runs", type=int, default=2)
    a = ap.parse_args()
    if a.cuda_first:
        import torch

        torch.cuda.set_device(0)
        torch.zeros(1, device="cuda")
    from devspace_amd.localkube.bench import bench_deploy

    for i in range(a.runs):
        trace = tempfile.mktemp(suffix=".jsonl")
        os.environ["LOCALKUBE_TRACE"] = trace
        t0 = time.time() * 1000.0
        r = bench_deploy(tempfile.mkdtemp())
        print(f"run {i}: cold {r['cold_s']:.3f}s warm {r['warm_s']:.3f}s phases {r['cold_phases_ms']}", flush=True)
        with open(trace) as f:
            for line in f:
                e = json.loads(line)
                if e["res"] in ("pods", "deployments", "replicasets", "nodes", "kubelet"):
                    extra = {k: v for k, v in e.items() if k not in ("t_ms", "ev", "res", "name", "phase", "ready")}
                    print(f"  +{e['t_ms'] - t0:8.1f} ms {e['ev']:8s} {e['res']:12s} {e['name'][:40]:40s} "
                          f"phase={e['phase']} ready={e['ready']} {extra or ''}")


if __name__ == "__main__":
    main()
