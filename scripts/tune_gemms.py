#!/usr/bin/env python3
"""Tune the GEMMs of the rocm-pytorch example step on an MI355X with PyTorch TunableOp and
write the table that devspace_amd/ops/gemm_tuning.py ships (tuned/gemm_gfx950.csv); then A/B
the training step with the tuned table against the library heuristics (interleaved rounds in
one process, TunableOp toggled between them).

    PYTORCH_TUNABLEOP_VERBOSE=1 python scripts/tune_gemms.py --out gpurun_out/gemm_gfx950.csv
"""

import argparse
import importlib.util
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load_train():
    spec = importlib.util.spec_from_file_location("tinylm_tune", os.path.join(ROOT, "examples", "rocm-pytorch", "train.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1000.0 / iters


def write_table(path):
    tunable = torch.cuda.tunable
    lines = [f"Validator,{k},{v}" for k, v in tunable.get_validators()]
    lines += [",".join(str(x) for x in r) for r in tunable.get_results()]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return len(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--tune-ms", type=int, default=15, help="max profiling time per solution")
    ap.add_argument("--tune-iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default="")
    a = ap.parse_args()

    tunable = torch.cuda.tunable
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.record_untuned_enable(False)
    tunable.set_max_tuning_duration(a.tune_ms)
    tunable.set_max_tuning_iterations(a.tune_iters)
    tunable.set_numerical_check_tolerances(True, 1e-2, 1e-2)  # reject solutions that disagree with the default
    tunable.set_filename(a.out + ".exit.csv")  # TunableOp's own exit-time dump; ours is written below

    from devspace_amd.runner import Context  # what the runner hands train.py

    def Ctx():
        return Context(0, 1, 0, torch.device("cuda"))

    mod = load_train()
    state = mod.setup(Ctx())
    t0 = time.perf_counter()
    for i in range(3):  # every GEMM shape of fwd + bwd + the optimizer is seen in step 1
        mod.step(Ctx(), state)
        torch.cuda.synchronize()
        print(f"tuning step {i} done at {time.perf_counter() - t0:.1f}s", flush=True)
    n = write_table(a.out)
    print(f"wrote {n} lines to {a.out}", flush=True)
    tunable.tuning_enable(False)

    res = {"heuristic": [], "tuned": []}
    for _ in range(a.rounds):
        tunable.enable(False)
        res["heuristic"].append(timeit(lambda: mod.step(Ctx(), state), a.iters))
        tunable.enable(True)
        res["tuned"].append(timeit(lambda: mod.step(Ctx(), state), a.iters))
    h, t = statistics.median(res["heuristic"]), statistics.median(res["tuned"])
    print(f"TinyLM step (B8xT512, 4x1024): heuristic {h:.3f} ms  tuned {t:.3f} ms  speedup {h / t:.3f}x "
          f"(median of {a.rounds} interleaved rounds x {a.iters} steps)")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0), "heuristic_ms": h, "tuned_ms": t, "rounds": res}, f,
                      indent=1)


if __name__ == "__main__":
    main()
