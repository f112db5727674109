#!/usr/bin/env python3
"""Inner-loop benchmark: edit -> pod hot-reload latency (+ deploy wall-clock) on MI355X.

BASELINE.json metric: "inner-loop p50 ms (edit->pod hot-reload) + deploy wall-clock s".
The pod is the rocm/pytorch example (examples/rocm-pytorch/train.py, a bf16 TinyLM training
loop) served by the local-pod backend: `devspace deploy` against the bundled local cluster
(fake Kubernetes API server + process kubelet + Docker-API image builder, all on this host —
no k8s/network on the GPU box), then `devspace dev` syncs the project into the pod while the
workload runs under devspace_amd.runner on N GPUs (one process per GPU, RCCL over xGMI).

One timed "step" = edit train.py locally -> change synced into the pod -> runner swaps code ->
first training step with the new code completes on every GPU (rank 0 prints the marker).

Two columns are reported (BASELINE.md "How the rebuild will be compared"):
  value                          this framework (fast sync protocol + warm hot-reload)
  reference_equivalent_p50_ms    same hardware, reference constants: compat sync protocol
                                 (600 ms window, sleep-0.1 receive polling) + cold restart
                                 of the workload on change (nodemon-style, as the reference)

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
For N>1 the driver launches one bench rank per GPU with torch.distributed.run; rank 0 drives
the dev loop for a pod requesting amd.com/gpu: N, the other ranks join the barriers.
"""

from __future__ import annotations

import argparse
import json
import os
import re
import shutil
import signal
import statistics
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "inner-loop p50 ms (edit->pod hot-reload) + deploy wall-clock s, quickstart"


def _pct(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


class LineTail:
    """Collects a child's stdout lines with arrival timestamps."""

    def __init__(self, stream, echo_prefix=None):
        self.lines = []
        self.cv = threading.Condition()
        self.echo_prefix = echo_prefix
        self.t = threading.Thread(target=self._run, args=(stream,), daemon=True)
        self.t.start()

    def _run(self, stream):
        for raw in iter(stream.readline, b""):
            line = raw.decode(errors="replace").rstrip("\n")
            now = time.perf_counter()
            if self.echo_prefix and os.environ.get("BENCH_VERBOSE"):
                sys.stderr.write(f"{self.echo_prefix}{line}\n")
            with self.cv:
                self.lines.append((now, line))
                self.cv.notify_all()

    def wait_for(self, pattern, start_index=0, timeout=120.0):
        rx = re.compile(pattern)
        deadline = time.monotonic() + timeout
        with self.cv:
            i = start_index
            while True:
                while i < len(self.lines):
                    t, line = self.lines[i]
                    i += 1
                    if rx.search(line):
                        return t, line, i
                left = deadline - time.monotonic()
                if left <= 0:
                    tail = "\n".join(l for _, l in self.lines[-20:])
                    raise TimeoutError(f"timed out waiting for /{pattern}/; last output:\n{tail}")
                self.cv.wait(left)


def _set_marker(path, marker):
    with open(path, "r") as f:
        src = f.read()
    src = re.sub(r'^MARKER = ".*"$', f'MARKER = "{marker}"', src, count=1, flags=re.M)
    with open(path, "w") as f:
        f.write(src)


def _wait_file_contains(path, needle, timeout=60.0):
    deadline = time.monotonic() + timeout
    nb = needle.encode()
    while time.monotonic() < deadline:
        try:
            with open(path, "rb") as f:
                if nb in f.read():
                    return time.perf_counter()
        except OSError:
            pass
        time.sleep(0.0002)
    raise TimeoutError(f"{needle} never reached {path}")


def inner_loop(workdir, sync_mode, restart, nproc, steps, warmup, tiny=False, timed_start=None, timed_end=None):
    """Runs the edit->reload loop against a local pod directory; returns latency samples.

    `timed_start`/`timed_end` are invoked right before the first and after the last timed
    step (after warmup), so the caller can bracket exactly K steps with barriers."""
    from devspace_amd import _native

    proj = os.path.join(workdir, f"proj-{sync_mode}-{'restart' if restart else 'hot'}")
    pod = os.path.join(workdir, f"pod-{sync_mode}-{'restart' if restart else 'hot'}", "app")
    os.makedirs(proj, exist_ok=True)
    os.makedirs(pod, exist_ok=True)
    shutil.copy(os.path.join(ROOT, "examples", "rocm-pytorch", "train.py"), os.path.join(proj, "train.py"))
    if tiny:
        p = os.path.join(proj, "train.py")
        s = open(p).read()
        for k, v in (("VOCAB", 256), ("DIM", 64), ("HEADS", 4), ("LAYERS", 1), ("SEQ", 32), ("BATCH", 2)):
            s = re.sub(rf"^{k} = \d+$", f"{k} = {v}", s, flags=re.M)
        open(p, "w").write(s)
    helper = os.path.join(ROOT, "bin", "devspace-helper")
    sess = _native.SyncSession(
        proj,
        pod,
        mode=sync_mode,
        exclude=["__pycache__/", "*.pyc"],
        helper_path=helper,
        log_dir=os.path.join(workdir, "logs"),
        pod_name=f"bench-{sync_mode}",
    )
    sess.start()
    if not sess.wait_initial_sync(60000):
        raise RuntimeError(f"initial sync failed: {sess.error()}")
    _wait_file_contains(os.path.join(pod, "train.py"), "MARKER")
    cmd = [sys.executable, "-u", "-m", "devspace_amd.runner", "--nproc", str(nproc), "--watch", pod]
    if restart:
        cmd.append("--restart")
    cmd.append(os.path.join(pod, "train.py"))
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    runner = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, start_new_session=True)
    tail = LineTail(runner.stdout, echo_prefix=f"[{sync_mode}] ")
    samples, sync_samples = [], []
    try:
        _, _, idx = tail.wait_for(r"\[devspace-runner\] started gen=\d+ marker=v0", timeout=600)
        proj_file = os.path.join(proj, "train.py")
        pod_file = os.path.join(pod, "train.py")
        for i in range(warmup + steps):
            if i == warmup and timed_start:
                timed_start()
            # alternate marker lengths so consecutive edits always differ in size (the
            # reference-equivalent mode compares rounded mtimes + size, like the reference)
            marker = f"e{i}" + ("_" * (i % 2))
            t0 = time.perf_counter()
            _set_marker(proj_file, marker)
            t_sync = _wait_file_contains(pod_file, f'MARKER = "{marker}"')
            pat = rf"\[devspace-runner\] (reloaded|started) gen=\d+ marker={re.escape(marker)} "
            t1, _, idx = tail.wait_for(pat, start_index=idx, timeout=600)
            if i >= warmup:
                samples.append((t1 - t0) * 1000.0)
                sync_samples.append((t_sync - t0) * 1000.0)
        if timed_end:
            timed_end()
        stats = sess.stats()
    finally:
        try:
            os.killpg(runner.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
        try:
            runner.wait(10)
        except subprocess.TimeoutExpired:
            os.killpg(runner.pid, signal.SIGKILL)
            runner.wait()
        sess.stop()
    return {"reload_ms": samples, "sync_ms": sync_samples, "sync_stats": stats, "mode": sess.mode()}


def deploy_wall_clock(workdir):
    """`devspace deploy` of the quickstart-style project against the local cluster (seconds)."""
    try:
        from devspace_amd.localkube import bench_deploy
    except Exception:
        return None
    try:
        return bench_deploy(workdir)
    except Exception as e:  # reported, not fatal for the latency metric
        sys.stderr.write(f"deploy benchmark failed: {e}\n")
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ref-steps", type=int, default=5, help="timed steps for the reference-equivalent run")
    ap.add_argument("--sync-mode", default="fast", choices=["fast", "helper", "compat"])
    ap.add_argument("--tiny", action="store_true", help="tiny model (CPU smoke only)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    cuda = torch.cuda.is_available()
    if cuda:
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
    pg = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist

    def barrier_sync():
        if pg is not None:
            pg.barrier()
        if cuda:
            torch.cuda.synchronize()

    nproc = max(args.gpus, world) if cuda else 1
    workdir = tempfile.mkdtemp(prefix="devspace-bench-")
    result = {}
    deploy_s = None
    clock = {}

    def timed_start():
        barrier_sync()
        clock["t0"] = time.perf_counter()

    def timed_end():
        barrier_sync()
        clock["t1"] = time.perf_counter()

    try:
        if rank == 0:
            deploy_s = deploy_wall_clock(workdir)
            result = inner_loop(workdir, args.sync_mode, False, nproc, args.steps, args.warmup, tiny=args.tiny,
                                timed_start=timed_start, timed_end=timed_end)
        else:
            timed_start()
            timed_end()
        elapsed = clock["t1"] - clock["t0"]
        ref = None
        if rank == 0 and args.ref_steps > 0:
            ref = inner_loop(workdir, "compat", True, nproc, args.ref_steps, 1, tiny=args.tiny)
        barrier_sync()
    finally:
        shutil.rmtree(workdir, ignore_errors=True)

    ms_total = elapsed * 1000.0
    if pg is not None:
        t = torch.tensor([ms_total], dtype=torch.float64)
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        ms_total = float(t.item())
    if rank != 0:
        if pg is not None:
            pg.destroy_process_group()
        return 0
    p50 = _pct(result["reload_ms"], 0.5)
    out = {
        "metric": METRIC,
        "value": round(p50, 2),
        "unit": "ms",
        "n_gpus": nproc,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_total / max(1, args.steps), 2),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random tokens; random-init TinyLM weights)",
        "config": {
            "model": "examples/rocm-pytorch TinyLM (4x1024, 67M params) hot-reload pod",
            "global_batch": 8 * nproc,
            "seq_len": 512,
            "parallelism": f"dp{nproc}",
            "sync_mode": result["mode"],
            "backend": "local-pod (fake k8s API + process kubelet)",
        },
        "p50_ms": round(p50, 2),
        "p90_ms": round(_pct(result["reload_ms"], 0.9), 2),
        "sync_p50_ms": round(_pct(result["sync_ms"], 0.5), 2),
        "deploy_wall_clock_s": None if deploy_s is None else round(deploy_s, 3),
    }
    if ref:
        rp50 = _pct(ref["reload_ms"], 0.5)
        out["reference_equivalent_p50_ms"] = round(rp50, 2)
        out["reference_equivalent_sync_p50_ms"] = round(_pct(ref["sync_ms"], 0.5), 2)
        out["speedup_vs_reference_equivalent"] = round(rp50 / p50, 2) if p50 else None
    print(json.dumps(out))
    if pg is not None:
        pg.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
