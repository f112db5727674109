#!/usr/bin/env python3
"""Large-file sync throughput of one protocol, with the CPU time each process spent: which side
limits a checkpoint transfer (the CLI, the in-container helper, tar/gzip in the shell
protocols, or the pipe).

    python scripts/sync_throughput.py [--mode helper|fast|compat] [--mib 1024]

Runs the real `devspace sync --local-root` (local shells stand in for kubectl exec, as in
tests/test_sync_large.py): one incompressible file up, another down, each timed from the
moment it appears to the moment it is complete on the other side."""
import argparse
import os
import signal
import subprocess
import tempfile
import time

import psutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin", "devspace")


def _rand(path, size):
    with open(path, "wb") as f:
        left = size
        while left:
            n = min(left, 16 << 20)
            f.write(os.urandom(n))
            left -= n


def _cpu(tree_root):
    out = {}
    try:
        procs = [tree_root] + tree_root.children(recursive=True)
    except psutil.Error:
        return out
    for p in procs:
        try:
            t = p.cpu_times()
            name = p.name()
            name = "devspace-helper" if name.startswith("devspace-helpe") else name
            out[name] = out.get(name, 0.0) + t.user + t.system
        except psutil.Error:
            pass
    return out


def _wait(path, size, timeout, tick):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        try:
            if os.path.getsize(path) == size:
                return
        except OSError:
            pass
        tick()
        time.sleep(0.01)
    raise TimeoutError(path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="helper")
    ap.add_argument("--mib", type=int, default=1024)
    a = ap.parse_args()
    size = a.mib << 20
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        src, pod = os.path.join(d, "src"), os.path.join(d, "pod")
        os.makedirs(src)
        os.makedirs(os.path.join(pod, "app"))
        up, down = os.path.join(d, "up.bin"), os.path.join(d, "down.bin")
        _rand(up, size)
        _rand(down, size)
        env = dict(os.environ, HOME=os.path.join(d, "home"), DEVSPACE_NONINTERACTIVE="1",
                   DEVSPACE_SKIP_UPDATE_CHECK="1", DEVSPACE_SYNC_WARN_FILE_MB="0")
        p = subprocess.Popen([BIN, "sync", "--local-root", pod, "--local", src, "--container", "/app", "--mode", a.mode],
                             cwd=d, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.STDOUT, start_new_session=True)
        root = psutil.Process(p.pid)
        seen = {}

        def tick():  # children exit between phases: keep the last CPU reading of each name
            for k, v in _cpu(root).items():
                seen[k] = max(seen.get(k, 0.0), v)

        try:
            time.sleep(1.0)
            base = dict(seen)
            t0 = time.perf_counter()
            os.link(up, os.path.join(src, "up.bin"))
            _wait(os.path.join(pod, "app", "up.bin"), size, 600, tick)
            up_s = time.perf_counter() - t0
            cpu_up = {k: round(v - base.get(k, 0.0), 2) for k, v in seen.items()}
            base = dict(seen)
            t1 = time.perf_counter()
            os.link(down, os.path.join(pod, "app", "down.bin"))
            _wait(os.path.join(src, "down.bin"), size, 600, tick)
            down_s = time.perf_counter() - t1
            cpu_down = {k: round(v - base.get(k, 0.0), 2) for k, v in seen.items()}
        finally:
            os.killpg(p.pid, signal.SIGINT)
            p.wait(30)
    print(f"{a.mode}: up {size / up_s / 1e6:.0f} MB/s ({up_s:.2f} s) cpu {cpu_up}")
    print(f"{a.mode}: down {size / down_s / 1e6:.0f} MB/s ({down_s:.2f} s) cpu {cpu_down}")


if __name__ == "__main__":
    main()
