"""What the runner's rescue snapshots cost on the flagship example, and what they save.

Runs examples/rocm-pytorch/train.py (TinyLM, model + AdamW in HBM) under the hot-reload runner
with --rescue-dir and a short --rescue-every, kills the process outright (SIGKILL, as an OOM kill
or a GPU fault would) after a few snapshots, starts it again and reads back:
  * snapshot size per rank, the time each snapshot paused training for and the time its
    (background) write to shared memory took,
  * the restore time and the step the new process resumed from (instead of step 0),
  * the steady-state step period with snapshots on.
Prints one JSON line.

    python scripts/rescue_cost.py [--every 2] [--snapshots 3]
"""

import argparse
import json
import os
import queue
import re
import shutil
import signal
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class Proc:
    def __init__(self, cmd, env, cwd):
        self.p = subprocess.Popen(cmd, env=env, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                  start_new_session=True)
        self.q = queue.Queue()
        self.lines = []
        threading.Thread(target=lambda: [self.q.put(l) for l in self.p.stdout], daemon=True).start()

    def until(self, pat, timeout):
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            try:
                line = self.q.get(timeout=max(0.01, deadline - time.monotonic()))
            except queue.Empty:
                break
            self.lines.append(line)
            sys.stderr.write(line)
            m = re.search(pat, line)
            if m:
                return m
        raise TimeoutError(f"no {pat!r} in {timeout}s:\n" + "".join(self.lines[-30:]))

    def kill(self):
        if self.p.poll() is None:
            os.killpg(self.p.pid, signal.SIGKILL)
        self.p.wait()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--every", type=float, default=2.0)
    ap.add_argument("--snapshots", type=int, default=3)
    ap.add_argument("--layers", type=int, default=0, help="TinyLM layers (default: the example's)")
    ap.add_argument("--dim", type=int, default=0, help="TinyLM width (default: the example's)")
    args = ap.parse_args()
    work = tempfile.mkdtemp(prefix="rescue-cost-")
    try:
        app = os.path.join(work, "app")
        shutil.copytree(os.path.join(ROOT, "examples", "rocm-pytorch"), app,
                        ignore=shutil.ignore_patterns("devspace_amd", "__pycache__"))
        if args.layers or args.dim:  # a bigger model than the example's, same code
            import re

            train = os.path.join(app, "train.py")
            src = open(train).read()
            if args.layers:
                src = re.sub(r"^LAYERS = \d+$", f"LAYERS = {args.layers}", src, count=1, flags=re.M)
            if args.dim:
                src = re.sub(r"^DIM = \d+$", f"DIM = {args.dim}", src, count=1, flags=re.M)
            open(train, "w").write(src)
        keep = os.path.join(work, "rescue")
        env = dict(os.environ, PYTHONPATH=ROOT)
        cmd = [sys.executable, "-u", "-m", "devspace_amd.runner", "--watch", app, "--log-every", "5",
               "--rescue-every", str(args.every), "--rescue-dir", keep, os.path.join(app, "train.py")]
        first = Proc(cmd, env, app)
        snaps = []
        try:
            first.until(r"started gen=1 ", 300)
            for _ in range(args.snapshots):
                m = first.until(r"rescue snapshot step=(\d+) gen=\d+ ([\d.]+) MiB/rank: training paused ([\d.]+) ms, "
                                r"(.*) in ([\d.]+) ms", 120)
                snaps.append({"step": int(m.group(1)), "mib": float(m.group(2)), "pause_ms": float(m.group(3)),
                              "how": m.group(4), "write_ms": float(m.group(5))})
            period = first.until(r"step=\d+ gen=\d+ loss=(\S+) period_ms=([\d.]+)", 120)
        finally:
            first.kill()
        second = Proc(cmd, env, app)
        try:
            m = second.until(r"restored step=(\d+) gen=\d+ from the rescue snapshot \(age ([\d.]+) s, "
                             r"([\d.]+) MiB/rank in ([\d.]+) ms\)", 300)
            restored = {"step": int(m.group(1)), "age_s": float(m.group(2)), "mib": float(m.group(3)),
                        "ms": float(m.group(4))}
            started = second.until(r"started gen=1 .*loss=(\S+) startup_ms=([\d.]+)", 120)
        finally:
            second.kill()
        out = {
            "what": "examples/rocm-pytorch TinyLM under the runner: rescue snapshots every "
                    f"{args.every:g} s, SIGKILL, restart with the same --rescue-dir",
            "model": {"layers": args.layers or "example", "dim": args.dim or "example"},
            "snapshots": snaps,
            "pause_ms_p50": sorted(s["pause_ms"] for s in snaps)[len(snaps) // 2],
            "write_ms_p50": sorted(s["write_ms"] for s in snaps)[len(snaps) // 2],
            "step_period_ms": float(period.group(2)),
            "pause_at_default_interval_pct": round(100.0 * sorted(s["pause_ms"] for s in snaps)[len(snaps) // 2] / 60000.0,
                                                   5),
            "loss_before_kill": period.group(1),
            "restored": restored,
            "resumed_from_step": restored["step"],
            "restart_startup_ms": float(started.group(2)),
            "first_loss_after_restart": started.group(1),
        }
        print(json.dumps(out))
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
