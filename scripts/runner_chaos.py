"""Chaos run of the hot-reload runner: faults of every kind on random ranks, edits in between,
and the invariants checked after each one.

A training module whose state carries its own consistency check (the optimizer's step count, a
tensor and a Python int must agree; see tests/test_runner_failsafe.py RESCUE_STEP) runs under
the runner with N ranks and rescue snapshots every --rescue-every seconds. The driver then, in a
loop: lets the group train, optionally makes a harmless edit (a reload), and injects one fault on
a random rank through a trigger file outside the synced tree:

  raise  an exception in step()                     -> the group restarts
  exit   os._exit(1) in step() (a crashed process)  -> the group restarts
  kill   SIGKILL to the rank (OOM killer)           -> the group restarts
  hang   the rank sleeps inside step()              -> --group-timeout ends the group, it restarts

After each fault it waits for the group to be back (`started gen=`) and checks: it resumed from
the newest committed snapshot or later than it (never from step 0 once one exists), and every
step's self-check held (no negative loss). Prints one JSON line with the recovery times.

    python scripts/runner_chaos.py [--nproc 2] [--faults 8] [--gpu]
"""

import argparse
import json
import os
import queue
import random
import re
import shutil
import signal
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TRAIN = '''
import os
import time

import torch
import torch.distributed as dist

MARKER = "v0"
SETUP_VERSION = 1
TRIGGER = os.environ["CHAOS_TRIGGER"]


def _fault(ctx):
    try:
        with open(TRIGGER) as f:
            rank, kind = f.read().split()
    except (OSError, ValueError):
        return
    if int(rank) != ctx.rank:
        return
    os.unlink(TRIGGER)
    if kind == "raise":
        raise RuntimeError(f"chaos: raise on rank {ctx.rank}")
    if kind == "exit":
        os._exit(1)
    if kind == "kill":
        os.kill(os.getpid(), 9)
    if kind == "hang":
        time.sleep(3600)


def setup(ctx):
    torch.manual_seed(0)
    dev = ctx.device
    model = torch.nn.Linear(64, 64).to(dev)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    return {"model": model, "opt": opt, "n": 0, "seen": torch.zeros(1, device=dev)}


def step(ctx, state):
    _fault(ctx)
    model, opt = state["model"], state["opt"]
    x = torch.ones(8, 64, device=ctx.device)
    loss = model(x).pow(2).mean()
    opt.zero_grad()
    loss.backward()
    if ctx.distributed:
        for p in model.parameters():
            dist.all_reduce(p.grad)
    opt.step()
    state["n"] += 1
    state["seen"] += 1
    time.sleep(0.002)
    p0 = next(iter(model.parameters()))
    same = int(opt.state[p0]["step"]) == state["n"] == int(state["seen"].item())
    return {"loss": state["n"] if same else -state["n"]}
'''


class Runner:
    def __init__(self, cmd, env, cwd):
        self.p = subprocess.Popen(cmd, env=env, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                  start_new_session=True)
        self.q = queue.Queue()
        self.lines = []
        threading.Thread(target=lambda: [self.q.put((time.monotonic(), l)) for l in self.p.stdout],
                         daemon=True).start()

    def until(self, pat, timeout):
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            try:
                t, line = self.q.get(timeout=max(0.01, deadline - time.monotonic()))
            except queue.Empty:
                break
            self.lines.append(line)
            if os.environ.get("CHAOS_VERBOSE"):
                sys.stderr.write(line)
            m = re.search(pat, line)
            if m:
                return t, m
        raise TimeoutError(f"no {pat!r} within {timeout}s:\n" + "".join(self.lines[-40:]))

    def stop(self):
        if self.p.poll() is None:
            os.killpg(self.p.pid, signal.SIGTERM)
            try:
                self.p.wait(30)
            except subprocess.TimeoutExpired:
                os.killpg(self.p.pid, signal.SIGKILL)
                self.p.wait()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, default=2)
    ap.add_argument("--faults", type=int, default=8)
    ap.add_argument("--kinds", default="raise,exit,kill,hang")
    ap.add_argument("--rescue-every", type=float, default=0.5)
    ap.add_argument("--group-timeout", type=float, default=4.0)
    ap.add_argument("--gpu", action="store_true", help="ranks on the GPU (several ranks share it over gloo)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--settle", type=float, default=0.0,
                    help="seconds of training before each fault (lets the warm standby finish its imports, as "
                         "between real failures)")
    a = ap.parse_args(argv)
    rng = random.Random(a.seed)
    work = tempfile.mkdtemp(prefix="runner-chaos-")
    r = None
    try:
        app, trig = os.path.join(work, "app"), os.path.join(work, "trigger")
        os.makedirs(app)
        entry = os.path.join(app, "train.py")
        with open(entry, "w") as f:
            f.write(TRAIN)
        env = dict(os.environ, PYTHONPATH=ROOT, CHAOS_TRIGGER=trig, DEVSPACE_RESCUE_ROOT=work)
        if a.gpu:
            env["DEVSPACE_DIST_BACKEND"] = "gloo"
        else:
            env.update(HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1", OMP_NUM_THREADS="1")
        cmd = [sys.executable, "-u", "-m", "devspace_amd.runner", "--nproc", str(a.nproc), "--watch", app,
               "--log-every", "50", "--rescue-every", str(a.rescue_every), "--group-timeout", str(a.group_timeout),
               "--max-restarts", "100", entry]
        r = Runner(cmd, env, app)
        r.until(r"started gen=1 ", 300)
        kinds = a.kinds.split(",")
        events, committed = [], 0
        for i in range(a.faults):
            # train until a snapshot newer than the last one is committed
            _, m = r.until(r"rescue snapshot step=(\d+) ", 120)
            committed = int(m.group(1))
            if rng.random() < 0.5:  # a harmless edit: a reload between faults
                src = open(entry).read()
                with open(entry, "w") as f:
                    f.write(re.sub(r'^MARKER = ".*"$', f'MARKER = "e{i}"', src, count=1, flags=re.M))
                _, m = r.until(rf"reloaded gen=\d+ marker=e{i} ", 60)
                _, m = r.until(r"rescue snapshot step=(\d+) ", 120)
                committed = int(m.group(1))
            if a.settle:
                time.sleep(a.settle)
                _, m = r.until(r"rescue snapshot step=(\d+) ", 120)
                committed = int(m.group(1))
            kind, rank = rng.choice(kinds), rng.randrange(a.nproc)
            t0 = time.monotonic()
            with open(trig + ".tmp", "w") as f:
                f.write(f"{rank} {kind}")
            os.replace(trig + ".tmp", trig)
            _, m = r.until(r"restored step=(\d+) ", 120)
            resumed = int(m.group(1))
            t_up, m2 = r.until(r"started gen=\d+ .*loss=(-?\d+) ", 120)
            first_loss = int(m2.group(1))
            ev = {"fault": kind, "rank": rank, "committed_before": committed, "resumed_from": resumed,
                  "first_loss": first_loss, "recovery_s": round(t_up - t0, 2)}
            events.append(ev)
            if resumed < committed or first_loss != resumed + 1:
                raise AssertionError(f"bad recovery: {ev}\n" + "".join(r.lines[-40:]))
        bad = [l for l in r.lines if re.search(r"loss=-\d", l)]
        if bad:
            raise AssertionError("a step saw inconsistent state:\n" + "".join(bad[:5]))
        rec = sorted(e["recovery_s"] for e in events)
        print(json.dumps({"nproc": a.nproc, "device": "gpu" if a.gpu else "cpu", "faults": len(events),
                          "settle_s": a.settle, "warm_standby": os.environ.get("DEVSPACE_WARM_STANDBY", "1") != "0",
                          "recovery_s_p50": rec[len(rec) // 2], "recovery_s_max": rec[-1], "events": events}))
        return 0
    finally:
        if r is not None:
            r.stop()
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
