#!/usr/bin/env python3
"""Inner-loop benchmark: edit -> pod hot-reload latency (+ deploy wall-clock) on MI355X.

BASELINE.json metric: "inner-loop p50 ms (edit->pod hot-reload) + deploy wall-clock s".

Everything goes through the real `devspace` CLI against the bundled local cluster (fake
Kubernetes API server + process kubelet advertising amd.com/gpu + Docker Engine API builder,
all on this host — the GPU box has no k8s/Docker/network). By default the API server speaks
TLS (https + wss, client certificates), as every real cluster does (`--transport plain` for ws).

  value (timed, K steps): examples/rocm-pytorch (BASELINE configs[4]; bf16 TinyLM training pod,
     amd.com/gpu: N, one process per GPU under the hot-reload runner with an RCCL process group).
     `devspace dev` deploys it, syncs the project into the pod over the exec WebSocket and
     attaches to its output. One step = edit train.py locally -> change synced into the pod ->
     runner swaps code at the step boundary -> first training step with the new code finishes
     on every GPU -> its log line reaches `devspace dev`'s terminal.
  quickstart (untimed extra): examples/quickstart (Node.js) under `devspace dev` with the
     container running watch.js (restart on change, as nodemon in the reference's quickstart).
     One sample = edit index.js -> HTTP GET through devspace's port-forward shows the new text.
     Repeated with the reference's compat sync protocol -> `tool_attributable` (same app, same
     restart, same transport; only the sync protocol differs).
  deploy (untimed extra): `devspace deploy` of examples/quickstart on a fresh cluster, cold and
     forced-warm, with per-phase times and TCP/TLS handshake counts from the CLI's trace.
     `control_plane_only`: the bundled Docker daemon does not execute RUN steps.
  reference_equivalent: rocm-pytorch with compat sync + cold workload restart per change.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
For N>1 the driver launches one bench rank per GPU with torch.distributed.run; rank 0 drives
the dev loop for a pod requesting amd.com/gpu: N; the other ranks join the timing barriers.
"""

from __future__ import annotations

import argparse
import json
import os
import random
import re
import shutil
import signal
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "inner-loop p50 ms (edit->pod hot-reload) + deploy wall-clock s, quickstart"
EDIT_JITTER_S = 0.010  # uniform think time before each edit (> 2 training steps of the example)
BUILDER_FIDELITY = ("bundled Docker Engine API daemon: Dockerfile parsed, context hashed/tarred, "
                    "RUN steps not executed; pods run on the host runtime")
TINY = (("VOCAB", 256), ("DIM", 64), ("HEADS", 4), ("LAYERS", 1), ("SEQ", 32), ("BATCH", 2))


def _pct(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def _log(msg):
    sys.stderr.write(f"[bench] {msg}\n")
    sys.stderr.flush()


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
                    tail = "\n".join(l for _, l in self.lines[-30:])
                    raise TimeoutError(f"timed out waiting for /{pattern}/; last output:\n{tail}")
                self.cv.wait(left)

    def size(self):
        with self.cv:
            return len(self.lines)


def _set_marker(path, marker):
    with open(path, "r") as f:
        src = f.read()
    src = re.sub(r'^MARKER = ".*"$', f'MARKER = "{marker}"', src, count=1, flags=re.M)
    with open(path, "w") as f:
        f.write(src)


def _shrink(path):
    s = open(path).read()
    for k, v in TINY:
        s = re.sub(rf"^{k} = \d+$", f"{k} = {v}", s, flags=re.M)
    open(path, "w").write(s)


def _wait_file_contains(path, needle, timeout=60.0, interval=0.0002):
    deadline = time.monotonic() + timeout
    nb = needle.encode()
    while time.monotonic() < deadline:
        try:
            with open(path, "rb") as f:
                if nb in f.read():
                    return time.perf_counter()
        except OSError:
            pass
        time.sleep(interval)
    raise TimeoutError(f"{needle} never reached {path}")


def _killpg(p, grace=15):
    if p is None or p.poll() is not None:
        return
    try:
        os.killpg(p.pid, signal.SIGINT)
        p.wait(grace)
    except (ProcessLookupError, subprocess.TimeoutExpired):
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.wait()


# ---------------------------------------------------------------------------- full CLI path


def dev_loop(workdir, nproc, gpus, steps, warmup, tiny=False, timed_start=None, timed_end=None, tls=True):
    """`devspace deploy` + `devspace dev` of examples/rocm-pytorch on the local cluster."""
    from devspace_amd.localkube import LocalCluster
    from devspace_amd.localkube.bench import devspace_env, run_devspace

    base = os.path.join(workdir, "dev-bench")
    proj = os.path.join(base, "rocm-pytorch")
    shutil.copytree(os.path.join(ROOT, "examples", "rocm-pytorch"), proj, symlinks=True)
    train = os.path.join(proj, "train.py")
    if tiny:
        _shrink(train)
    values = os.path.join(proj, "chart", "values.yaml")
    v = open(values).read()
    v = re.sub(r"gpu: \d+", f"gpu: {gpus}", v)
    open(values, "w").write(v)

    cluster = LocalCluster(os.path.join(base, "cluster"), gpus=gpus, tls=tls).start()
    dev = None
    try:
        env = devspace_env(cluster, base)
        env["DEVSPACE_NPROC"] = str(nproc)  # used when the pod requests no GPU (CPU smoke)
        cluster.kubelet.extra_env["DEVSPACE_NPROC"] = str(nproc)
        # `devspace dev` builds (dev image cache), deploys the chart, waits for the rollout,
        # then starts sync + attach on the newest running pod.
        t_dev = time.perf_counter()
        dev = subprocess.Popen([os.path.join(ROOT, "bin", "devspace"), "dev", "--terminal=false",
                                "--portforwarding=false"], cwd=proj, env=env, stdout=subprocess.PIPE,
                               stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, start_new_session=True)
        tail = LineTail(dev.stdout, echo_prefix="[dev] ")
        _, line, idx = tail.wait_for(r"Sync started on", timeout=900)
        deploy_s = time.perf_counter() - t_dev
        ns, pod_name = re.search(r"Pod: ([^/\s]+)/([^)\s]+)", line).groups()
        pod = cluster.store.get("", "pods", ns, pod_name)
        cname = pod["spec"]["containers"][0]["name"]
        root = json.loads(pod["metadata"]["annotations"]["devspace.sh/local-roots"])[cname]
        _log(f"dev: pod {pod_name} synced after {deploy_s:.2f}s")
        _, _, idx = tail.wait_for(r"Attached to container", start_index=idx, timeout=120)
        _wait_file_contains(root + ".log", "[devspace-runner] started gen=", timeout=900, interval=0.05)
        m = re.search(r"\[devspace-runner\] started gen=\d+ .*?world=(\d+) device=(\S+)", open(root + ".log").read())
        pod_world = int(m.group(1)) if m else 0
        _log(f"runner up: {pod_world} rank(s), rank 0 on {m.group(2) if m else '?'}")
        if pod_world != nproc:
            raise RuntimeError(f"the pod runs {pod_world} training rank(s), expected {nproc}")
        mode = os.environ.get("DEVSPACE_SYNC_MODE") or (
            "helper" if os.path.exists(os.path.join(ROOT, "bin", "devspace-helper")) else "fast")
        pod_file = os.path.join(root, "app", "train.py")
        samples, sync_samples = [], []
        parts = {"pickup_ms": [], "inflight_ms": [], "step_ms": [], "code_swap_ms": [], "log_delivery_ms": [],
             "train_period_ms": []}
        rng = random.Random(1234)
        for i in range(warmup + steps):
            if i == warmup and timed_start:
                timed_start()
            marker = f"e{i}" + ("_" * (i % 2))
            # think time before each edit: a developer's save lands at a random point of the
            # pod's training step, not right after the previous reload's log line (that would
            # fix the phase and always wait out the same share of the in-flight step)
            time.sleep(rng.uniform(0.0, EDIT_JITTER_S))
            t0 = time.perf_counter()
            _set_marker(train, marker)
            t_sync = _wait_file_contains(pod_file, f'MARKER = "{marker}"')
            pat = rf"\[devspace-runner\] (reloaded|started) gen=\d+ marker={re.escape(marker)} "
            t1, line, idx = tail.wait_for(pat, start_index=idx, timeout=600)
            if i >= warmup:
                samples.append((t1 - t0) * 1000.0)
                sync_samples.append((t_sync - t0) * 1000.0)
                # where the time goes: runner-side pickup (change seen -> new step done),
                # delivery (runner print -> line in `devspace dev` output; same host clock)
                f = dict(re.findall(r"(\w+_ms|t_mono)=([\d.]+)", line))
                if "t_mono" in f:
                    parts["pickup_ms"].append(float(f["pickup_ms"]))
                    parts["step_ms"].append(float(f["step_ms"]))
                    parts["code_swap_ms"].append(float(f["reload_ms"]))
                    if "inflight_ms" in f:
                        parts["inflight_ms"].append(float(f["inflight_ms"]))
                        parts["train_period_ms"].append(float(f["period_ms"]))
                    parts["log_delivery_ms"].append((t1 - float(f["t_mono"])) * 1000.0)
        if timed_end:
            timed_end()
        return {"reload_ms": samples, "sync_ms": sync_samples, "mode": mode, "pod_deploy_s": deploy_s,
                "parts": parts}
    finally:
        _killpg(dev)
        cluster.stop()


# ---------------------------------------------------------------------------- quickstart (Node.js)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _http_get(port, timeout=2.0):
    import http.client

    c = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout)
    try:
        c.request("GET", "/")
        return c.getresponse().read().decode(errors="replace")
    except (OSError, http.client.HTTPException):
        return None
    finally:
        c.close()


QS_GREETING = re.compile(r"res\.end\('[^']*' \+")


def _qs_edit(path, marker):
    src = open(path).read()
    src, n = QS_GREETING.subn(f"res.end('Hello [{marker}] from ' +", src, count=1)
    assert n == 1, "examples/quickstart/index.js greeting line not found"
    with open(path, "w") as f:
        f.write(src)


def quickstart_loop(workdir, steps, warmup, sync_mode=None, tls=True):
    """examples/quickstart edit -> reload, the way its README runs the dev loop: `devspace dev`
    (sync + port-forward) with the container running `npm run dev` (watch.js restarts node on
    change, as nodemon does in the reference's quickstart). One sample = edit index.js locally ->
    HTTP GET through devspace's port-forward returns the new greeting. CPU-only pod."""
    import yaml

    from devspace_amd.localkube import LocalCluster
    from devspace_amd.localkube.bench import devspace_env

    tag = sync_mode or "default"
    base = os.path.join(workdir, f"qs-bench-{tag}")
    proj = os.path.join(base, "quickstart")
    shutil.copytree(os.path.join(ROOT, "examples", "quickstart"), proj, symlinks=True)
    remote, local = _free_port(), _free_port()
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["dev"]["overrideImages"][0]["entrypoint"] = ["node", "watch.js", "index.js"]
    cfg["dev"]["ports"][0]["portMappings"] = [{"localPort": local, "remotePort": remote}]
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    values = os.path.join(proj, "chart", "values.yaml")
    v = yaml.safe_load(open(values))
    v["components"][0]["containers"][0]["env"] = [{"name": "PORT", "value": str(remote)}]
    open(values, "w").write(yaml.safe_dump(v))

    cluster = LocalCluster(os.path.join(base, "cluster"), gpus=0, tls=tls).start()
    dev = None
    try:
        env = devspace_env(cluster, base)
        if sync_mode:
            env["DEVSPACE_SYNC_MODE"] = sync_mode
        dev = subprocess.Popen([os.path.join(ROOT, "bin", "devspace"), "dev", "--terminal=false"], cwd=proj, env=env,
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                               start_new_session=True)
        tail = LineTail(dev.stdout, echo_prefix=f"[qs-{tag}] ")
        _, line, idx = tail.wait_for(r"Sync started on", timeout=300)
        ns, pod_name = re.search(r"Pod: ([^/\s]+)/([^)\s]+)", line).groups()
        pod = cluster.store.get("", "pods", ns, pod_name)
        cname = pod["spec"]["containers"][0]["name"]
        root = json.loads(pod["metadata"]["annotations"]["devspace.sh/local-roots"])[cname]
        deadline = time.monotonic() + 60
        while not (_http_get(local) or "").startswith("Hello"):
            if time.monotonic() > deadline:
                raise TimeoutError("quickstart server never answered through the port-forward")
            time.sleep(0.01)
        index, pod_index = os.path.join(proj, "index.js"), os.path.join(root, "app", "index.js")
        samples, sync_samples = [], []
        rng = random.Random(4321)
        for i in range(warmup + steps):
            marker = f"q{i}" + ("_" * (i % 2))  # compat mode compares size + mtime (s)
            time.sleep(rng.uniform(0.0, EDIT_JITTER_S))
            t0 = time.perf_counter()
            _qs_edit(index, marker)
            t_sync = _wait_file_contains(pod_index, f"[{marker}]", timeout=60)
            deadline = time.monotonic() + 60
            while True:
                body = _http_get(local)
                if body and f"[{marker}]" in body:
                    t1 = time.perf_counter()
                    break
                if time.monotonic() > deadline:
                    raise TimeoutError(f"edit {marker} never reached the forwarded server (last: {body!r})")
                time.sleep(0.0005)
            if i >= warmup:
                samples.append((t1 - t0) * 1000.0)
                sync_samples.append((t_sync - t0) * 1000.0)
        return {"reload_ms": samples, "sync_ms": sync_samples}
    finally:
        _killpg(dev)
        cluster.stop()


# ---------------------------------------------------------------------------- reference-equivalent


def inner_loop(workdir, sync_mode, restart, nproc, steps, warmup, tiny=False):
    """Edit -> reload against a pod directory through the sync engine directly.

    Used for the reference-equivalent column: compat sync protocol (the reference's shell
    scripts and timing constants) + cold restart of the workload on every change."""
    from devspace_amd import _native

    tag = f"{sync_mode}-{'restart' if restart else 'hot'}"
    proj = os.path.join(workdir, f"proj-{tag}")
    pod = os.path.join(workdir, f"pod-{tag}", "app")
    os.makedirs(proj, exist_ok=True)
    os.makedirs(pod, exist_ok=True)
    shutil.copy(os.path.join(ROOT, "examples", "rocm-pytorch", "train.py"), os.path.join(proj, "train.py"))
    if tiny:
        _shrink(os.path.join(proj, "train.py"))
    sess = _native.SyncSession(proj, pod, mode=sync_mode, exclude=["__pycache__/", "*.pyc"],
                               helper_path=os.path.join(ROOT, "bin", "devspace-helper"),
                               log_dir=os.path.join(workdir, "logs"), pod_name=f"bench-{sync_mode}")
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
    tail = LineTail(runner.stdout, echo_prefix=f"[{tag}] ")
    samples, sync_samples = [], []
    try:
        _, _, idx = tail.wait_for(r"\[devspace-runner\] started gen=\d+ marker=v0", timeout=600)
        proj_file, pod_file = os.path.join(proj, "train.py"), os.path.join(pod, "train.py")
        rng = random.Random(1234)
        for i in range(warmup + steps):
            # alternate marker lengths so consecutive edits always differ in size (compat mode
            # compares rounded mtimes + size, like the reference)
            marker = f"e{i}" + ("_" * (i % 2))
            time.sleep(rng.uniform(0.0, EDIT_JITTER_S))
            t0 = time.perf_counter()
            _set_marker(proj_file, marker)
            t_sync = _wait_file_contains(pod_file, f'MARKER = "{marker}"')
            pat = rf"\[devspace-runner\] (reloaded|started) gen=\d+ marker={re.escape(marker)} "
            t1, _, idx = tail.wait_for(pat, start_index=idx, timeout=600)
            if i >= warmup:
                samples.append((t1 - t0) * 1000.0)
                sync_samples.append((t_sync - t0) * 1000.0)
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
    return {"reload_ms": samples, "sync_ms": sync_samples, "mode": sess.mode()}


# ---------------------------------------------------------------------------- main


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ref-steps", type=int, default=3, help="timed steps for the reference-equivalent run (0=skip)")
    ap.add_argument("--no-deploy-bench", action="store_true", help="skip the quickstart deploy wall-clock")
    ap.add_argument("--tiny", action="store_true", help="tiny model (CPU smoke only)")
    ap.add_argument("--transport", choices=("tls", "plain"), default="tls",
                    help="API server transport of the local cluster (tls = https + wss with mTLS, as a real cluster)")
    ap.add_argument("--qs-steps", type=int, default=10, help="timed quickstart (Node.js) reloads (0=skip)")
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

        # bench ranks only coordinate timing; the workload's own RCCL group lives in the pod
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist

    def barrier_sync():
        if pg is not None:
            pg.barrier()
        if cuda:
            torch.cuda.synchronize()

    nproc = max(args.gpus, world)
    gpus = nproc if cuda else 0
    if not cuda:
        # CPU rehearsal of the N>1 shape: the pod runs one gloo rank per bench rank
        nproc = world
    workdir = tempfile.mkdtemp(prefix="devspace-bench-")
    tls = args.transport == "tls"
    result, ref, deploy, qs, qs_compat = {}, None, None, None, None
    clock = {}

    def timed_start():
        barrier_sync()
        clock["t0"] = time.perf_counter()

    def timed_end():
        barrier_sync()
        clock["t1"] = time.perf_counter()

    try:
        if rank == 0:
            if not args.no_deploy_bench:
                try:
                    deploy = __import__("devspace_amd.localkube.bench", fromlist=["bench_deploy"]).bench_deploy(workdir, tls=tls)
                    _log(f"quickstart deploy cold {deploy['cold_s']:.3f}s warm {deploy['warm_s']:.3f}s "
                         f"phases {deploy.get('cold_phases_ms')}")
                except Exception as e:  # reported, not fatal for the latency metric
                    _log(f"deploy benchmark failed: {e}")
            result = dev_loop(workdir, nproc, gpus, args.steps, args.warmup, tiny=args.tiny,
                              timed_start=timed_start, timed_end=timed_end, tls=tls)
        else:
            timed_start()
            timed_end()
        elapsed = clock["t1"] - clock["t0"]
        if rank == 0 and args.qs_steps > 0:
            # untimed extras (outside the barrier-bracketed region): the Node.js quickstart loop,
            # this tool's sync vs the reference's compat protocol on the same app and restart
            try:
                qs = quickstart_loop(workdir, args.qs_steps, 2, tls=tls)
                _log(f"quickstart reload p50 {_pct(qs['reload_ms'], 0.5):.2f} ms")
                qs_compat = quickstart_loop(workdir, max(1, args.ref_steps), 1, sync_mode="compat", tls=tls)
            except Exception as e:
                _log(f"quickstart loop failed: {e}")
        if rank == 0 and args.ref_steps > 0:
            try:
                ref = inner_loop(workdir, "compat", True, nproc, args.ref_steps, 1, tiny=args.tiny)
            except Exception as e:
                _log(f"reference-equivalent run failed: {e}")
        if pg is not None:
            pg.barrier()
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
        "data": "synthetic (random tokens; random-init TinyLM weights; examples/quickstart + examples/rocm-pytorch)",
        "config": {
            # what `value` measured: BASELINE.json configs[4] (rocm/pytorch pod hot-reloading a
            # train.py on MI355X); the Node.js quickstart loop is reported under "quickstart"
            "model": "examples/rocm-pytorch TinyLM (4x1024) hot-reload pod" + (" [tiny]" if args.tiny else ""),
            "app": "examples/rocm-pytorch",
            "global_batch": 8 * nproc,
            "seq_len": 512,
            "parallelism": f"dp{nproc}",
            "path": "devspace dev (exec-WebSocket sync + attach) on the bundled local cluster",
            "transport": "https + wss, mTLS" if tls else "plain http + ws",
            "builder": BUILDER_FIDELITY,
            "sync_mode": result["mode"],
        },
        # BASELINE.json's metric string (kept verbatim for the driver) ends in "quickstart"; `value`
        # is measured on the GPU pod of BASELINE configs[4], the Node.js quickstart loop is
        # reported separately under "quickstart"
        "measured": "edit -> hot-reload p50 of the examples/rocm-pytorch GPU pod (BASELINE configs[4]); "
                    "examples/quickstart: see quickstart.reload_p50_ms",
        "p50_ms": round(p50, 2),
        "p90_ms": round(_pct(result["reload_ms"], 0.9), 2),
        "sync_p50_ms": round(_pct(result["sync_ms"], 0.5), 2),
        "gpu_pod_deploy_s": round(result["pod_deploy_s"], 3),
    }
    if deploy:
        out["deploy"] = {
            "app": "examples/quickstart",
            "wall_clock_s": round(deploy["cold_s"], 3),
            "warm_wall_clock_s": round(deploy["warm_s"], 3),
            "phases_ms": deploy.get("cold_phases_ms"),
            "net": deploy.get("net"),
            # the bundled Docker daemon does not execute RUN steps and the pod runs on the host's
            # runtime: this is CLI + API-server control-plane time, not a real image build/pull
            "control_plane_only": True,
            "host_runtime_prewarmed": deploy.get("host_runtime_prewarmed"),
        }
    if qs:
        q = {"app": "examples/quickstart (node watch.js restart-on-change, as nodemon)",
             "sample": "edit index.js -> HTTP GET through devspace port-forward returns the new text",
             "reload_p50_ms": round(_pct(qs["reload_ms"], 0.5), 2),
             "reload_p90_ms": round(_pct(qs["reload_ms"], 0.9), 2),
             "sync_p50_ms": round(_pct(qs["sync_ms"], 0.5), 2),
             "n": len(qs["reload_ms"])}
        if qs_compat:
            q["compat_reload_p50_ms"] = round(_pct(qs_compat["reload_ms"], 0.5), 2)
            q["compat_sync_p50_ms"] = round(_pct(qs_compat["sync_ms"], 0.5), 2)
        out["quickstart"] = q
        if qs_compat:
            # tool-attributable comparison: the same app, restart and transport; only the sync
            # protocol differs (this tool's default vs the reference's shell scripts + timing)
            out["tool_attributable"] = {
                "sync_p50_ms": q["sync_p50_ms"],
                "reference_protocol_sync_p50_ms": q["compat_sync_p50_ms"],
                "sync_speedup": round(q["compat_sync_p50_ms"] / max(q["sync_p50_ms"], 1e-3), 1),
                "quickstart_reload_speedup": round(q["compat_reload_p50_ms"] / max(q["reload_p50_ms"], 1e-3), 1),
            }
    parts = {k: round(_pct(v, 0.5), 2) for k, v in result.get("parts", {}).items() if v}
    if parts:
        # p50 components of one reload: sync (edit -> bytes in the pod) -> pickup (runner sees
        # the change -> in-flight step drains -> code swap -> first new step done) -> log
        # delivery back to `devspace dev`; other = inotify wake-ups + scheduling slack
        parts["sync_ms"] = out["sync_p50_ms"]
        parts["other_ms"] = round(
            max(0.0, p50 - parts["sync_ms"] - parts.get("pickup_ms", 0) - parts.get("log_delivery_ms", 0)), 2)
        out["breakdown_p50"] = parts
    if ref:
        rp50 = _pct(ref["reload_ms"], 0.5)
        out["reference_equivalent"] = {
            "what": "rocm-pytorch with the reference's compat sync protocol + a cold restart of the "
                    "Python/torch workload per change (nodemon-style); dominated by interpreter + torch "
                    "start-up, so it prices the hot-reload runner more than the CLI",
            "p50_ms": round(rp50, 2),
            "sync_p50_ms": round(_pct(ref["sync_ms"], 0.5), 2),
            "speedup": round(rp50 / p50, 2) if p50 else None,
        }
    print(json.dumps(out), flush=True)
    if pg is not None:
        pg.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
