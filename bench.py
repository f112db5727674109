#!/usr/bin/env python3
"""Inner-loop benchmark: edit -> pod hot-reload latency (+ deploy wall-clock), BASELINE.json metric
"inner-loop p50 ms (edit->pod hot-reload) + deploy wall-clock s, quickstart".

Everything goes through the real `devspace` CLI against the bundled local cluster (fake
Kubernetes API server + process kubelet advertising amd.com/gpu + Docker Engine API builder,
all on this host — the GPU box has no k8s/Docker/network). The API server speaks TLS (https +
wss, client certificates) as every real cluster does (`--transport plain` for ws).

  value (timed, K steps) — BASELINE configs[0], the metric's named config: examples/quickstart
     (Node.js) under `devspace dev`, its container running `npm run dev` with cold restarts
     (WATCH_STANDBY=0: a fresh, cold node process per edit, as nodemon does in the reference's
     quickstart). One step = edit index.js locally -> synced into the pod -> node restarts -> an
     HTTP GET through devspace's port-forward returns the new text (a request sent while the app
     restarts is held by the port-forward and answered by the new server). Edits land after a
     random 0-10 ms think time. This is the tool's own loop: what it adds on top of the app's
     restart is sync + port-forward.
  standby_pool (untimed extra): the same loop with the example app's watch.js keeping pre-booted
     node standbys (its default). App-side, not the tool: reported, never the headline.
  reference_equivalent (same box): the same app and loop with the reference's behaviour: its
     sync protocol and waits (compat shell scripts, 600 ms batching, 1.3 s poll; 1 s
     pod-discovery sleeps), cold restarts as nodemon does (WATCH_STANDBY=0) and kubectl's
     port-forward (connections refused mid-restart are dropped) — BASELINE.md "How the rebuild
     will be compared" (the reference publishes no numbers: vs_baseline null).
  deploy: `devspace deploy` of the quickstart on a fresh cluster — its image build runs the
     Dockerfile's RUN steps (`npm install`) on the host runtime — then an edit of index.js deployed
     (the npm layer comes from the build cache), and a forced redeploy of the unchanged project;
     phase times and TCP/TLS counts; and the same with reference timing (1 s pod sleeps, 5 s
     rollout polls, no kept-alive connections, compat sync). Not covered: pulling a base image
     (the pod runs on the host's node runtime).
  gpu_pod — BASELINE configs[4] at amd.com/gpu: N (N = --gpus; the 8-GPU scaling run is configs[4]
     itself): examples/rocm-pytorch, a bf16 TinyLM training pod, one process per GPU under the
     hot-reload runner with an RCCL group. One sample = edit train.py -> synced -> the runner swaps
     the code at the step boundary -> first step with the new code done on every GPU -> its log
     line reaches `devspace dev`. Plus its reference-equivalent (compat sync + cold restart), and
     a fault drill at the end: an edit makes one rank fail once; the group is replaced from the
     runner's warm standby and resumes from its last rescue snapshot.
  wan: the headline loop, its reference column and the deploy with the cluster behind a shaped
     30 ms RTT / 100 Mbit/s link (devspace_amd/localkube/netem.py).
  php_mysql, microservices, kaniko — BASELINE configs[1-3]: deploy cold/warm and edit -> bytes in
     the pod(s) p50 (microservices: both services edited at once, two sync paths, two port
     forwards; kaniko: in-cluster build with the context uploaded over exec), each with the
     reference-timing + compat-protocol column.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
For N>1 the driver launches one bench rank per GPU with torch.distributed.run; rank 0 drives
the CLI (its GPU pod requests amd.com/gpu: N); the other ranks join the timing barriers.
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
BUILDER_FIDELITY = ("bundled Docker Engine API daemon: Dockerfile parsed, context hashed/tarred; "
                    "RUN steps executed on the host runtime for the deploy measurement "
                    "(deploy.run_steps_executed), recorded only (RUN steps not executed) on the "
                    "dev-loop cluster; base images not pulled; pods run on the host runtime")
TINY = (("VOCAB", 256), ("DIM", 64), ("HEADS", 4), ("LAYERS", 1), ("SEQ", 32), ("BATCH", 2))


def _pct(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


_DEADLINE = [None]  # monotonic deadline of the untimed extras (set once the headline is measured)


def _budget(timeout):
    """A wait's timeout, cut to what is left of the extras' time budget: a workload that hangs
    (e.g. a collective that never completes in an N-GPU pod) ends its extra, not the bench."""
    if _DEADLINE[0] is None:
        return timeout
    left = _DEADLINE[0] - time.monotonic()
    if left <= 0:
        raise TimeoutError("extras time budget spent (--extras-budget-s)")
    return min(timeout, left)


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


def dev_loop(workdir, nproc, gpus, steps, warmup, tiny=False, timed_start=None, timed_end=None, tls=True, wan=None):
    """`devspace deploy` + `devspace dev` of examples/rocm-pytorch on the local cluster.
    wan=(rtt_ms, mbit): the API server behind a shaped link (the fault drill is skipped)."""
    from devspace_amd.localkube import LocalCluster
    from devspace_amd.localkube.bench import devspace_env, run_devspace

    base = os.path.join(workdir, "dev-bench" + ("-wan" if wan else ""))
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
    dev = link = None
    try:
        env = devspace_env(cluster, base)
        if wan:  # a laptop editing train.py for a pod on a remote MI355X node
            from devspace_amd.localkube.netem import ShapedLink, point_kubeconfig

            link = ShapedLink(("127.0.0.1", cluster.port), rtt_ms=wan[0], mbit=wan[1]).start()
            point_kubeconfig(env["KUBECONFIG"], cluster.server, link.url("https" if tls else "http"))
        env["DEVSPACE_NPROC"] = str(nproc)  # used when the pod requests no GPU (CPU smoke)
        cluster.kubelet.extra_env["DEVSPACE_NPROC"] = str(nproc)
        if os.environ.get("DEVSPACE_DIST_BACKEND"):  # rehearsal: N ranks sharing fewer GPUs (gloo)
            cluster.kubelet.extra_env["DEVSPACE_DIST_BACKEND"] = os.environ["DEVSPACE_DIST_BACKEND"]
        # the fault drill at the end resumes from a snapshot: take them every 10 s
        cluster.kubelet.extra_env["DEVSPACE_RESCUE_EVERY_S"] = "10"
        # `devspace dev` builds (dev image cache), deploys the chart, waits for the rollout,
        # then starts sync + attach on the newest running pod.
        t_dev = time.perf_counter()
        dev = subprocess.Popen([os.path.join(ROOT, "bin", "devspace"), "dev", "--terminal=false",
                                "--portforwarding=false"], cwd=proj, env=env, stdout=subprocess.PIPE,
                               stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, start_new_session=True)
        tail = LineTail(dev.stdout, echo_prefix="[dev] ")
        _, line, idx = tail.wait_for(r"Sync started on", timeout=_budget(900))
        deploy_s = time.perf_counter() - t_dev
        ns, pod_name = re.search(r"Pod: ([^/\s]+)/([^)\s]+)", line).groups()
        pod = cluster.store.get("", "pods", ns, pod_name)
        cname = pod["spec"]["containers"][0]["name"]
        root = json.loads(pod["metadata"]["annotations"]["devspace.sh/local-roots"])[cname]
        _log(f"dev: pod {pod_name} synced after {deploy_s:.2f}s")
        _, _, idx = tail.wait_for(r"Attached to container", start_index=idx, timeout=_budget(120))
        _wait_file_contains(root + ".log", "[devspace-runner] started gen=", timeout=_budget(900), interval=0.05)
        # `devspace dev` start -> image built, chart deployed, pod running, every rank through
        # import torch, model setup and its first training step on the GPU
        first_step_s = time.perf_counter() - t_dev
        pod_log = open(root + ".log").read()
        m = re.search(r"\[devspace-runner\] started gen=\d+ .*?world=(\d+) device=(\S+)", pod_log)
        pod_world = int(m.group(1)) if m else 0
        fm = re.search(r"\[devspace-runner\] fused=(.*)", pod_log)
        fused = fm.group(1).strip() if fm else "unknown"
        _log(f"pod training ops: fused={fused}")
        _log(f"runner up: {pod_world} rank(s), rank 0 on {m.group(2) if m else '?'}")
        if pod_world != nproc:
            raise RuntimeError(f"the pod runs {pod_world} training rank(s), expected {nproc}")
        mode = os.environ.get("DEVSPACE_SYNC_MODE") or (
            "helper" if os.path.exists(os.path.join(ROOT, "bin", "devspace-helper")) else "fast")
        pod_file = os.path.join(root, "app", "train.py")
        samples, sync_samples, agreed = [], [], []
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
            t1, line, idx = tail.wait_for(pat, start_index=idx, timeout=_budget(600))
            # the runner prints ranks=<world> once every rank confirmed one code digest
            rm = re.search(r" ranks=(\d+) ", line)
            if rm:
                agreed.append(int(rm.group(1)))
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
        out = {"reload_ms": samples, "sync_ms": sync_samples, "mode": mode, "pod_deploy_s": deploy_s,
               "parts": parts, "fused": fused, "world": pod_world, "first_step_s": first_step_s,
               "ranks_agreed": bool(agreed) and all(a == pod_world for a in agreed)}
        if pod_world >= 1 and not wan:
            try:
                out["fault_drill"] = _fault_drill(train, tail, idx, pod_world)
            except Exception as e:  # reported with the loop's numbers, which stand on their own
                out["fault_drill"] = {"error": str(e)[-500:]}
        return out
    finally:
        _killpg(dev)
        if link is not None:
            link.stop()
        cluster.stop()


def _fault_drill(train, tail, idx, world):
    """The pod's failure path, once: an edit makes one rank fail in its next step (once: a flag
    file marks it done) — rank 1 raises with several ranks (the group must be stopped), the only
    rank crashes outright with one (an exception would just pause it) — so the group is replaced
    (from the warm standby), resumes from its latest rescue snapshot and trains the edited code."""
    import uuid

    rank = 1 if world > 1 else 0
    fail = "raise RuntimeError('bench fault drill')" if world > 1 else "os._exit(1)  # a hard crash"

    flag = os.path.join(tempfile.gettempdir(), f"devspace-bench-drill-{uuid.uuid4().hex[:8]}")
    src = open(train).read()
    src = re.sub(r'^MARKER = ".*"$', 'MARKER = "drill"', src, count=1, flags=re.M)
    src += (f"\n\n_drill_step = step\n\n\ndef step(ctx, state):  # bench fault drill\n"
            f"    import os\n    if ctx.rank == {rank} and not os.path.exists({flag!r}):\n"
            f"        open({flag!r}, 'w').close()\n        {fail}\n"
            f"    return _drill_step(ctx, state)\n")
    # a snapshot to resume from (every 10 s in the drill's pod), and the standby warm by then
    if not any("rescue snapshot step=" in l for _, l in tail.lines):
        _, _, idx = tail.wait_for(r"\[devspace-runner\] rescue snapshot step=", start_index=idx, timeout=_budget(60))
    t0 = time.perf_counter()
    with open(train, "w") as f:
        f.write(src)
    t_fail, line, idx = tail.wait_for(rf"\[devspace-runner\] rank={rank} exited with code \d+: restarting the group",
                                      start_index=idx, timeout=_budget(300))
    standby = "from the warm standby" in line
    t_up, line, idx = tail.wait_for(r"\[devspace-runner\] started gen=\d+ marker=drill ", start_index=idx,
                                    timeout=_budget(300))
    restored = [l for _, l in tail.lines[-200:] if "restored step=" in l]
    m = re.search(r"restored step=(\d+)", restored[-1]) if restored else None
    try:
        os.unlink(flag)
    except OSError:
        pass
    return {"ranks": world, "failure": "exception on rank 1" if world > 1 else "hard crash (os._exit) of the only rank",
            "recovered": True, "warm_standby": standby, "resumed_from_step": int(m.group(1)) if m else None,
            "edit_to_failure_s": round(t_fail - t0, 3), "failure_to_training_s": round(t_up - t_fail, 3)}


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


WAN = (30, 100)  # rtt ms, Mbit/s: the WAN extra's link

QS_GREETING = re.compile(r"res\.end\('[^']*' \+")


def _qs_edit(path, marker):
    src = open(path).read()
    src, n = QS_GREETING.subn(f"res.end('Hello [{marker}] from ' +", src, count=1)
    assert n == 1, "examples/quickstart/index.js greeting line not found"
    with open(path, "w") as f:
        f.write(src)


def _pf_spans(trace_path, windows):
    """The devspace port-forward's streams during the timed samples (trace.jsonl
    `portforward.stream` spans: one per attempt; an attempt the restarting app refused is retried
    on a new stream): how they went over the link, per edit."""
    spans = []
    try:
        with open(trace_path) as f:
            for line in f:
                if '"portforward.stream"' not in line:
                    continue
                sp = json.loads(line)
                t = sp.get("start_us", 0) / 1e6
                if any(a <= t <= b for a, b in windows):
                    spans.append(sp)
    except OSError:
        return None
    if not spans:
        return None
    n = max(1, len(windows))
    replies = [sp for sp in spans if sp.get("outcome") == "reply"]

    def ms(key, rows):
        v = [int(sp[key]) / 1000.0 for sp in rows if int(sp.get(key, -1)) >= 0]
        return round(_pct(v, 0.5), 2) if v else None

    return {"via": sorted({sp.get("via", "websocket") for sp in spans}),
            "streams_per_edit": round(len(spans) / n, 2),
            "refused_per_edit": round(sum(sp.get("outcome") == "refused" for sp in spans) / n, 2),
            # attempts of held GETs sent while earlier ones were in flight (the app may see those)
            "hedged_per_edit": round(sum(sp.get("hedged") == "1" for sp in spans) / n, 2),
            "open_ms_p50": ms("open_us", spans), "reply_first_byte_ms_p50": ms("first_us", replies)}


def _app_requests_per_edit(req_log, marks):
    """Requests the restarted server of each timed edit served: the server that answered the
    edit's GET is the last one in that edit's slice of the app's request log, and every line of
    its pid in the slice is one delivery of that GET (the bench sends no other request to it).
    1.0 = each request reached the app once."""
    try:
        data = open(req_log, "rb").read()
    except OSError:
        return None
    counts = []
    for k, start in enumerate(marks):
        end = marks[k + 1] if k + 1 < len(marks) else len(data)
        rows = [l.split(b" ", 1)[0] for l in data[start:end].splitlines() if l.strip()]
        if rows:
            counts.append(sum(1 for r in rows if r == rows[-1]))
    return counts


def quickstart_loop(workdir, steps, warmup, sync_mode=None, tls=True, reference=False, timed_start=None,
                    timed_end=None, cold=None, wan=None):
    """examples/quickstart edit -> reload, the way its README runs the dev loop: `devspace dev`
    (sync + port-forward) with the container running `npm run dev` (watch.js restarts node on
    change, as nodemon does in the reference's quickstart). One sample = edit index.js locally ->
    HTTP GET through devspace's port-forward returns the new greeting. CPU-only pod."""
    import yaml

    from devspace_amd.localkube import LocalCluster
    from devspace_amd.localkube.bench import devspace_env

    cold = reference if cold is None else cold  # cold restarts: nodemon's (no standby pool)
    tag = ("ref-" if reference else "") + ("cold-" if cold and not reference else "") + (sync_mode or "default")
    tag += "-wan" if wan else ""
    base = os.path.join(workdir, f"qs-bench-{tag}")
    proj = os.path.join(base, "quickstart")
    shutil.copytree(os.path.join(ROOT, "examples", "quickstart"), proj, symlinks=True)
    remote, local = _free_port(), _free_port()
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["dev"]["overrideImages"][0]["entrypoint"] = ["node", "watch.js", "index.js"]
    cfg["dev"]["ports"][0]["portMappings"] = [{"localPort": local, "remotePort": remote}]
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    # app-side request log (pid + request line per request the app serves): how many copies of
    # the held GET of each edit reached the restarted server
    req_log = os.path.join(base, "app-requests.log")
    index_src = open(os.path.join(proj, "index.js")).read()
    hook = "http.createServer((req, res) => {"
    assert hook in index_src, "examples/quickstart/index.js request handler not found"
    open(os.path.join(proj, "index.js"), "w").write(index_src.replace(
        hook, hook + "\n  if (process.env.REQUEST_LOG) require('fs').appendFileSync(process.env.REQUEST_LOG, "
        "process.pid + ' ' + req.method + ' ' + req.url + '\\n');", 1))
    values = os.path.join(proj, "chart", "values.yaml")
    v = yaml.safe_load(open(values))
    v["components"][0]["containers"][0]["env"] = [{"name": "PORT", "value": str(remote)},
                                                  {"name": "REQUEST_LOG", "value": req_log}]
    if cold:  # nodemon's cold restarts
        v["components"][0]["containers"][0]["env"].append({"name": "WATCH_STANDBY", "value": "0"})
    open(values, "w").write(yaml.safe_dump(v))

    cluster = LocalCluster(os.path.join(base, "cluster"), gpus=0, tls=tls).start()
    dev = link = None
    try:
        env = devspace_env(cluster, base)
        if wan:  # the cluster behind a WAN link: every API request, exec and forward pays it
            from devspace_amd.localkube.netem import ShapedLink, point_kubeconfig

            link = ShapedLink(("127.0.0.1", cluster.port), rtt_ms=wan[0], mbit=wan[1]).start()
            point_kubeconfig(env["KUBECONFIG"], cluster.server, link.url("https" if tls else "http"))
        if sync_mode:
            env["DEVSPACE_SYNC_MODE"] = sync_mode
        if reference:
            env["DEVSPACE_REFERENCE_TIMING"] = "1"
        t_dev = time.perf_counter()
        dev = subprocess.Popen([os.path.join(ROOT, "bin", "devspace"), "dev", "--terminal=false"], cwd=proj, env=env,
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                               start_new_session=True)
        tail = LineTail(dev.stdout, echo_prefix=f"[qs-{tag}] ")
        _, line, idx = tail.wait_for(r"Sync started on", timeout=_budget(300))
        ns, pod_name = re.search(r"Pod: ([^/\s]+)/([^)\s]+)", line).groups()
        pod = cluster.store.get("", "pods", ns, pod_name)
        cname = pod["spec"]["containers"][0]["name"]
        root = json.loads(pod["metadata"]["annotations"]["devspace.sh/local-roots"])[cname]
        deadline = time.monotonic() + 60
        while not (_http_get(local) or "").startswith("Hello"):
            if time.monotonic() > deadline:
                raise TimeoutError("quickstart server never answered through the port-forward")
            time.sleep(0.01)
        # `devspace dev` start -> build, deploy, pod running, sync + port-forward up -> the app
        # answers through the forward (the first iteration of the loop)
        dev_start_s = time.perf_counter() - t_dev
        index, pod_index = os.path.join(proj, "index.js"), os.path.join(root, "app", "index.js")
        samples, sync_samples, conns, windows, log_marks = [], [], [], [], []
        rng = random.Random(4321)
        for i in range(warmup + steps):
            if i == warmup and timed_start:
                timed_start()
            marker = f"q{i}" + ("_" * (i % 2))  # compat mode compares size + mtime (s)
            time.sleep(rng.uniform(0.0, EDIT_JITTER_S))
            c0 = link.connections if link is not None else 0
            if i >= warmup:
                log_marks.append(os.path.getsize(req_log) if os.path.exists(req_log) else 0)
            w0 = time.monotonic()  # (trace spans carry CLOCK_MONOTONIC microseconds)
            t0 = time.perf_counter()
            _qs_edit(index, marker)
            t_sync = _wait_file_contains(pod_index, f"[{marker}]", timeout=_budget(60))
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
                conns.append((link.connections if link is not None else 0) - c0)
                windows.append((w0, time.monotonic()))
        if timed_end:
            timed_end()
        time.sleep(0.2)  # a late copy of the last edit's request would land now
        out = {"reload_ms": samples, "sync_ms": sync_samples, "dev_start_s": dev_start_s,
               "app_requests": _app_requests_per_edit(req_log, log_marks)}
        if link is not None:
            out["link"] = {"connections": link.connections, "per_edit": conns}
            out["portforward"] = _pf_spans(os.path.join(proj, ".devspace", "logs", "trace.jsonl"), windows)
        return out
    finally:
        _killpg(dev)
        if link is not None:
            link.stop()
        cluster.stop()


# ---------------------------------------------------------------------------- BASELINE configs[1-3]


def _yaml_edit(path, fn):
    import yaml

    with open(path) as f:
        v = yaml.safe_load(f)
    fn(v)
    with open(path, "w") as f:
        f.write(yaml.safe_dump(v, sort_keys=False))


def _prep_php_mysql(proj):
    """php + mysql in one StatefulSet pod with a PVC. The offline local registry has no mysql:8
    or php/apache runtime: mysql becomes a `sleep` stand-in (the pod shape, volume and two
    containers stay) and the php container idles under `devspace dev` (overrideImages)."""
    def values(v):
        for c in v["components"][0]["containers"]:
            if c.get("name") == "mysql":
                c["image"] = "busybox"
            c["command"] = ["sleep", "999999999"]  # php: apache's place (no php runtime here)
    _yaml_edit(os.path.join(proj, "chart", "values.yaml"), values)

    def cfg(c):
        c.setdefault("dev", {})["overrideImages"] = [{"name": "default", "entrypoint": ["sleep", "999999999999"]}]
        c["dev"]["ports"][0]["portMappings"][0]["localPort"] = _free_port()
    _yaml_edit(os.path.join(proj, ".devspace", "config.yaml"), cfg)
    return [("index.php", {"app.kubernetes.io/component": "default"}, "var/www/html/index.php")]


def _prep_microservices(proj):
    """Two services (node via kubectl manifests, php via helm), two sync paths and two port
    forwards in one `devspace dev`; both containers idle (overrideImages), as the node one does
    in the example's own config."""
    def cfg(c):
        c["dev"]["overrideImages"] = [{"name": "node", "entrypoint": ["sleep", "999999999999"]},
                                      {"name": "php", "entrypoint": ["sleep", "999999999999"]}]
        for pf in c["dev"]["ports"]:
            pf["portMappings"][0]["localPort"] = _free_port()
    _yaml_edit(os.path.join(proj, ".devspace", "config.yaml"), cfg)
    # `deploy` runs the image's own command and there is no php/apache runtime on the host: a
    # sleep stand-in keeps the pod running, so the helm rollout wait (`wait`, default true, as in
    # the reference: deploy/helm/deploy.go:163-166) completes in both columns
    with open(os.path.join(proj, "php", "Dockerfile"), "a") as f:
        f.write('CMD ["sleep", "999999999"]\n')
    return [("node/index.js", {"release": "devspace-node"}, "app/index.js"),
            ("php/index.php", {"release": "devspace-php"}, "var/www/html/index.php")]


def _prep_kaniko(proj):
    def cfg(c):
        c["dev"]["ports"][0]["portMappings"][0]["localPort"] = _free_port()
    _yaml_edit(os.path.join(proj, ".devspace", "config.yaml"), cfg)
    return [("app.py", {"app.kubernetes.io/component": "default"}, "app/app.py")]


EXAMPLES = {"php_mysql": ("php-mysql-example", _prep_php_mysql, "php-mysql"),
            "microservices": ("microservices", _prep_microservices, "microservices"),
            "kaniko": ("kaniko", _prep_kaniko, "kaniko")}
EXAMPLE_NOTES = {
    "php_mysql": "BASELINE configs[1]: StatefulSet with a PVC and two containers; mysql:8 is a sleep stand-in "
                 "(not in the offline registry), the php container idles under dev (no php runtime on the host)",
    "microservices": "BASELINE configs[2]: two deployments (kubectl + helm), two sync paths edited at once, two "
                     "port forwards; sample = both edits in their pods; the php image runs a sleep stand-in for "
                     "apache (no php runtime on the host), so the helm rollout wait (on, as in the reference) "
                     "completes in both columns",
    "kaniko": "BASELINE configs[3]: no Docker daemon; the image builds in an in-cluster kaniko pod (emulated "
              "executor) with the context uploaded over exec",
}


def _pod_root(cluster, ns, labels):
    sel = ",".join(f"{k}={v}" for k, v in labels.items())
    for p in cluster.store.list("", "pods", ns, sel):
        if (p.get("status") or {}).get("phase") == "Running" and not p["metadata"].get("deletionTimestamp"):
            roots = json.loads(p["metadata"]["annotations"]["devspace.sh/local-roots"])
            return next(iter(roots.values()))
    return None


def example_loop(workdir, key, steps, warmup, tls=True, reference=False):
    """`devspace deploy` (cold, then forced warm) + `devspace dev` of one BASELINE example; one
    sample = edit every synced file -> all edits in their pods (through the exec WebSocket).
    reference=True: the reference's sync protocol and waits (DEVSPACE_SYNC_MODE=compat,
    DEVSPACE_REFERENCE_TIMING=1)."""
    from devspace_amd.localkube import LocalCluster
    from devspace_amd.localkube.bench import _phases, devspace_env, run_devspace

    example, prep, ns = EXAMPLES[key]
    tag = key + ("-ref" if reference else "")
    base = os.path.join(workdir, f"ex-{tag}")
    proj = os.path.join(base, example)
    shutil.copytree(os.path.join(ROOT, "examples", example), proj, symlinks=True)
    edits = prep(proj)
    cluster = LocalCluster(os.path.join(base, "cluster"), gpus=0, tls=tls).start()
    dev = None
    try:
        env = devspace_env(cluster, base)
        if reference:
            env.update(DEVSPACE_SYNC_MODE="compat", DEVSPACE_REFERENCE_TIMING="1")
        if key == "kaniko":
            env.pop("DOCKER_HOST", None)  # no local daemon: images build in-cluster
        trace = os.path.join(proj, ".devspace", "logs", "trace.jsonl")
        cold, out = run_devspace(["deploy"], proj, env, timeout=600)
        phases, net = _phases(trace)
        warm, _ = run_devspace(["deploy", "-d"], proj, env, timeout=600)
        dev = subprocess.Popen([os.path.join(ROOT, "bin", "devspace"), "dev", "--terminal=false"], cwd=proj, env=env,
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                               start_new_session=True)
        tail = LineTail(dev.stdout, echo_prefix=f"[{tag}] ")
        t_dev = time.perf_counter()
        idx = 0
        for _ in edits:
            _, _, idx = tail.wait_for(r"Sync started on", start_index=idx, timeout=_budget(600))
        dev_ready_s = time.perf_counter() - t_dev
        with tail.cv:
            forwards = sum(1 for _, l in tail.lines if "Port forwarding started" in l)
        targets = []
        for local, labels, in_pod in edits:
            root = None
            deadline = time.monotonic() + 60
            while root is None and time.monotonic() < deadline:
                root = _pod_root(cluster, ns, labels)
                time.sleep(0.05)
            if root is None:
                raise RuntimeError(f"{key}: no running pod for {labels}")
            targets.append((os.path.join(proj, local), os.path.join(root, in_pod)))
        samples = []
        rng = random.Random(99)
        for i in range(warmup + steps):
            marker = f"m{i}" + ("_" * (i % 2))
            time.sleep(rng.uniform(0.0, EDIT_JITTER_S))
            t0 = time.perf_counter()
            for local, _ in targets:
                with open(local, "a") as f:
                    f.write(f"\n// edit {marker}\n" if not local.endswith(".py") else f"\n# edit {marker}\n")
            t_last = max(_wait_file_contains(pod_file, f"edit {marker}", timeout=_budget(120)) for _, pod_file in targets)
            if i >= warmup:
                samples.append((t_last - t0) * 1000.0)
        _killpg(dev)
        dev = None
        run_devspace(["purge"], proj, env, timeout=300)
        return {"deploy_cold_s": round(cold, 3), "deploy_warm_s": round(warm, 3), "deploy_phases_ms": phases,
                "net": net, "dev_ready_s": round(dev_ready_s, 3), "sync_paths": len(edits),
                "port_forwards": forwards, "edit_to_pod_p50_ms": round(_pct(samples, 0.5), 2),
                "edit_to_pod_p90_ms": round(_pct(samples, 0.9), 2), "n": len(samples)}
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
        _, _, idx = tail.wait_for(r"\[devspace-runner\] started gen=\d+ marker=v0", timeout=_budget(600))
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
            t1, _, idx = tail.wait_for(pat, start_index=idx, timeout=_budget(600))
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
    ap.add_argument("--ref-steps", type=int, default=3, help="samples of every reference-equivalent column (0=skip)")
    ap.add_argument("--gpu-steps", type=int, default=20, help="edit -> reload samples of the GPU pod (0=skip)")
    ap.add_argument("--example-steps", type=int, default=5,
                    help="samples per BASELINE example (php-mysql, microservices, kaniko; 0=skip)")
    ap.add_argument("--no-deploy-bench", action="store_true", help="skip the quickstart deploy wall-clock")
    ap.add_argument("--tiny", action="store_true", help="tiny GPU-pod model (CPU smoke only)")
    ap.add_argument("--extras-budget-s", type=float, default=600.0,
                    help="wall-clock budget of all untimed extras together (each wait is cut to what is left)")
    ap.add_argument("--transport", choices=("tls", "plain"), default="tls",
                    help="API server transport of the local cluster (tls = https + wss with mTLS, as a real cluster)")
    args = ap.parse_args()
    # the `devspace` processes this bench starts end with it, however it ends
    os.environ["DEVSPACE_PARENT_PID"] = str(os.getpid())

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
    qs, extras = None, {}
    clock = {}

    def timed_start():
        barrier_sync()
        clock["t0"] = time.perf_counter()

    def timed_end():
        barrier_sync()
        clock["t1"] = time.perf_counter()

    def extra(name, fn):
        try:
            if os.environ.get("DEVSPACE_BENCH_FAIL_EXTRA") == name:  # test hook (tests/test_bench.py)
                raise RuntimeError(f"forced failure of {name} (DEVSPACE_BENCH_FAIL_EXTRA)")
            extras[name] = fn()
        except Exception as e:  # reported, not fatal for the headline metric
            _log(f"{name} failed: {e}")
            extras[name] = {"error": str(e)[-500:]}

    try:
        if rank == 0:
            from devspace_amd.localkube.bench import bench_deploy

            if not args.no_deploy_bench:
                extra("deploy", lambda: bench_deploy(workdir, tls=tls))
                if args.ref_steps > 0:
                    extra("deploy_ref", lambda: bench_deploy(workdir, tls=tls, reference=True))
            # the headline: BASELINE configs[0] with cold (nodemon-style) restarts, timed
            # between barriers: the tool's own loop, not the example app's standby pool
            qs = quickstart_loop(workdir, args.steps, args.warmup, tls=tls, timed_start=timed_start,
                                 timed_end=timed_end, cold=True)
            _log(f"quickstart reload p50 (cold restarts) {_pct(qs['reload_ms'], 0.5):.2f} ms")
        else:
            timed_start()
            timed_end()
        elapsed = clock["t1"] - clock["t0"]
        if rank == 0:
            # untimed extras (outside the barrier-bracketed region), within one time budget
            t_extras = time.monotonic()
            _DEADLINE[0] = t_extras + args.extras_budget_s
            if args.ref_steps > 0:
                # the example app's own standby pool (watch.js default): app-side, reported apart
                extra("qs_pool", lambda: quickstart_loop(workdir, max(args.ref_steps, 10), 1, tls=tls, cold=False))
                extra("qs_ref", lambda: quickstart_loop(workdir, args.ref_steps, 1, sync_mode="compat", tls=tls,
                                                        reference=True))
                # the same loops with the cluster 30 ms / 100 Mbit/s away (a laptop and a cloud
                # cluster): round trips per edit and per connection, not loopback, decide here
                extra("qs_wan", lambda: quickstart_loop(workdir, max(args.ref_steps, 10), 1, tls=tls, cold=True, wan=WAN))
                extra("qs_wan_ref", lambda: quickstart_loop(workdir, args.ref_steps, 1, sync_mode="compat", tls=tls,
                                                            reference=True, wan=WAN))
                if not args.no_deploy_bench:
                    from devspace_amd.localkube.bench import bench_deploy

                    extra("deploy_wan", lambda: bench_deploy(workdir, tls=tls, wan=WAN))
                    extra("deploy_wan_ref", lambda: bench_deploy(workdir, tls=tls, reference=True, wan=WAN))
            if args.gpu_steps > 0:
                extra("gpu_pod", lambda: dev_loop(workdir, nproc, gpus, args.gpu_steps, 3, tiny=args.tiny, tls=tls))
                if args.ref_steps > 0:  # the same loop with the cluster 30 ms away
                    extra("gpu_pod_wan", lambda: dev_loop(workdir, nproc, gpus, 10, 2, tiny=args.tiny, tls=tls,
                                                          wan=WAN))
                if args.ref_steps > 0:
                    extra("gpu_pod_ref", lambda: inner_loop(workdir, "compat", True, nproc, args.ref_steps, 1,
                                                            tiny=args.tiny))
            if args.example_steps > 0:
                for key in EXAMPLES:
                    extra(key, lambda key=key: example_loop(workdir, key, args.example_steps, 1, tls=tls))
                    if args.ref_steps > 0:
                        extra(key + "_ref", lambda key=key: example_loop(workdir, key, args.ref_steps, 1, tls=tls,
                                                                        reference=True))
            _log(f"extras took {time.monotonic() - t_extras:.1f}s")
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
    print(json.dumps(report(args, nproc, tls, ms_total, qs, extras)), flush=True)
    if pg is not None:
        pg.destroy_process_group()
    return 0


def _mean(xs):
    return round(sum(xs) / len(xs), 2) if xs else None


def _ok(x):
    return isinstance(x, dict) and "error" not in x


def report(args, nproc, tls, ms_total, qs, extras):
    p50 = _pct(qs["reload_ms"], 0.5)
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
        "vs_baseline": None,  # the reference publishes no numbers; see reference_equivalent
        "dtype": None,  # a CLI loop: no tensor math in the headline (the GPU pod extra trains in bf16)
        "data": "synthetic edits of the examples' sources (no dataset); GPU pod: random tokens, random-init TinyLM",
        "config": {
            # BASELINE.json metric + configs[0]: examples/quickstart, edit -> pod hot-reload
            "model": "examples/quickstart (Node.js hello-world) dev loop",
            "app": "examples/quickstart",
            "global_batch": None,  # a CLI benchmark: one edit per step, no batch
            "seq_len": None,
            "parallelism": f"none (CLI); GPU pod extra: dp{nproc}",
            "sample": "edit index.js -> synced into the pod -> node restarts cold (npm run dev with "
                      "WATCH_STANDBY=0: a fresh node process per edit, as nodemon) -> "
                      "HTTP GET through devspace's port-forward returns the new text",
            "restart": "cold",
            "path": "devspace dev (exec-WebSocket sync + port-forward) on the bundled local cluster",
            "transport": "https + wss, mTLS" if tls else "plain http + ws",
            "builder": BUILDER_FIDELITY,
        },
        "p50_ms": round(p50, 2),
        "p90_ms": round(_pct(qs["reload_ms"], 0.9), 2),
        "sync_p50_ms": round(_pct(qs["sync_ms"], 0.5), 2),
        # untimed: `devspace dev` on a fresh cluster until the app answers through the forward
        "dev_start_s": round(qs["dev_start_s"], 3),
        "app_requests_per_edit": _mean(qs.get("app_requests")),
    }
    ref = extras.get("qs_ref")
    if _ok(ref):
        rp50 = _pct(ref["reload_ms"], 0.5)
        out["reference_equivalent"] = {
            "what": "the same quickstart app and loop with the reference's sync protocol (compat shell scripts, "
                    "600 ms batching, 1.3 s poll), waits (1 s pod-discovery sleeps), cold nodemon-style restarts "
                    "and kubectl's port-forward (no hold): BASELINE.md's same-box column",
            "p50_ms": round(rp50, 2),
            "sync_p50_ms": round(_pct(ref["sync_ms"], 0.5), 2),
            "n": len(ref["reload_ms"]),
            "speedup": round(rp50 / p50, 2) if p50 else None,
            "sync_speedup": round(_pct(ref["sync_ms"], 0.5) / max(out["sync_p50_ms"], 1e-3), 1),
            "dev_start_s": round(ref["dev_start_s"], 3),
        }
    wan, wan_ref = extras.get("qs_wan"), extras.get("qs_wan_ref")
    if _ok(wan):
        wp50 = _pct(wan["reload_ms"], 0.5)
        out["wan"] = {
            "what": f"the headline loop (cold restarts) with the cluster behind a shaped link of {WAN[0]} ms RTT and "
                    f"{WAN[1]} Mbit/s each way (devspace_amd/localkube/netem.py): API requests, exec sync and the "
                    f"port-forward all cross it",
            "rtt_ms": WAN[0], "mbit": WAN[1],
            "p50_ms": round(wp50, 2), "p90_ms": round(_pct(wan["reload_ms"], 0.9), 2),
            "sync_p50_ms": round(_pct(wan["sync_ms"], 0.5), 2), "n": len(wan["reload_ms"]),
            # copies of each edit's GET that reached the restarted app (1.0: delivered once)
            "app_requests_per_edit": _mean(wan.get("app_requests")),
            "dev_start_s": round(wan["dev_start_s"], 3), "link_connections": wan.get("link", {}).get("connections"),
            "connections_per_edit": round(sum(wan["link"]["per_edit"]) / max(1, len(wan["link"]["per_edit"])), 2)
            if wan.get("link", {}).get("per_edit") else None,
            # where a sample's time goes: the edit reaching the pod, then the app's restart plus the
            # request through the port-forward (its streams below)
            "breakdown_p50_ms": {"sync": round(_pct(wan["sync_ms"], 0.5), 2),
                                 "restart_and_request": round(_pct([r - s for r, s in zip(wan["reload_ms"],
                                                                                          wan["sync_ms"])], 0.5), 2)},
            "portforward": wan.get("portforward"),
        }
        dw, dwr = extras.get("deploy_wan"), extras.get("deploy_wan_ref")
        if _ok(dw):
            out["wan"]["deploy"] = {"wall_clock_s": round(dw["cold_s"], 3), "warm_wall_clock_s": round(dw["warm_s"], 3),
                                    "net": dw.get("net")}
            if _ok(dwr):
                out["wan"]["deploy"]["reference_equivalent"] = {
                    "wall_clock_s": round(dwr["cold_s"], 3), "warm_wall_clock_s": round(dwr["warm_s"], 3),
                    "net": dwr.get("net"), "speedup": round(dwr["cold_s"] / max(dw["cold_s"], 1e-3), 1)}
        if _ok(wan_ref):
            wr50 = _pct(wan_ref["reload_ms"], 0.5)
            out["wan"]["reference_equivalent"] = {
                "p50_ms": round(wr50, 2), "sync_p50_ms": round(_pct(wan_ref["sync_ms"], 0.5), 2),
                "n": len(wan_ref["reload_ms"]), "dev_start_s": round(wan_ref["dev_start_s"], 3),
                "link_connections": wan_ref.get("link", {}).get("connections"),
                "connections_per_edit": round(sum(wan_ref["link"]["per_edit"]) / max(1, len(wan_ref["link"]["per_edit"])), 2)
                if wan_ref.get("link", {}).get("per_edit") else None,
                "speedup": round(wr50 / wp50, 2) if wp50 else None,
            }
    pool = extras.get("qs_pool")
    if _ok(pool):
        pp50 = _pct(pool["reload_ms"], 0.5)
        out["standby_pool"] = {
            "what": "the same loop with the example app's watch.js keeping pre-booted node standbys (its default, "
                    "WATCH_STANDBY=4): app-side, not the tool's; never the headline",
            "p50_ms": round(pp50, 2), "p90_ms": round(_pct(pool["reload_ms"], 0.9), 2),
            "sync_p50_ms": round(_pct(pool["sync_ms"], 0.5), 2), "n": len(pool["reload_ms"]),
        }
    dep, dep_ref = extras.get("deploy"), extras.get("deploy_ref")
    if _ok(dep):
        out["deploy"] = {
            "app": "examples/quickstart",
            "wall_clock_s": round(dep["cold_s"], 3),
            "edit_redeploy_s": round(dep["edit_s"], 3) if dep.get("edit_s") else None,
            "warm_wall_clock_s": round(dep["warm_s"], 3),
            "phases_ms": dep.get("cold_phases_ms"),
            "edit_phases_ms": dep.get("edit_phases_ms"),
            "net": dep.get("net"),
            # the image build executes the Dockerfile's RUN steps (npm install) on the host runtime;
            # the base image is not pulled (the pod runs on the host's node runtime)
            "control_plane_only": not dep.get("run_steps", False),
            "run_steps_executed": bool(dep.get("run_steps")),
            "base_image_pulled": False,
            "host_runtime_prewarmed": dep.get("host_runtime_prewarmed"),
        }
        if _ok(dep_ref):
            out["deploy"]["reference_equivalent"] = {
                "what": "same deploy with the reference's waits: 1 s pod sleeps, 5 s rollout polls, no kept-alive "
                        "connections (DEVSPACE_REFERENCE_TIMING)",
                "wall_clock_s": round(dep_ref["cold_s"], 3),
                "edit_redeploy_s": round(dep_ref["edit_s"], 3) if dep_ref.get("edit_s") else None,
                "warm_wall_clock_s": round(dep_ref["warm_s"], 3),
                "net": dep_ref.get("net"),
                "speedup": round(dep_ref["cold_s"] / max(dep["cold_s"], 1e-3), 1),
            }
    gp = extras.get("gpu_pod")
    if _ok(gp):
        gp50 = _pct(gp["reload_ms"], 0.5)
        g = {"config": f"examples/rocm-pytorch TinyLM (4x1024) training pod, amd.com/gpu: {nproc} (BASELINE "
                       f"configs[4] at {nproc} GPU(s); configs[4] itself at 8)" + (" [tiny]" if args.tiny else ""),
             "global_batch": 8 * nproc, "seq_len": 512, "parallelism": f"dp{nproc}", "dtype": "bf16",
             "fused_ops": gp.get("fused"), "sync_mode": gp.get("mode"), "ranks": gp.get("world"),
             "ranks_agreed_on_code": gp.get("ranks_agreed"),
             "reload_p50_ms": round(gp50, 2), "reload_p90_ms": round(_pct(gp["reload_ms"], 0.9), 2),
             "sync_p50_ms": round(_pct(gp["sync_ms"], 0.5), 2), "n": len(gp["reload_ms"]),
             "pod_deploy_s": round(gp["pod_deploy_s"], 3),
             "dev_to_first_step_s": round(gp["first_step_s"], 3) if gp.get("first_step_s") else None}
        if gp.get("fault_drill"):
            g["fault_drill"] = dict(gp["fault_drill"], what="an edit makes one rank fail once: the group is stopped, "
                                                          "replaced and resumes from its last rescue snapshot")
        parts = {k: round(_pct(v, 0.5), 2) for k, v in gp.get("parts", {}).items() if v}
        if parts:
            parts["sync_ms"] = g["sync_p50_ms"]
            parts["other_ms"] = round(max(0.0, gp50 - parts["sync_ms"] - parts.get("pickup_ms", 0) -
                                          parts.get("log_delivery_ms", 0)), 2)
            g["breakdown_p50"] = parts
        gr = extras.get("gpu_pod_ref")
        if _ok(gr):
            rp50 = _pct(gr["reload_ms"], 0.5)
            g["reference_equivalent"] = {
                "what": "compat sync protocol + a cold restart of the Python/torch workload per change "
                        "(nodemon-style): prices the hot-reload runner more than the CLI",
                "p50_ms": round(rp50, 2), "sync_p50_ms": round(_pct(gr["sync_ms"], 0.5), 2),
                "speedup": round(rp50 / gp50, 1) if gp50 else None}
        gw = extras.get("gpu_pod_wan")
        if _ok(gw):  # edit train.py on a laptop -> the remote pod's reload line back on the laptop
            g["wan"] = {"rtt_ms": WAN[0], "mbit": WAN[1],
                        "reload_p50_ms": round(_pct(gw["reload_ms"], 0.5), 2),
                        "reload_p90_ms": round(_pct(gw["reload_ms"], 0.9), 2),
                        "sync_p50_ms": round(_pct(gw["sync_ms"], 0.5), 2), "n": len(gw["reload_ms"]),
                        "pod_deploy_s": round(gw["pod_deploy_s"], 3)}
        elif gw is not None:
            g["wan"] = gw
        out["gpu_pod"] = g
    for key in EXAMPLES:
        e, er = extras.get(key), extras.get(key + "_ref")
        if e is None:
            continue
        if _ok(e) and _ok(er):
            e = dict(e)
            e["reference_equivalent"] = {k: er[k] for k in ("deploy_cold_s", "deploy_warm_s", "edit_to_pod_p50_ms",
                                                             "dev_ready_s", "n")}
            e["reference_equivalent"]["edit_to_pod_speedup"] = round(
                er["edit_to_pod_p50_ms"] / max(e["edit_to_pod_p50_ms"], 1e-3), 1)
        if _ok(e):
            e = dict(e, note=EXAMPLE_NOTES[key])
        out[key] = e
    # an extra that failed is named with its message (its block is otherwise absent or {"error"})
    errors = {k: v["error"] for k, v in extras.items() if isinstance(v, dict) and "error" in v}
    if errors:
        out["extra_errors"] = errors
    return out


if __name__ == "__main__":
    sys.exit(main())
