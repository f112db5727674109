"""Hot-reload runner (workload side): code swap without losing state."""
import os
import re
import subprocess
import sys
import time

import pytest

from conftest import ROOT

TRAIN = os.path.join(ROOT, "examples", "rocm-pytorch", "train.py")


def _tiny_copy(tmp_path):
    src = open(TRAIN).read()
    for k, v in (("VOCAB", 128), ("DIM", 64), ("HEADS", 4), ("LAYERS", 1), ("SEQ", 16), ("BATCH", 2)):
        src = re.sub(rf"^{k} = \d+$", f"{k} = {v}", src, flags=re.M)
    p = tmp_path / "train.py"
    p.write_text(src)
    return p


def _run_reload(tmp_path, extra_env=None, nproc=1):
    p = _tiny_copy(tmp_path)
    env = dict(os.environ, PYTHONPATH=ROOT, **(extra_env or {}))
    proc = subprocess.Popen([sys.executable, "-u", "-m", "devspace_amd.runner", "--nproc", str(nproc), "--watch",
                             str(tmp_path), str(p)],
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True)
    lines = []
    try:
        t0 = time.time()
        while time.time() - t0 < 180:
            line = proc.stdout.readline()
            lines.append(line)
            if "started gen=1" in line:
                break
        assert any("started gen=1" in l for l in lines), "".join(lines)
        p.write_text(p.read_text().replace('MARKER = "v0"', 'MARKER = "edited"'))
        t0 = time.time()
        while time.time() - t0 < 60:
            line = proc.stdout.readline()
            lines.append(line)
            if "marker=edited" in line:
                break
        reload_line = [l for l in lines if "marker=edited" in l]
        assert reload_line, "".join(lines[-20:])
        # a broken edit keeps the previous version running
        p.write_text(p.read_text() + "\nthis is not python\n")
        t0 = time.time()
        while time.time() - t0 < 60:
            line = proc.stdout.readline()
            lines.append(line)
            if "reload failed" in line:
                break
        failed = [l for l in lines if "reload failed" in l]
        assert failed
        # one generation per edit on every rank count (no second, spurious reload of the first edit)
        assert "gen=3" in failed[0], "".join(lines[-20:])
        assert proc.poll() is None
        return reload_line[0] + "".join(l for l in lines if "started gen=1" in l)
    finally:
        import psutil

        kids = psutil.Process(proc.pid).children(recursive=True)
        proc.terminate()
        proc.wait(10)
        # the ranks go with the supervisor (no orphaned workers left training)
        _, alive = psutil.wait_procs(kids, timeout=20)
        for k in alive:
            k.kill()
        assert not alive, f"workers outlived the supervisor: {alive}"


def test_runner_hot_reload_cpu(tmp_path):
    line = _run_reload(tmp_path, {"HIP_VISIBLE_DEVICES": "-1", "CUDA_VISIBLE_DEVICES": "-1"})
    assert "gen=2" in line
    # the code swap stays cheap with torch's thousands of modules imported (a per-reload scan of
    # sys.modules with realpath() once cost ~50 ms here)
    assert float(re.search(r"reload_ms=([\d.]+)", line).group(1)) < 15, line


def test_runner_hot_reload_two_ranks_cpu(tmp_path):
    """The N>1 path of the pod (one process per GPU, DDP, generation agreement by all-reduce),
    rehearsed with two gloo ranks on the CPU."""
    line = _run_reload(tmp_path, {"HIP_VISIBLE_DEVICES": "-1", "CUDA_VISIBLE_DEVICES": "-1"}, nproc=2)
    assert "gen=2" in line and "world=2" in line


@pytest.mark.gpu
def test_runner_hot_reload_gpu(tmp_path):
    line = _run_reload(tmp_path)
    assert "gen=2" in line


@pytest.mark.gpu
def test_runner_hot_reload_two_ranks_on_the_gpu(tmp_path):
    """The multi-rank pod on real GPU streams (DDP, generation agreement, GPU-side preemption
    drain): two ranks on the one device of the box, joined over gloo (RCCL refuses two ranks on
    one GPU; the 8-GPU node runs RCCL)."""
    line = _run_reload(tmp_path, {"DEVSPACE_DIST_BACKEND": "gloo"}, nproc=2)
    assert "gen=2" in line and "world=2" in line and "device=cuda" in line, line


SLOW_STEP = '''
import time
MARKER = "v0"


def setup(ctx):
    return {"updates": 0}


def step(ctx, state):
    # a 0.8 s "step" with a preemption point every 10 ms, then the state update
    for _ in range(80):
        time.sleep(0.01)
        ctx.preempt_point()
    state["updates"] += 1
    return {"loss": state["updates"]}
'''


SLOW_STEP_GPU = '''
import torch
MARKER = "v0"


def setup(ctx):
    a = torch.randn(4096, 4096, device=ctx.device, dtype=torch.bfloat16)
    return {"a": a, "updates": 0}


def step(ctx, state):
    # ~0.4 s of queued matmuls, a preemption point (drains: the loop period is > 20 ms), then
    # another ~0.4 s and the state update
    a = state["a"]
    for _ in range(1500):
        b = a @ a
    ctx.preempt_point()
    for _ in range(1500):
        b = a @ a
    state["updates"] += 1
    torch.cuda.synchronize()
    return {"loss": state["updates"]}
'''


def _pickup_ms(tmp_path, preempt, src=SLOW_STEP, gpu=False, nproc=1, extra_env=None):
    p = tmp_path / "slow.py"
    p.write_text(src)
    env = dict(os.environ, PYTHONPATH=ROOT, **(extra_env or {}))
    if not gpu:
        env.update(HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1")
    cmd = [sys.executable, "-u", "-m", "devspace_amd.runner", "--nproc", str(nproc), "--watch", str(tmp_path), str(p)]
    if not preempt:
        cmd.insert(-1, "--no-preempt")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True)
    try:
        lines = []
        while True:
            line = proc.stdout.readline()
            assert line, "".join(lines)
            lines.append(line)
            if "started gen=1" in line:
                break
        time.sleep(0.3 if not gpu else 1.5)  # a few steps in: the loop period is known
        p.write_text(src.replace('MARKER = "v0"', 'MARKER = "v1"'))
        while True:
            line = proc.stdout.readline()
            assert line, "".join(lines)
            lines.append(line)
            if "marker=v1" in line:
                break
        f = dict(re.findall(r"(\w+_ms)=([\d.]+)", line))
        # the abandoned step never reached its state update; the new step did
        assert re.search(r"loss=(\d+)", line), line
        if gpu:
            return float(f["pickup_ms"]), float(f["period_ms"])
        return float(f["inflight_ms"]), int(re.search(r"loss=(\d+)", line).group(1))
    finally:
        proc.terminate()
        proc.wait(10)


def test_preempt_point_cuts_inflight_wait(tmp_path):
    """ctx.preempt_point(): an edit landing mid-step abandons the rest of the old step (before
    its state update) instead of waiting for it; --no-preempt waits for the whole step."""
    inflight, updates = _pickup_ms(tmp_path, preempt=True)
    assert inflight < 200, inflight
    # started step = 1 update; the preempted step added none; the new-code step adds one
    assert updates == 2, updates
    inflight_np, updates_np = _pickup_ms(tmp_path, preempt=False)
    assert inflight_np > 250, inflight_np
    assert updates_np == 3


def test_preempt_point_four_ranks_cpu(tmp_path):
    """world > 1 preempts too: the ranks decide together at the point (rank 0's
    change feed, one gloo all-reduce of a CPU flag), so an edit landing mid-step is picked up
    within a fraction of the 0.8 s step on 4 gloo ranks, as with one rank, and every rank skips
    the rest of the old step (its state update) at the same point."""
    inflight, updates = _pickup_ms(tmp_path, preempt=True, nproc=4)
    assert inflight < 200, inflight
    assert updates == 2, updates
    inflight_np, updates_np = _pickup_ms(tmp_path, preempt=False, nproc=4)
    assert inflight_np > 250, inflight_np
    assert updates_np == 3


def test_control_plane_never_touches_the_device():
    """The multi-rank control plane (generation + preemption agreement) runs on CPU tensors over
    its own gloo group, and the steady-state training loop holds no device sync (`.item()`,
    `.tolist()`, `torch.cuda.synchronize()`): the host keeps running ahead of the GPUs."""
    import ast
    import types

    import torch

    from devspace_amd import runner

    calls = []

    def all_reduce(t, op=None, group=None):
        calls.append((t.device.type, group, op))
        t.mul_(1)  # a single-rank MAX is the identity

    fake = types.SimpleNamespace(all_reduce=all_reduce, ReduceOp=types.SimpleNamespace(MAX="max"),
                                 new_group=lambda backend: f"group:{backend}")
    a = runner.Agreement(fake)
    assert a.group == "group:gloo"
    assert a.boundary(7, True) == (7, True, False)
    assert a.preempt(True) is True and a.preempt(False) is False
    assert calls and all(c == ("cpu", "group:gloo", "max") for c in calls), calls

    tree = ast.parse(open(runner.__file__).read())
    worker = next(n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == "worker_main")
    # the training loop (the other one is the startup retry loop, which may synchronize)
    loop = next(n for n in ast.walk(worker) if isinstance(n, ast.While) and "not stop" in ast.unparse(n.test))
    reload_branch = next(n for n in loop.body if isinstance(n, ast.If) and "target > gen" in ast.unparse(n.test))
    steady = [n for n in loop.body if n is not reload_branch]
    syncing = []
    for stmt in steady:
        for n in ast.walk(stmt):
            if isinstance(n, ast.Call) and isinstance(n.func, ast.Attribute) and n.func.attr in (
                    "item", "tolist", "synchronize", "cpu"):
                syncing.append(ast.unparse(n))
    assert not syncing, syncing
    assert not [n for n in ast.walk(worker) if isinstance(n, ast.Attribute) and n.attr == "tolist"]


@pytest.mark.gpu
def test_preempt_point_drains_gpu_queue(tmp_path):
    """On the GPU the point drains the queued work while polling the change feed: an edit that
    lands during the first half of a long step does not wait for the second half."""
    pickup, period = _pickup_ms(tmp_path, preempt=True, src=SLOW_STEP_GPU, gpu=True)
    assert period > 100, period
    # edit -> new step done <= rest of the phase in flight (<= half a step) + one full new step;
    # without the drain it is the rest of the whole step + one new step (up to two periods)
    assert pickup < 1.6 * period, (pickup, period)


@pytest.mark.gpu
def test_preempt_point_drains_gpu_queue_two_ranks(tmp_path):
    """The same with two ranks on the GPU: each drains its own queue, then the ranks decide
    together, so both leave the long step at the same point."""
    pickup, period = _pickup_ms(tmp_path, preempt=True, src=SLOW_STEP_GPU, gpu=True, nproc=2,
                                extra_env={"DEVSPACE_DIST_BACKEND": "gloo"})
    assert period > 100, period
    assert pickup < 1.6 * period, (pickup, period)


def test_preempt_point_noop_without_feed():
    from devspace_amd.runner import Context, Preempted

    class Feed:
        n = 0

        def pending(self):
            return self.n > 0

    import torch

    ctx = Context(0, 1, 0, torch.device("cpu"))
    ctx.preempt_point()  # no feed attached: never raises
    ctx._feed = Feed()
    ctx.preempt_point()
    ctx._feed.n = 1
    with pytest.raises(Preempted):
        ctx.preempt_point()


def test_edit_during_slow_setup_is_picked_up(tmp_path):
    """An edit that lands while setup() (or the first step) is still running must neither crash
    the runner (the first step is outside the preemption handler) nor be lost."""
    mod = tmp_path / "slow.py"
    flag = tmp_path / "in_setup"
    mod.write_text(
        'import time\nMARKER = "v0"\n'
        f'def setup(ctx):\n    open({str(flag)!r}, "w").close()\n    time.sleep(1.5)\n    return {{}}\n'
        'def step(ctx, state):\n    ctx.preempt_point()\n    time.sleep(0.01)\n    ctx.preempt_point()\n'
        '    return {"loss": 1.0}\n')
    env = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1")
    proc = subprocess.Popen([sys.executable, "-u", "-m", "devspace_amd.runner", "--watch", str(tmp_path), str(mod)],
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True)
    lines = []
    try:
        t0 = time.time()
        while not flag.exists() and time.time() - t0 < 120:
            time.sleep(0.01)
        assert flag.exists(), "setup never ran"
        mod.write_text(mod.read_text().replace('MARKER = "v0"', 'MARKER = "during_setup"'))
        t0 = time.time()
        while time.time() - t0 < 60:
            line = proc.stdout.readline()
            if not line:
                break
            lines.append(line)
            if "marker=during_setup" in line:
                break
        assert any("marker=during_setup" in l for l in lines), "".join(lines)
        assert proc.poll() is None, "".join(lines)
        assert not any("Traceback" in l for l in lines), "".join(lines)
    finally:
        proc.terminate()
        proc.wait(10)


def test_preempted_is_not_swallowed_by_generic_handlers():
    from devspace_amd.runner import Preempted

    assert not issubclass(Preempted, Exception)
    with pytest.raises(Preempted):
        try:
            raise Preempted()
        except Exception:  # a user step's catch-all must let the preemption through
            pass


def test_workload_kit_is_the_package(tmp_path):
    """The workload kit (runner + gfx950 fused ops) that `devspace init` vendors into rocm-pytorch
    projects and the build writes into examples/rocm-pytorch is the package itself: one source
    (devspace_amd/KIT), byte-identical copies, no tracked duplicate in git."""
    from devspace_amd import kit

    names = kit.files()
    assert {"runner.py", "ops/fused.py", "ops/fused_ops.hip", "ops/build.py"} <= set(names)
    kit.write_kit(str(tmp_path))
    for rel in names:
        assert (tmp_path / "devspace_amd" / rel).read_bytes() == open(os.path.join(ROOT, "devspace_amd", rel), "rb").read()
    tracked = subprocess.run(["git", "ls-files", "examples/rocm-pytorch", "templates/rocm-pytorch"], cwd=ROOT,
                             capture_output=True, text=True).stdout.split()
    assert not [t for t in tracked if "devspace_amd/" in t or t.endswith("devspace_runner.py")], tracked
    # the example carries the kit after a build (the test session's ensure_built)
    for rel in names:
        assert open(os.path.join(ROOT, "examples", "rocm-pytorch", "devspace_amd", rel), "rb").read() == \
            open(os.path.join(ROOT, "devspace_amd", rel), "rb").read(), rel


def test_vendored_runner_runs_without_the_checkout(tmp_path):
    """A project with the kit and no devspace_amd on the Python path (a pod): the runner and the
    fused ops import from the project, the file watcher is the ctypes inotify one, and train.py
    says which op path runs (fused=... line; eager on this CPU-only machine)."""
    from devspace_amd import kit

    proj = tmp_path / "proj"
    proj.mkdir()
    kit.write_kit(str(proj))
    src = open(TRAIN).read()
    for k, v in (("VOCAB", 128), ("DIM", 64), ("HEADS", 4), ("LAYERS", 1), ("SEQ", 16), ("BATCH", 2)):
        src = re.sub(rf"^{k} = \d+$", f"{k} = {v}", src, flags=re.M)
    (proj / "train.py").write_text(src)
    env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    env.update(HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1")
    probe = subprocess.run([sys.executable, "-c", "import devspace_amd, devspace_amd.runner as r; "
                            "print(devspace_amd.__file__); print(type(r.make_watcher('.')).__name__)"],
                           cwd=str(proj), env=env, capture_output=True, text=True)
    assert probe.returncode == 0, probe.stderr
    where, watcher = probe.stdout.split()
    assert where.startswith(str(proj)), where
    assert watcher == "_InotifyWatcher", watcher
    proc = subprocess.Popen([sys.executable, "-u", "-m", "devspace_amd.runner", "--max-steps", "3", "--watch",
                             str(proj), "train.py"], cwd=str(proj), env=env, stdout=subprocess.PIPE,
                            stderr=subprocess.STDOUT, text=True)
    out, _ = proc.communicate(timeout=180)
    assert proc.returncode == 0, out
    assert "fused=eager (no GPU)" in out and "started gen=1" in out, out


HELPER_ENTRY = '''
import helper_mod
MARKER = helper_mod.MARKER


def setup(ctx):
    return {}


def step(ctx, state):
    import time
    time.sleep(0.01)
    return {"loss": helper_mod.value()}
'''


def test_runner_reloads_edited_helper_module(tmp_path):
    """An edit of a module the entry file imports (not only of the entry file) takes effect at
    the next reload: the runner drops the synced tree's modules from the import cache."""
    (tmp_path / "helper_mod.py").write_text('MARKER = "v0"\n\n\ndef value():\n    return 1\n')
    entry = tmp_path / "train.py"
    entry.write_text(HELPER_ENTRY)
    env = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1")
    proc = subprocess.Popen([sys.executable, "-u", "-m", "devspace_amd.runner", "--watch", str(tmp_path), str(entry)],
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True, cwd=str(tmp_path))
    import queue
    import threading

    lines, q = [], queue.Queue()
    threading.Thread(target=lambda: [q.put(l) for l in proc.stdout], daemon=True).start()

    def until(pat, timeout=60):
        deadline = time.time() + timeout
        while time.time() < deadline:
            try:
                line = q.get(timeout=max(0.01, deadline - time.time()))
            except queue.Empty:
                break
            lines.append(line)
            if re.search(pat, line):
                return line
        raise AssertionError(f"no line matching {pat!r}:\n" + "".join(lines[-20:]))

    try:
        until(r"started gen=1 marker=v0")
        (tmp_path / "helper_mod.py").write_text('MARKER = "v1"\n\n\ndef value():\n    return 2\n')
        line = until(r"reloaded gen=\d+ marker=v1")
        assert "loss=2" in line, line
        # an edit of the entry file alone keeps the (unchanged) helper cached and still reloads
        entry.write_text(HELPER_ENTRY.replace("MARKER = helper_mod.MARKER", 'MARKER = "entry-" + helper_mod.MARKER'))
        until(r"reloaded gen=\d+ marker=entry-v1")
    finally:
        proc.terminate()
        proc.wait(10)


def test_change_feed_ignores_sync_temp_file(tmp_path):
    """The in-pod sync helper writes `<name>.devspace-tmp`, then renames it into place: only
    the rename is an edit (one change batch, compiled from the new bytes), and the in-pod
    inotify watcher reports it without waiting out a long burst window."""
    from devspace_amd import runner

    entry = tmp_path / "train.py"
    entry.write_text('MARKER = "v0"\n')
    w = runner._InotifyWatcher(str(tmp_path))
    feed = runner.ChangeFeed(w, str(entry))
    try:
        time.sleep(0.05)
        tmp = tmp_path / ("train.py" + runner.SYNC_TMP_SUFFIX)
        tmp.write_text('MARKER = "v1"\n')
        time.sleep(0.02)  # the temp file's close-write lands in a batch of its own
        assert feed.take(0.05)[0] == 0, "the helper's temp file counted as an edit"
        t0 = time.perf_counter()
        os.rename(tmp, entry)
        n, t_first, _ = feed.take(5.0)
        assert n == 1
        assert t_first - t0 < 0.5
        assert feed.prepared_for(b'MARKER = "v1"\n') is not None
    finally:
        feed.close()
        w.close()


def test_inotify_watcher_returns_a_rename_at_once(tmp_path):
    from devspace_amd import runner

    w = runner._InotifyWatcher(str(tmp_path))
    try:
        (tmp_path / "a.py.devspace-tmp").write_text("x = 1\n")
        os.rename(tmp_path / "a.py.devspace-tmp", tmp_path / "a.py")
        t0 = time.perf_counter()
        got = w.poll(1000)
        took = time.perf_counter() - t0
        assert str(tmp_path / "a.py") in got
        assert runner._ignored(str(tmp_path / "a.py.devspace-tmp"))
        assert took < 0.05, took  # events already queued: no multi-ms burst wait
    finally:
        w.close()


def _agree_stop_worker(rank, world, init_file, out):
    import torch.distributed as dist

    from devspace_amd import runner

    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        agree = runner.Agreement(dist)
        first = agree.boundary(3, False, stop=False)
        second = agree.boundary(3 + rank, rank == 0, stop=(rank == world - 1))  # only the last rank got SIGTERM
        out.put((rank, first, second))
    finally:
        dist.destroy_process_group()


def test_agreement_stops_every_rank_at_the_same_boundary(tmp_path):
    """SIGTERM reaches the ranks at different moments: the stop flag is agreed like the
    generation, so every rank leaves at the same step boundary (none is left waiting in a
    collective of a step the others never start)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    world = 3
    procs = [ctx.Process(target=_agree_stop_worker, args=(r, world, str(tmp_path / "init"), out)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(out.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, first, second in res:
        assert first == (3, False, False)
        assert second == (3 + world - 1, True, True), (rank, second)


def test_default_rescue_dir_outside_a_pod_sweeps_dead_runners_leftovers(tmp_path, monkeypatch):
    """Outside a pod the snapshots are scoped to the supervisor's pid; a runner killed outright
    cannot clean up, so the next one drops directories whose process is gone (and only those)."""
    from devspace_amd import runner

    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    monkeypatch.setenv("DEVSPACE_RESCUE_ROOT", str(tmp_path))
    dead = tmp_path / "devspace-rescue-999999999"
    alive = tmp_path / f"devspace-rescue-{os.getppid()}"
    other = tmp_path / "devspace-rescue-notapid"
    for d in (dead, alive, other):
        d.mkdir()
        (d / "rank0-step1.json").write_text("{}")
    got = runner._default_rescue_dir("train.py", 2)
    assert got == str(tmp_path / f"devspace-rescue-{os.getpid()}")
    assert not dead.exists() and alive.exists() and other.exists()
    # in a pod: a stable path per entry file and rank count (survives a container restart)
    monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "10.96.0.1")
    a, b = runner._default_rescue_dir("train.py", 2), runner._default_rescue_dir("train.py", 2)
    assert a == b != runner._default_rescue_dir("train.py", 4)
