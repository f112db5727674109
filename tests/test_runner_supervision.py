"""The runner's supervision rules that round 4 got wrong (VERDICT r4 "Next round" items 1-2):

* a long healthy step is never mistaken for a stuck one: the stuck-step restart needs an edit
  pending in a steady-state step, the step past max(--stuck-after, 10 x the longest step so far),
  no rank's main thread moving for --stuck-after, and a rescue snapshot to resume from; a long
  step that does not meet that is reported once and left alone;
* a restart stops the whole process tree of a group, including what the ranks started, what
  escaped into its own session and what was orphaned (the supervisor is a child subreaper);
* replicated (DDP) state is snapshotted once for the group, not once per rank.

The reference's model for all three: a fresh process tree per reload (nodemon,
/root/reference/examples/quickstart/package.json:7; redeploy, /root/reference/cmd/dev.go:225-234)
and acting only on evidence seen twice (/root/reference/pkg/devspace/sync/downstream.go:117-123).
Rehearsed on CPU with gloo ranks.
"""
import os
import re
import time
import uuid

import psutil
import pytest

from test_runner_failsafe import Runner, _set_marker

LONG_EVAL = '''
import os
import time

import torch
import torch.distributed as dist

MARKER = "v0"
EVAL = {eval!r}


def setup(ctx):
    return {{"n": 0}}


def step(ctx, state):
    flag = torch.tensor([1.0 if ctx.rank == 0 and os.path.exists(EVAL) else 0.0])
    if ctx.distributed:
        dist.all_reduce(flag)
    if flag.item():
        if ctx.rank == 0:
            os.unlink(EVAL)
            t0 = time.monotonic()
            x = torch.randn(128, 128)
            while time.monotonic() - t0 < 5.0:  # a 5 s evaluation: busy, healthy
                x = torch.tanh(x @ x.t() / 128.0)
            ctx.log("eval done")
        if ctx.distributed:
            dist.barrier()  # the other ranks wait here for rank 0's eval, standing still
    state["n"] += 1
    time.sleep(0.005)
    return {{"loss": state["n"]}}
'''


@pytest.mark.parametrize("nproc", [1, 2])
def test_a_long_healthy_step_survives_an_edit(tmp_path, nproc):
    """VERDICT r4 Weak #1: a step that runs a 5 s evaluation with --stuck-after 1 while an edit
    lands (and rescue snapshots exist) is not restarted: rank 0's main thread moves the whole
    time. The long step is reported once, and the edit applies right after the evaluation."""
    trigger = tmp_path.parent / (tmp_path.name + "-eval")
    entry = tmp_path / "train.py"
    entry.write_text(LONG_EVAL.format(eval=str(trigger)))
    r = Runner(tmp_path, entry, nproc, extra_args=("--log-every", "50", "--rescue-every", "0.5", "--stuck-after", "1"))
    try:
        r.until(r"started gen=1 marker=v0", timeout=180)
        r.until(r"rescue snapshot step=\d+ ", timeout=60)
        trigger.write_text("1")
        time.sleep(1.5)  # inside the evaluation
        _set_marker(entry, "v1")
        _, line = r.until(r"rank=\d in step for \d+ s at train.py:\d+; edit pending: rank=0 is making progress",
                          timeout=30)
        t_done, _ = r.until(r"eval done", timeout=30)
        t_reload, _ = r.until(r"reloaded gen=2 marker=v1 ", timeout=30)
        assert t_reload >= t_done
        time.sleep(1.0)
        text = r.text()
        assert "made no progress" not in text and "exited with code" not in text, text[-3000:]
        assert len(re.findall(r"in step for \d+ s", text)) == 1, text[-3000:]  # reported once
    finally:
        r.stop()


SLOW_SETUP = '''
import time

MARKER = "v0"
SETUP_VERSION = 1


def setup(ctx):
    if SETUP_VERSION == 2:
        time.sleep(4.0)  # loading a bigger model: the main thread stands still, in setup()
    return {"n": 0}


def step(ctx, state):
    state["n"] += 1
    time.sleep(0.005)
    return {"loss": state["n"]}
'''


def test_a_slow_setup_on_reload_is_not_stuck(tmp_path):
    """a reload whose setup() (SETUP_VERSION changed) takes longer than --stuck-after,
    standing still, is a reload, not a stuck step: no restart."""
    entry = tmp_path / "train.py"
    entry.write_text(SLOW_SETUP)
    r = Runner(tmp_path, entry, 1, extra_args=("--log-every", "50", "--rescue-every", "0.5", "--stuck-after", "1"))
    try:
        r.until(r"started gen=1 marker=v0", timeout=180)
        r.until(r"rescue snapshot step=\d+ ", timeout=60)
        entry.write_text(SLOW_SETUP.replace("SETUP_VERSION = 1", "SETUP_VERSION = 2").replace('"v0"', '"v1"'))
        time.sleep(1.5)
        _set_marker(entry, "v2")  # a second edit while setup() runs
        r.until(r"reloaded gen=\d+ marker=v2 ", timeout=30)
        assert "made no progress" not in r.text() and "exited with code" not in r.text(), r.text()[-3000:]
    finally:
        r.stop()


TREE = '''
import os
import subprocess
import time

import torch
import torch.distributed as dist

MARKER = "v0"
TAG = {tag!r}


def setup(ctx):
    kids = [subprocess.Popen(["sleep", TAG + "1"]),  # a plain child (an eval worker)
            subprocess.Popen(["sleep", TAG + "2"], start_new_session=True)]  # escaped into its own session
    subprocess.Popen(["sh", "-c", "sleep " + TAG + "3 &"]).wait()  # a daemon, orphaned at once
    return {{"kids": kids, "n": 0}}


def step(ctx, state):
    if MARKER == "crash" and state["n"] > 20 and ctx.rank == ctx.world_size - 1:
        os._exit(7)  # a hard crash after the group came up: restarted, up to --max-restarts
    if ctx.distributed:
        dist.all_reduce(torch.ones(1))
    state["n"] += 1
    time.sleep(0.005)
    return {{"loss": state["n"]}}
'''


def _tagged(tag):
    out = []
    for p in psutil.process_iter(["cmdline", "status"]):
        cmd = p.info["cmdline"] or []
        if len(cmd) == 2 and cmd[0] == "sleep" and cmd[1].startswith(tag):
            out.append(p)
    return out


@pytest.mark.parametrize("nproc", [1, 2])
def test_restarts_stop_the_whole_process_tree(tmp_path, nproc):
    """VERDICT r4 Missing #1 / Weak #3: each rank's setup() starts a child, a child in its own
    session and an orphaned daemon. One crashing edit makes the group crash and be restarted
    --max-restarts (3) times, then wait for the next edit. Afterwards none of those processes of
    the four dead groups is alive and no zombie is left under the supervisor; while a group runs,
    exactly its own are."""
    tag = str(7000 + uuid.uuid4().int % 1000)
    entry = tmp_path / "train.py"
    entry.write_text(TREE.format(tag=tag))
    r = Runner(tmp_path, entry, nproc, extra_args=("--log-every", "50", "--rescue-every", "0"))
    try:
        r.until(r"started gen=1 marker=v0", timeout=180)
        time.sleep(0.5)
        assert len(_tagged(tag)) == 3 * nproc, [p.info for p in _tagged(tag)]
        _set_marker(entry, "crash")
        r.until(r"restarts without an edit: waiting for a file change", timeout=180)
        assert len(re.findall(r"exited with code 7", r.text())) >= 4, r.text()[-3000:]
        time.sleep(0.5)
        alive = [p for p in _tagged(tag) if p.status() != psutil.STATUS_ZOMBIE]
        assert not alive, [(p.pid, p.cmdline(), p.ppid()) for p in alive]
        zombies = [k for k in psutil.Process(r.proc.pid).children() if k.status() == psutil.STATUS_ZOMBIE]
        assert not zombies, zombies
        _set_marker(entry, "fixed")
        r.until(r"started gen=1 marker=fixed", timeout=60)
        time.sleep(0.5)
        assert len(_tagged(tag)) == 3 * nproc  # the new group's own, and nothing else
    finally:
        r.stop()
        for p in _tagged(tag):
            p.kill()
    assert not _tagged(tag)  # a clean stop takes them too


DDP_STATE = '''
import os

import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as DDP

from devspace_amd.rescue import digests

MARKER = "v0"
SETUP_VERSION = 1
MB = {mb}
LOG = {log!r}
FAIL = {fail!r}


def setup(ctx):
    torch.manual_seed(0)
    dim = 1024
    layers = max(1, MB * 2**20 // (3 * 4 * dim * dim))  # fp32 weights + AdamW's two moments
    blocks = []
    for _ in range(layers):  # normalised blocks: every layer gets a gradient (no tensor of zeros)
        blocks += [torch.nn.Linear(dim, dim, bias=False), torch.nn.LayerNorm(dim)]
    model = DDP(torch.nn.Sequential(*blocks), gradient_as_bucket_view=True)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    return {{"model": model, "opt": opt, "cursor": torch.tensor([ctx.rank * 1000 + 1])}}


def _digest(state):
    ts = list(state["model"].state_dict().values()) + [state["cursor"]]
    for s in state["opt"].state.values():
        ts += [v for v in s.values() if isinstance(v, torch.Tensor)]
    return "".join(digests(ts))[:32] if ts else "-"


def step(ctx, state):
    with open(LOG + str(ctx.rank), "a") as f:  # the state this step starts from, bit for bit
        f.write(f"{{ctx.step}} {{_digest(state)}}\\n")
    if ctx.rank == 1 and os.path.exists(FAIL):
        os.unlink(FAIL)
        raise RuntimeError("once")
    model, opt = state["model"], state["opt"]
    x = torch.randn(8, model.module[0].in_features, generator=torch.Generator().manual_seed(ctx.step * 8 + ctx.rank))
    loss = model(x).pow(2).mean()
    opt.zero_grad()
    loss.backward()
    opt.step()
    state["cursor"] += 1
    return {{"loss": float(loss)}}
'''


def _digest_at(path, step):
    last = None
    with open(path) as f:
        for line in f:
            s, d = line.split()
            if int(s) == step:
                last = d
    return last


def test_ddp_snapshot_is_written_once_and_restores_bit_exact(tmp_path):
    """VERDICT r4 Weak #2: 8 gloo ranks under DDP. The group's snapshot takes one rank's worth
    of shared memory (plus the per-rank cursors), not eight; after rank 1 fails, the restarted
    group resumes with every rank's model, optimizer moments and cursor bit-identical to the
    snapshot step. RESCUE_TEST_MB sets the state per rank (default 24 MiB; the profile in
    profiles/r5_rescue_dedup_*.json is this test at 2048)."""
    mb = int(os.environ.get("RESCUE_TEST_MB", "24"))
    world = int(os.environ.get("RESCUE_TEST_RANKS", "8"))
    log = str(tmp_path.parent / (tmp_path.name + "-digest"))
    fail = tmp_path.parent / (tmp_path.name + "-fail")
    entry = tmp_path / "train.py"
    entry.write_text(DDP_STATE.format(mb=mb, log=log, fail=str(fail)))
    shm = tmp_path.parent / (tmp_path.name + "-shm")
    r = Runner(tmp_path, entry, world, extra_args=("--log-every", "10", "--rescue-every", "2"),
               extra_env={"KUBERNETES_SERVICE_HOST": "10.96.0.1", "DEVSPACE_RESCUE_ROOT": str(shm),
                          "DEVSPACE_WARM_STANDBY": "0"})
    try:
        r.until(rf"started gen=1 marker=v0 .*world={world}", timeout=600)
        _, line = r.until(r"rescue snapshot step=(\d+) ", timeout=600)
        snap_line = line
        m = re.search(r"rescue snapshot step=(\d+) .*\(group: ([\d.]+) MiB in shared memory for ([\d.]+) MiB of state", line)
        step, group_mib, state_mib = int(m.group(1)), float(m.group(2)), float(m.group(3))
        d = next(shm.iterdir())
        on_disk = sum(f.stat().st_size for f in d.iterdir() if re.match(rf"rank\d+-step{step}\.bin$", f.name))
        print(f"world={world} state {state_mib:.1f} MiB over the ranks, group snapshot {group_mib:.1f} MiB, "
              f"on disk {on_disk / 2**20:.1f} MiB")
        assert abs(on_disk / 2**20 - group_mib) < 0.5
        assert group_mib < state_mib / world * 1.05 + 1, line  # one rank's worth, not `world` of them
        fail.write_text("1")
        r.until(r"rank=1 exited with code 3: restarting the group", timeout=600)
        snapped = max(int(s) for s in re.findall(r"rescue snapshot step=(\d+)", r.text()))
        _, line = r.until(r"restored step=(\d+) ", timeout=900)
        restored = int(re.search(r"restored step=(\d+)", line).group(1))
        assert restored == snapped, (restored, snapped)
        _, up = r.until(rf"started gen=1 marker=v0 .*world={world}", timeout=600)
        if os.environ.get("RESCUE_TEST_OUT"):  # the profile of a large run (profiles/r5_rescue_dedup_*.json)
            import json

            restore = re.search(r"restored step=\d+ .*\(age ([\d.]+) s, ([\d.]+) MiB/rank in ([\d.]+) ms\)", line)
            with open(os.environ["RESCUE_TEST_OUT"], "w") as f:
                json.dump({"ranks": world, "state_mib_per_rank": round(state_mib / world, 1),
                           "state_mib_all_ranks": state_mib, "group_snapshot_mib": group_mib,
                           "on_disk_mib": round(on_disk / 2**20, 1), "restored_step": restored,
                           "restore_ms_rank0": float(restore.group(3)) if restore else None,
                           "digest_ms": float(re.search(r"digest ([\d.]+) ms", snap_line).group(1))
                           if re.search(r"digest ([\d.]+) ms", snap_line) else None,
                           "snapshot_line": re.sub(r"^.*\[devspace-runner\] ", "", snap_line.strip()),
                           "bit_exact_on_every_rank": True}, f, indent=1)
        for rank in range(world):
            path = log + str(rank)
            with open(path) as f:
                lines = f.read().split("\n")
            # the step the restarted group starts from was written before the failure, and again after
            firsts = [l for l in lines if l.startswith(f"{restored} ")]
            assert len(firsts) >= 2 and len(set(firsts)) == 1, (rank, firsts)
    finally:
        r.stop()


CHATTY = '''
import os

MARKER = "v0"
LINES = {lines}


def setup(ctx):
    # every rank floods its stdout and stderr at once, lines of different lengths, some without a
    # flush between them: the supervisor must relay each as one whole line
    import sys

    for i in range(LINES):
        pad = "x" * (i % 97)
        out = sys.stderr if i % 5 == 0 else sys.stdout
        out.write(f"R={{ctx.rank}} I={{i}} {{pad}}|\\n")
    sys.stdout.flush()
    sys.stderr.flush()
    return {{"n": 0}}


def step(ctx, state):
    state["n"] += 1
    return {{"loss": state["n"]}}
'''


def test_eight_ranks_logs_are_whole_prefixed_lines(tmp_path):
    """8 gloo ranks writing 10k lines each at once. Every line reaches the
    supervisor's stdout whole and once, prefixed `[rank N]` with its own rank; gloo's 8
    per-connection lines become one `group of 8 rank(s) connected` line; each rank's
    `started`-line is prefixed as well."""
    world, lines = 8, 10000
    entry = tmp_path / "train.py"
    entry.write_text(CHATTY.format(lines=lines))
    r = Runner(tmp_path, entry, world, extra_args=("--log-every", "1000000", "--max-steps", "3"))
    try:
        r.until(rf"\[rank 0\] \[devspace-runner\] started gen=1 marker=v0 .*world={world}", timeout=600)
        time.sleep(1.0)
    finally:
        r.stop()
    seen = {}
    line_re = re.compile(r"^\[rank (\d)\] R=(\d) I=(\d+) (x*)\|$")
    for raw in r.lines:
        line = raw.rstrip("\n")
        if " R=" not in line and not line.startswith("R="):
            continue
        m = line_re.match(line)
        assert m, f"split or merged line: {line!r}"
        rank, r2, i, pad = int(m.group(1)), int(m.group(2)), int(m.group(3)), m.group(4)
        assert rank == r2 and len(pad) == i % 97, line
        seen.setdefault(rank, set()).add(i)
    assert sorted(seen) == list(range(world)) and all(len(v) == lines for v in seen.values()), \
        {k: len(v) for k, v in seen.items()}
    text = r.text()
    # one start line per rank, each with its rank's prefix
    starts = sorted(int(m) for m in re.findall(r"^\[rank (\d)\] \[devspace-runner\] started gen=1 ", text, re.M))
    assert starts == list(range(world)), starts
    assert "[Gloo] Rank" not in text, [l for l in r.lines if "[Gloo]" in l][:3]
    assert text.count(f"group of {world} rank(s) connected") >= 1, text[-2000:]


def test_log_relay_flushes_a_last_line_without_a_newline():
    """What a rank wrote without a final newline goes out, with one, when its pipe closes; a line
    longer than the relay's limit goes out in pieces instead of growing without bound."""
    from devspace_amd.supervise import LogRelay

    import threading

    out_r, out_w = os.pipe()
    got = []

    def reader():
        while True:
            chunk = os.read(out_r, 1 << 20)
            if not chunk:
                return
            got.append(chunk)

    t = threading.Thread(target=reader, daemon=True)
    t.start()
    relay = LogRelay(2, out_fd=out_w)
    a_r, a_w = os.pipe()
    b_r, b_w = os.pipe()
    relay.add(0, a_r)
    relay.add(1, b_r)
    os.write(a_w, b"one\ntwo without newline")
    os.write(b_w, b"y" * (LogRelay.MAX_LINE + 10))
    os.close(a_w)
    os.close(b_w)
    assert relay.drain(5.0)
    os.close(out_w)
    t.join(5.0)
    lines = b"".join(got).decode().split("\n")
    assert "[rank 0] one" in lines and "[rank 0] two without newline" in lines, lines[:4]
    ys = [l for l in lines if l.startswith("[rank 1] ")]
    assert len(ys) == 2 and sum(len(l) - len("[rank 1] ") for l in ys) == LogRelay.MAX_LINE + 10


def test_log_relay_folds_a_warning_every_rank_prints_alike():
    """torch's C++ logger warnings that several ranks print alike at group start (c10d's
    "hostname of the client socket cannot be retrieved", once per rank) go out as one
    `[ranks 0-3]` line; a warning only some ranks print goes out once the hold ends, with those
    ranks; errors and ordinary lines are never held."""
    from devspace_amd.supervise import LogRelay

    import threading

    out_r, out_w = os.pipe()
    got = []

    def reader():
        while True:
            chunk = os.read(out_r, 1 << 20)
            if not chunk:
                return
            got.append(chunk)

    t = threading.Thread(target=reader, daemon=True)
    t.start()
    relay = LogRelay(4, out_fd=out_w)
    pipes = [os.pipe() for _ in range(4)]
    for r, (rd, _) in enumerate(pipes):
        relay.add(r, rd)
    warn = "[W1019 04:35:{:02d}.97835526{} socket.cpp:207] [c10d] The hostname of the client socket cannot be retrieved. err=-3\n"
    for r, (_, wr) in enumerate(pipes):
        os.write(wr, warn.format(r, r).encode())
        os.write(wr, f"plain {r}\n".encode())
    os.write(pipes[2][1], b"[W1019 04:35:09.1 other.cpp:1] only some ranks\n")
    os.write(pipes[3][1], b"[W1019 04:35:09.2 other.cpp:1] only some ranks\n")
    os.write(pipes[1][1], b"[E1019 04:35:09.3 other.cpp:2] an error\n")
    time.sleep(LogRelay.HOLD_S + 0.5)
    for _, wr in pipes:
        os.close(wr)
    assert relay.drain(5.0)
    os.close(out_w)
    t.join(5.0)
    lines = [l for l in b"".join(got).decode().split("\n") if l]
    hostname = [l for l in lines if "hostname of the client socket" in l]
    assert len(hostname) == 1 and hostname[0].startswith("[ranks 0-3] [W1019 04:35:00"), lines
    some = [l for l in lines if "only some ranks" in l]
    assert len(some) == 1 and some[0].startswith("[ranks 2,3] "), lines
    assert "[rank 1] [E1019 04:35:09.3 other.cpp:2] an error" in lines
    assert all(f"[rank {r}] plain {r}" in lines for r in range(4)), lines


def test_a_single_rank_logs_without_a_prefix(tmp_path):
    entry = tmp_path / "train.py"
    entry.write_text(CHATTY.format(lines=50))
    r = Runner(tmp_path, entry, 1, extra_args=("--log-every", "1000000", "--max-steps", "3"))
    try:
        r.until(r"^\[devspace-runner\] started gen=1 marker=v0", timeout=300)
    finally:
        r.stop()
    assert "R=0 I=49 " in r.text() and "[rank 0]" not in r.text()


SPIN_WAIT = '''
import hashlib
import os
import time

MARKER = "v0"
HANG = {hang!r}


def setup(ctx):
    return {{"n": 0}}


def step(ctx, state):
    if os.path.exists(HANG) and MARKER == "v0":
        # a native call that burns CPU with the GIL released and never comes back to Python, as a
        # spinning HIP or RCCL wait does
        hashlib.pbkdf2_hmac("sha256", b"x", b"salt", 2 * 10 ** 9)  # (a C int: at most 2^31 - 1)
    state["n"] += 1
    time.sleep(0.005)
    return {{"loss": state["n"]}}
'''


@pytest.mark.parametrize("wait_call,restarted", [("pbkdf2_hmac", True), ("", False)],
                         ids=["wait-call", "computation"])
def test_a_wait_that_spins_the_cpu_is_not_progress(tmp_path, wait_call, restarted):
    """HIP and RCCL waits may spin. A rank stuck in such a wait (here a builtin named in
    DEVSPACE_RUNNER_WAIT_CALLS, as `item`, `synchronize` and the collectives are by default) burns
    CPU at one Python position: that is not progress, and an edit restarts the group. The same CPU
    burn in a call that computes (a name not on the list) counts as progress, as before."""
    trigger = tmp_path.parent / (tmp_path.name + "-hang")
    entry = tmp_path / "train.py"
    entry.write_text(SPIN_WAIT.format(hang=str(trigger)))
    env = {"DEVSPACE_RUNNER_WAIT_CALLS": wait_call} if wait_call else {}
    r = Runner(tmp_path, entry, 1, extra_args=("--log-every", "50", "--rescue-every", "0.5", "--stuck-after", "2"),
               extra_env=env)
    try:
        r.until(r"started gen=1 marker=v0", timeout=180)
        r.until(r"rescue snapshot step=\d+ ", timeout=60)
        trigger.write_text("1")
        time.sleep(3.0)
        _set_marker(entry, "fixed")
        if restarted:
            r.until(r"made no progress for \d+ s at train.py:\d+ and the code changed since", timeout=60)
            r.until(r"started gen=1 marker=fixed", timeout=120)
        else:
            r.until(r"edit pending: rank=0 is making progress at train.py:\d+", timeout=60)
            time.sleep(1.0)
            assert "made no progress" not in r.text(), r.text()[-3000:]
    finally:
        r.stop()


DEVICE_WAIT = '''
import os
import time

import torch

MARKER = "v0"
HANG = {hang!r}


def setup(ctx):
    return {{"n": 0}}


def step(ctx, state):
    if os.path.exists(HANG) and MARKER == "v0" and not state.get("queued"):
        state["queued"] = True
        # about half a minute of GPU work queued, then a host read of its result: the main thread
        # waits inside `.item()` (a HIP stream sync) the whole time, at one Python position
        a = torch.randn(32768, 32768, device=ctx.device, dtype=torch.bfloat16)
        c = torch.empty_like(a)
        for _ in range(400):
            torch.matmul(a, a, out=c)
        c[0, 0].item()
    state["n"] += 1
    time.sleep(0.005)
    return {{"loss": state["n"]}}
'''


@pytest.mark.gpu
def test_a_rank_waiting_on_the_device_is_not_progress_on_the_gpu(tmp_path):
    """ADVICE r5 on the MI355X: a rank whose main thread sits in `.item()` behind GPU work (the
    position a rank hung in a collective is in) is still, whether HIP's wait spins the CPU or
    sleeps; an edit restarts the group. The rank's CPU use during the wait is printed."""
    trigger = tmp_path.parent / (tmp_path.name + "-hang")
    entry = tmp_path / "train.py"
    entry.write_text(DEVICE_WAIT.format(hang=str(trigger)))
    r = Runner(tmp_path, entry, 1, extra_args=("--log-every", "50", "--rescue-every", "0.5", "--stuck-after", "2",
                                              "--no-warm-standby"), gpu=True)
    try:
        r.until(r"started gen=1 marker=v0 .*device=cuda", timeout=300)
        r.until(r"rescue snapshot step=\d+ ", timeout=60)
        trigger.write_text("1")
        time.sleep(2.0)
        ranks = [p for p in psutil.Process(r.proc.pid).children(recursive=True) if "--worker" in " ".join(p.cmdline())]
        if ranks:
            t0 = ranks[0].cpu_times()
            time.sleep(2.0)
            t1 = ranks[0].cpu_times()
            print(f"rank CPU while waiting on the device: {(t1.user + t1.system - t0.user - t0.system) / 2.0:.2f} "
                  f"cores")
        _set_marker(entry, "fixed")
        r.until(r"made no progress for \d+ s at train.py:\d+ and the code changed since", timeout=60)
        r.until(r"started gen=1 marker=fixed", timeout=180)
    finally:
        r.stop()


MISMATCHED = '''
import os
import time

import torch
import torch.distributed as dist

MARKER = "v0"
HANG = {hang!r}


def setup(ctx):
    return {{"n": 0}}


def step(ctx, state):
    flag = torch.tensor([1.0 if ctx.rank == 0 and os.path.exists(HANG) else 0.0])
    dist.all_reduce(flag)
    if flag.item() and MARKER == "v0":
        # mismatched collective calls: rank 0 enters an all_reduce that rank 1 never joins, rank 1
        # waits for a message rank 0 never sends. Both block in the collective library for good.
        if ctx.rank == 0:
            dist.all_reduce(torch.ones(4))
        else:
            dist.recv(torch.empty(4), src=0)
    state["n"] += 1
    time.sleep(0.005)
    return {{"loss": state["n"]}}
'''


def test_ranks_deadlocked_in_mismatched_collectives_are_restarted_by_an_edit(tmp_path):
    """ranks hung in mismatched collectives (rank 0 in an all_reduce rank 1 never joins,
    rank 1 in a recv rank 0 never matches) stand inside wait calls. With --stuck-after, an edit
    restarts the group ("made no progress") instead of waiting on it forever. Two gloo ranks."""
    trigger = tmp_path.parent / (tmp_path.name + "-hang")
    entry = tmp_path / "train.py"
    entry.write_text(MISMATCHED.format(hang=str(trigger)))
    r = Runner(tmp_path, entry, 2, extra_args=("--log-every", "50", "--rescue-every", "0.5", "--stuck-after", "2"))
    try:
        r.until(r"started gen=1 marker=v0", timeout=180)
        r.until(r"rescue snapshot step=\d+ ", timeout=60)
        trigger.write_text("1")
        time.sleep(3.0)
        _set_marker(entry, "fixed")
        r.until(r"made no progress for \d+ s at train.py:\d+ and the code changed since", timeout=60)
        r.until(r"started gen=1 marker=fixed", timeout=180)
        r.until(r"step=\d+ gen=\d+ loss=", timeout=60)  # training again
    finally:
        r.stop()
