"""The runner's supervisor: one process per GPU rank, started, watched and stopped as a group.

Failure containment the reference gets from a fresh process per reload (nodemon restarts the
process tree, examples/quickstart/package.json:7; a redeploy replaces the pod, cmd/dev.go:225-234):
any rank exiting non-zero stops the whole group, which is started again from fresh processes.
"""

from __future__ import annotations

import os
import re
import signal
import subprocess
import sys
import threading
import time

from devspace_amd.changefeed import _ignored, _IGNORED_DIRS, _OUT_LOCK, PREFIX, _log, make_watcher
from devspace_amd.rescue import _default_rescue_dir, _drop_rescue_dir, _in_pod

_KIT_PARENT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_SPAWNED = []  # every rank process this supervisor started (Popen); the live ones are never strays


def _free_port() -> int:
    """An OS-assigned free TCP port on 127.0.0.1 for the group's rendezvous (never a fixed
    range: the pod may itself run under a torchrun whose master port is in use)."""
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]



# gloo's per-connection line, one per rank and group start ("[Gloo] Rank 3 is connected to 7 peer
# ranks. Expected number of connected peer ranks is : 7"): folded into one line per group
_GLOO_CONNECTED = re.compile(rb"^\[Gloo\] Rank \d+ is connected to (\d+) peer ranks")
# a warning or info line of torch's C++ logger ("[W1019 04:35:09.978355262 socket.cpp:207] [c10d]
# The hostname of the client socket cannot be retrieved. err=-3"): the same message from several
# ranks at group start is one line, `[ranks 0-7] ...`. Errors (E/F) are never held.
_CPP_LOG = re.compile(rb"^\[[WI]\d{4} [\d:.]+ (\S+:\d+)\] (.*)$")


def _rank_list(ranks):
    rs = sorted(ranks)
    if rs == list(range(rs[0], rs[-1] + 1)) and len(rs) > 2:
        return f"{rs[0]}-{rs[-1]}"
    return ",".join(str(r) for r in rs)


class LogRelay:
    """Every rank's stdout and stderr, through pipes, onto the supervisor's stdout as whole lines:
    `[rank N] <line>` when the group has more than one rank, the line as it is with one. Ranks
    writing at once never split or merge each other's lines (each line is one write by one
    thread, under the lock the supervisor's own lines take too). gloo's per-rank connection lines
    become one `group of N connected` line per group; a warning of torch's C++ logger that several
    ranks print alike (the same source line and message) is held up to HOLD_S and goes out once,
    `[ranks 0-7] <line>`. What a rank printed without a final newline
    is flushed, with one, when its pipe closes. (The reference reformats its children's output
    line by line too: pkg/devspace/builder/kaniko/util.go:18-87, pkg/util/processutil/pipe.go:46.)"""

    MAX_LINE = 1 << 16  # a longer line (no newline yet: a progress bar) goes out in pieces
    HOLD_S = 1.0  # how long a C++ logger warning waits for the same line from the other ranks

    def __init__(self, nproc, out_fd=None):
        self.nproc = max(1, nproc)
        self.prefix = self.nproc > 1
        self.out_fd = sys.stdout.fileno() if out_fd is None else out_fd
        self._mu = threading.Lock()
        self._open = {}  # fd -> [rank, pending bytes]
        self._gloo = 0
        self._held = {}  # (source, message) -> [deadline, first line, ranks] (relay thread only)
        self._wake_r, self._wake_w = os.pipe()
        self._thread = threading.Thread(target=self._run, name="devspace-log-relay", daemon=True)
        self._thread.start()

    def add(self, rank, fd):
        with self._mu:
            self._open[fd] = [rank, b""]
        os.write(self._wake_w, b"x")

    def drain(self, timeout=2.0):
        """Waits until every pipe added so far was read to its end (its ranks exited)."""
        end = time.monotonic() + timeout
        while time.monotonic() < end:
            with self._mu:
                if not self._open and not self._held:
                    return True
            time.sleep(0.005)
        return False

    def write_line(self, text):
        """One line of the supervisor's own, never inside a rank's line."""
        self._write((text.rstrip("\n") + "\n").encode())

    def _write(self, data):
        with _OUT_LOCK:
            try:
                sys.stdout.flush()  # what the supervisor printed through sys.stdout goes first
            except (OSError, ValueError):
                pass
            view = memoryview(data)
            while view:
                try:
                    n = os.write(self.out_fd, view)
                except InterruptedError:
                    continue
                except OSError:
                    return  # nobody reads our stdout any more: drop, never block the ranks
                view = view[n:]

    def _emit(self, rank, line):
        m = _GLOO_CONNECTED.match(line)
        if m:
            with self._mu:
                self._gloo += 1
                done = self._gloo >= self.nproc
                if done:
                    self._gloo = 0
            if done:
                self._write(f"{PREFIX} group of {self.nproc} rank(s) connected (gloo)\n".encode())
            return
        if self.prefix:
            c = _CPP_LOG.match(line)
            if c:
                key = c.groups()
                h = self._held.get(key)
                if h is None:
                    h = self._held[key] = [time.monotonic() + self.HOLD_S, line, set()]
                h[2].add(rank)
                if len(h[2]) >= self.nproc:
                    self._flush_held(key)
                return
        self._write(((b"[rank %d] " % rank) if self.prefix else b"") + line + b"\n")

    def _flush_held(self, key):
        _, line, ranks = self._held.pop(key)
        who = b"[rank %d] " % next(iter(ranks)) if len(ranks) == 1 else f"[ranks {_rank_list(ranks)}] ".encode()
        self._write(who + line + b"\n")

    def _flush_expired(self, all_=False):
        now = time.monotonic()
        for key in [k for k, h in self._held.items() if all_ or h[0] <= now]:
            self._flush_held(key)

    def _run(self):
        import select

        while True:
            with self._mu:
                fds = list(self._open)
            if self._held and not fds:
                self._flush_expired(all_=True)  # every rank has exited: nothing more to wait for
            wait = None
            if self._held:
                wait = max(0.0, min(h[0] for h in self._held.values()) - time.monotonic())
            try:
                ready, _, _ = select.select(fds + [self._wake_r], [], [], wait)
            except (OSError, ValueError):
                ready = []
            if self._held:
                self._flush_expired()
            for fd in ready:
                if fd == self._wake_r:
                    os.read(self._wake_r, 4096)
                    continue
                try:
                    data = os.read(fd, 65536)
                except OSError:
                    data = b""
                with self._mu:
                    rank, pending = self._open[fd]
                if not data:
                    if pending:
                        self._emit(rank, pending)
                    with self._mu:
                        del self._open[fd]
                    os.close(fd)
                    continue
                pending += data
                *lines, pending = pending.split(b"\n")
                while len(pending) > self.MAX_LINE:
                    lines.append(pending[:self.MAX_LINE])
                    pending = pending[self.MAX_LINE:]
                for line in lines:
                    self._emit(rank, line)
                with self._mu:
                    self._open[fd][1] = pending


_RELAY = None  # the supervisor's LogRelay (one per supervisor: ranks of every group)


def _relay(nproc):
    global _RELAY
    if _RELAY is None:
        _RELAY = LogRelay(nproc)
    return _RELAY


def _spawn_group(args, port, status_fd=None, standby=False):
    """One process per rank, each the leader of its own session and process group (so the group's
    whole process tree can be stopped, see _stop_group); `standby`: warm standbys that import torch
    and then wait on stdin for `go <port>` (see _promote). Nothing runs in the child between fork
    and exec (no preexec_fn: the supervisor has threads); the worker ties its life to this
    supervisor itself (runner.die_with_supervisor, DEVSPACE_SUPERVISOR_PID). Its stdout and stderr
    go through this supervisor's LogRelay."""
    procs = []
    relay = _relay(args.nproc)
    for r in range(max(1, args.nproc)):
        env = dict(os.environ)
        env.update(
            RANK=str(r),
            WORLD_SIZE=str(max(1, args.nproc)),
            LOCAL_RANK=str(r),
            MASTER_ADDR="127.0.0.1",
            MASTER_PORT=str(port),
            HSA_ENABLE_IPC_MODE_LEGACY=env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
        )
        if status_fd is not None:
            env["DEVSPACE_RUNNER_STATUS_FD"] = str(status_fd)
        # the kit is a package: installed, in the checkout, or vendored next to train.py by
        # `devspace init` (rocm-pytorch template); its parent directory goes on the ranks' path
        env["PYTHONPATH"] = os.pathsep.join(filter(None, [_KIT_PARENT, env.get("PYTHONPATH")]))
        env["DEVSPACE_SUPERVISOR_PID"] = str(os.getpid())
        cmd = [sys.executable, "-m", "devspace_amd.runner", "--worker"] + (["--standby"] if standby else []) + \
            _forward(args)
        out_r, out_w = os.pipe()
        try:
            procs.append(subprocess.Popen(cmd, env=env, pass_fds=(status_fd,) if status_fd is not None else (),
                                          stdin=subprocess.PIPE if standby else None, stdout=out_w, stderr=out_w,
                                          start_new_session=True))
        except BaseException:
            os.close(out_r)
            raise
        finally:
            os.close(out_w)
        relay.add(r, out_r)
    _SPAWNED[:] = [p for p in _SPAWNED if p.returncode is None] + procs
    return procs


def _live_spawned() -> set:
    """pids of the rank processes this supervisor started that have not exited (reaped here)."""
    return {p.pid for p in _SPAWNED if p.poll() is None}


def _promote(procs, port) -> bool:
    """Turns a warm standby group into the running group (rendezvous on `port`); False when one of
    its processes is gone (then it is not used)."""
    if any(p.poll() is not None for p in procs):
        return False
    try:
        for p in procs:
            p.stdin.write(f"go {port}\n".encode())
            p.stdin.close()
    except OSError:
        return False
    return True


def _discard(group) -> None:
    procs, status_r = group
    for p in procs:
        try:
            p.stdin.close()  # a standby waiting for `go` exits on EOF
        except (OSError, AttributeError):
            pass
    _stop_group(procs)
    os.close(status_r)


def become_subreaper() -> bool:
    """prctl(PR_SET_CHILD_SUBREAPER): what a rank's processes leave behind when the rank dies (an
    eval subprocess, DataLoader workers, a profiler that daemonised) is re-parented to this
    supervisor instead of to init, so the supervisor can stop and reap it with the group. In a pod
    the supervisor is usually PID 1 and gets them anyway; this makes every other case the same."""
    try:
        import ctypes

        return ctypes.CDLL("libc.so.6", use_errno=True).prctl(36, 1, 0, 0, 0) == 0
    except (OSError, AttributeError):  # pragma: no cover - not Linux/glibc
        return False


def _children():
    """{pid: state letter} of this process's children, from /proc (no psutil in every image)."""
    me, out = os.getpid(), {}
    try:
        names = os.listdir("/proc")
    except OSError:  # pragma: no cover
        return out
    for name in names:
        if not name.isdigit():
            continue
        try:
            with open(f"/proc/{name}/stat", "rb") as f:
                data = f.read()
        except OSError:
            continue
        rest = data[data.rfind(b")") + 2:].split()  # after "pid (comm) "
        if len(rest) > 1 and int(rest[1]) == me:
            out[int(name)] = rest[0].decode()
    return out


def _reap(pid) -> None:
    try:
        os.waitpid(pid, os.WNOHANG)
    except ChildProcessError:
        pass


def reap_strays(keep=None) -> int:
    """Reaps the exited processes this supervisor adopted (children it did not start: not in
    `keep`, by default the live rank processes); live ones are left alone while their group runs.
    Returns how many it reaped."""
    keep = _live_spawned() if keep is None else keep
    n = 0
    for pid, st in _children().items():
        if pid not in keep and st == "Z":
            _reap(pid)
            n += 1
    return n


def kill_strays(keep=None, grace_s=0.5) -> list:
    """Stops every process this supervisor adopted that it did not start (not in `keep`): SIGTERM,
    SIGKILL after `grace_s`, reaped. Killing one re-parents its own children here, so this runs
    until none is left (bounded). Returns the pids it ended."""
    keep = _live_spawned() if keep is None else keep
    ended, termed = [], {}
    deadline = time.monotonic() + grace_s + 5.0
    while True:
        strays = {pid: st for pid, st in _children().items() if pid not in keep}
        if not strays or time.monotonic() > deadline:
            return ended
        now = time.monotonic()
        for pid, st in strays.items():
            if st == "Z":
                _reap(pid)
                ended.append(pid)
                continue
            try:
                if pid not in termed:
                    os.kill(pid, signal.SIGTERM)
                    termed[pid] = now
                elif now - termed[pid] >= grace_s:
                    os.kill(pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        time.sleep(0.01)


def _group_alive(pgid) -> bool:
    try:
        os.killpg(pgid, 0)
        return True
    except (ProcessLookupError, PermissionError):
        return False


def _signal_group(pgid, sig) -> None:
    try:
        os.killpg(pgid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def _stop_group(procs, grace_s=2.0):
    """Stops a group and everything its ranks started.

    1. SIGTERM to each rank process alone (the ranks agree to stop at the next step boundary,
       with a last snapshot; their DataLoader workers keep serving until then);
    2. after `grace_s`, SIGKILL to each rank's whole process group (a rank blocked inside a
       collective whose peer is gone never returns to Python to see the SIGTERM, and the rank's
       children go with it);
    3. a rank that exited in time may have left children in its process group: SIGTERM to the
       group, SIGKILL after 0.5 s;
    4. what escaped the process groups (a child that started its own session) was re-parented to
       this supervisor (a subreaper) when its parent died: stopped and reaped as well, except the
       rank processes of another group (a warm standby)."""
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.monotonic() + grace_s
    for p in procs:
        try:
            p.wait(max(0.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            _signal_group(p.pid, signal.SIGKILL)
            p.wait()
    left = [p.pid for p in procs if _group_alive(p.pid)]
    if left:
        for pgid in left:
            _signal_group(pgid, signal.SIGTERM)
        t_kill = time.monotonic() + 0.5
        while left and time.monotonic() < t_kill:
            reap_strays()
            left = [g for g in left if _group_alive(g)]
            time.sleep(0.01)
        for pgid in left:
            _signal_group(pgid, signal.SIGKILL)
    kill_strays()


def restart_main(args) -> int:
    """Restart-on-change mode (what the reference's nodemon-style dev entrypoints do): every
    edit kills the process group and cold-starts it. Kept as the reference-equivalent baseline."""
    watch_dir = os.path.abspath(args.watch or os.path.dirname(os.path.abspath(args.entry)))
    watcher = make_watcher(watch_dir)
    port = args.port or _free_port()
    become_subreaper()
    procs = _spawn_group(args, port)
    try:
        while True:
            changed = [p for p in watcher.poll(200) if not _ignored(p)]
            if changed:
                _log(f"change detected ({len(changed)} files), restarting")
                _stop_group(procs)
                port = port + 1 if args.port else _free_port()
                procs = _spawn_group(args, port)
            elif all(p.poll() is not None for p in procs) and not args.keep_alive:
                return max(p.returncode for p in procs)
    finally:
        _stop_group(procs)
        watcher.close()
        if _RELAY is not None:
            _RELAY.drain()  # the ranks' last lines


class Beat:
    """One rank's last heartbeat (sent once a second by a thread of the rank, see
    runner._Heartbeat): what its main thread is doing and since when, in this process's clock."""

    __slots__ = ("t", "step", "phase", "since", "longest", "still", "snap", "where")

    def __init__(self, t, step=0, phase="start", since=None, longest=0.0, still=0.0, snap=0, where="?"):
        self.t = t  # when it arrived
        self.step = step
        self.phase = phase  # start | reload | step | boundary | idle
        self.since = t if since is None else since  # when the phase began
        self.longest = longest  # longest steady-state step completed so far, seconds
        self.still = still  # seconds the main thread's Python position had not moved, at `t`
        self.snap = snap  # step of the newest committed rescue snapshot (0: none)
        self.where = where  # the main thread's innermost user frame, file:line

    @classmethod
    def parse(cls, parts, now):
        """`hb <rank> <step> <phase> <in_phase_s> <longest_s> <still_s> <snap_step> <where>`"""
        try:
            return cls(now, int(parts[2]), parts[3], now - float(parts[4]), float(parts[5]), float(parts[6]),
                       int(parts[7]), " ".join(parts[8:]) or "?")
        except (IndexError, ValueError):
            return None


class _GroupWatch:
    """The supervisor's view of one running group: exits (any rank, not all), the workers'
    status lines (`ready <rank>`, `fail <rank> <gen>`, heartbeats) and whether the synced tree
    changed since the group started (then a failed group restarts at once: the fix may already be
    there)."""

    BEAT_LATE = 3.0  # seconds without a heartbeat (sent every second) before silence counts

    def __init__(self, procs, status_r, watcher, stuck_after=0.0):
        self.procs = procs
        self.status_r = status_r
        self.watcher = watcher
        self.ready = set()
        self.failed = []  # ranks in the order their `fail` lines arrived
        self.changed = False
        self.last_change = 0.0  # monotonic time of the newest change of the synced tree
        self.stuck_after = stuck_after
        self.beat = {}  # rank -> Beat
        self.reported = False  # the long step in flight was reported (once per episode)
        self._buf = b""
        self._next_scan = 0.0
        self._next_reap = 0.0

    def _read_status(self, timeout):
        import select

        r, _, _ = select.select([self.status_r], [], [], timeout)
        if not r:
            return
        try:
            chunk = os.read(self.status_r, 65536)
        except BlockingIOError:
            return
        self._buf += chunk
        *lines, self._buf = self._buf.split(b"\n")
        now = time.monotonic()
        for line in lines:
            parts = line.decode(errors="replace").split()
            if len(parts) >= 2 and parts[0] == "ready":
                self.ready.add(int(parts[1]))
                self.beat.setdefault(int(parts[1]), Beat(now, phase="boundary"))
            elif len(parts) >= 2 and parts[0] == "fail":
                self.failed.append(int(parts[1]))
            elif len(parts) >= 9 and parts[0] == "hb":
                b = Beat.parse(parts, now)
                if b is not None:
                    self.beat[int(parts[1])] = b

    def _scan_tree(self):
        now = time.monotonic()
        if now < self._next_scan:
            return
        self._next_scan = now + 0.25
        if [p for p in self.watcher.poll(0) if not _ignored(p)]:
            self.changed = True
            self.last_change = now

    def assess(self, now=None):
        """The stuck-step rule. A group is restarted for being stuck only on evidence that it is:
          * an edit landed while the ranks were inside a steady-state step (never during setup(),
            a reload or the first step of new code: loading a model may take minutes);
          * the step has run longer than max(--stuck-after, 10 x the longest step completed so
            far) — a periodic eval that ran once before is not stuck the next time;
          * no rank's main thread has moved (its Python position, sampled 4x a second) for
            --stuck-after: a deadlock, a collective whose peer is gone or a `sleep` — a step that
            runs Python (an eval loop, a checkpoint save) is busy, and so is its group: the peers
            waiting for it in a barrier wait for progress;
          * a committed rescue snapshot exists, so the restart resumes from it, never from setup().
        Returns ('stuck', rank, seconds, where) to restart, ('wait', rank, seconds, where, why) the
        first time a long step with an edit pending is not restarted (logged once), or None."""
        if not self.stuck_after or len(self.ready) < len(self.procs) or len(self.beat) < len(self.procs):
            return None
        now = time.monotonic() if now is None else now
        beats = sorted(self.beat.items())
        # a rank silent since a beat at a step boundary is inside the next step (the loop goes
        # straight from one to the other; a native call holding the GIL starves the beat thread)
        beats = [(r, Beat(b.t, b.step, "step", b.t, b.longest, b.still, b.snap, b.where))
                 if b.phase == "boundary" and now - b.t > self.BEAT_LATE else (r, b) for r, b in beats]
        pending = [(r, b) for r, b in beats if b.phase == "step" and self.last_change > b.since]
        if not pending:
            self.reported = False
            return None
        rank, b = max(pending, key=lambda rb: now - rb[1].since)
        secs = now - b.since
        if secs <= max(self.stuck_after, 10.0 * b.longest):
            return None
        # a beat comes once a second; longer silence counts as stillness (a main thread holding the
        # GIL in C keeps the heartbeat thread from running)
        moving = [(r, x) for r, x in beats
                  if x.still + (now - x.t if now - x.t > self.BEAT_LATE else 0.0) < self.stuck_after]
        if not moving and len(pending) == len(beats) and b.snap > 0:
            return ("stuck", rank, secs, b.where)
        if self.reported:
            return None
        self.reported = True
        if moving:
            r, x = moving[0]
            why = f"rank={r} is making progress at {x.where}: not restarting"
        elif len(pending) < len(beats):
            why = "not every rank is inside the step: not restarting"
        else:
            why = "no rescue snapshot to resume from yet: not restarting (training would restart from setup())"
        return ("wait", rank, secs, b.where, why)

    def wait(self, on_ready=None):
        """('done', codes) when every rank exited 0; ('failed', rank, code) at the first rank
        that exits otherwise (the root cause: the first `fail` line, else the first exit seen);
        ('stuck', rank, seconds, where) for a group stuck in a step across an edit (see assess).
        `on_ready()` runs once, when every rank finished its first step."""
        while True:
            self._read_status(0.02)
            self._scan_tree()
            now = time.monotonic()
            if now >= self._next_reap:  # what a rank's children left when they exited
                self._next_reap = now + 1.0
                reap_strays()
            if on_ready is not None and len(self.ready) == len(self.procs):
                on_ready()
                on_ready = None
            verdict = self.assess(now)
            if verdict is not None and verdict[0] == "stuck":
                return verdict
            if verdict is not None:
                _, rank, secs, where, why = verdict
                _log(f"rank={rank} in step for {secs:.0f} s at {where}; edit pending: {why}")
            codes = [p.poll() for p in self.procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                self._read_status(0)
                root = next(((r, codes[r]) for r in self.failed if codes[r] not in (None, 0)), bad[0])
                return ("failed",) + root
            if all(c == 0 for c in codes):
                return ("done", codes)


def _wait_for_change(watcher, already=False):
    """nodemon's "app crashed - waiting for file changes before starting": block until the synced
    tree changes (a settled write, not a temp file)."""
    if already:
        return
    while not [p for p in watcher.poll(500) if not _ignored(p)]:
        pass


def supervisor_main(args) -> int:
    """Spawn one worker per GPU (torchrun-style env) and contain failures: any rank exiting
    non-zero stops the whole group (its peers may be blocked in a collective with it), which is
    started again from fresh processes — at once if it had come up (its ranks all finished a
    first step) and there are restarts left since the last edit, after the next edit otherwise."""
    if args.restart:
        return restart_main(args)
    nproc = max(1, args.nproc)
    if os.environ.get("DEVSPACE_RUNNER_INPROCESS") == "1":
        # one rank in this process (a debugger, a profiler that follows one process): no
        # supervisor, so a hard crash ends the runner (and the container) as a plain script would
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("LOCAL_RANK", "0")
        from devspace_amd.runner import worker_main

        return worker_main(args)
    # One rank is supervised too: an exception in step() pauses it in its warm process, but a
    # hard crash (a segfault in an extension, a GPU memory fault that aborts the process, the
    # OOM killer) would otherwise end the container and put it into CrashLoopBackOff; here the
    # warm standby takes over in about a second and resumes from the last snapshot.
    watch_dir = os.path.abspath(args.watch or os.path.dirname(os.path.abspath(args.entry)))
    watcher = make_watcher(watch_dir)
    port = args.port or _free_port()
    restarts = 0  # restarts since the last edit
    # the ranks' rescue snapshots live as long as this supervisor (a restarted group resumes
    # from them) and, in a pod, as long as the pod (a restarted container resumes from them); in
    # /dev/shm: the pod's memory-backed volume, sized per GPU by the chart
    rescue_dir = args.rescue_dir or _default_rescue_dir(args.entry, nproc)
    os.environ["DEVSPACE_RESCUE_DIR"] = rescue_dir
    _IGNORED_DIRS.append(os.path.abspath(rescue_dir))

    def _term(*_):
        raise KeyboardInterrupt

    signal.signal(signal.SIGTERM, _term)  # pod deletion / kill: stop the ranks, then exit
    become_subreaper()  # what the ranks leave behind comes back here to be stopped
    procs = []
    clean = False  # stopped or finished: no later run resumes from these snapshots
    standby = []  # [(procs, status_r)]: a warm group that replaces a failed one

    def _new_group(as_standby=False):
        status_r, status_w = os.pipe()
        os.set_blocking(status_r, False)
        group = (_spawn_group(args, port, status_w, standby=as_standby), status_r)
        os.close(status_w)
        return group

    def _warm_up():  # once the running group is up: its start-up is not slowed by the standby's
        if args.warm_standby and not standby:
            standby.append(_new_group(as_standby=True))

    try:
        while True:
            group = standby.pop() if standby else None
            if group is not None and not _promote(group[0], port):
                _discard(group)
                group = None
            procs, status_r = group or _new_group()
            gw = _GroupWatch(procs, status_r, watcher, stuck_after=args.stuck_after)
            outcome = gw.wait(on_ready=_warm_up)
            if outcome[0] == "done":
                os.close(status_r)
                clean = True
                return 0
            if outcome[0] == "stuck":
                _, rank, secs, where = outcome
                _log(f"rank={rank} made no progress for {secs:.0f} s at {where} and the code changed since (stuck in "
                     f"a step?): restarting the group of {nproc} with the new code" +
                     (" from the warm standby" if standby else ""))
                _stop_group(procs)  # the normal grace: a rank that does get out writes no half files
                os.close(status_r)
                restarts = 0
                port = port + 1 if args.port else _free_port()
                continue
            _, rank, code = outcome
            _stop_group(procs, grace_s=0.2)  # the peers of a failed group: nothing left to finish
            os.close(status_r)
            came_up = len(gw.ready) == nproc
            if gw.changed:
                restarts = 0
            restarts += 1
            if came_up and restarts <= args.max_restarts:
                _log(f"rank={rank} exited with code {code}: restarting the group of {nproc} "
                     f"({restarts}/{args.max_restarts} since the last edit)" + (" from the warm standby" if standby else ""))
            else:
                why = "before every rank finished a first step" if not came_up else \
                    f"{args.max_restarts} restarts without an edit"
                _log(f"rank={rank} exited with code {code} {why}: waiting for a file change "
                     f"before starting the group again")
                _wait_for_change(watcher, already=gw.changed)
                restarts = 0
                _log(f"change detected: restarting the group of {nproc}" + (" from the warm standby" if standby else ""))
            port = port + 1 if args.port else _free_port()
    except KeyboardInterrupt:
        # with a --rescue-dir the ranks take a last snapshot before they exit: give them the time
        _stop_group(procs, grace_s=30.0 if args.rescue_dir and args.rescue_every > 0 else 2.0)
        clean = True
        return 130
    finally:
        for group in standby:
            _discard(group)
        watcher.close()
        if _RELAY is not None:
            _RELAY.drain()  # the ranks' last lines
        if not args.rescue_dir and (clean or not _in_pod()):
            _drop_rescue_dir(rescue_dir)


def _forward(args):
    out = ["--watch", args.watch or "", "--log-every", str(args.log_every), "--max-steps", str(args.max_steps),
           "--gemm-tuning", args.gemm_tuning]
    if not args.train:
        out.append("--no-train")
    if not args.preempt:
        out.append("--no-preempt")
    out += ["--preempt-drain-ms", str(args.preempt_drain_ms), "--group-timeout", str(args.group_timeout),
            "--rescue-every", str(args.rescue_every)]
    if args.rescue_dir:  # (the ranks find it in DEVSPACE_RESCUE_DIR too; this says it was asked for)
        out += ["--rescue-dir", args.rescue_dir]
    return out + [args.entry]
