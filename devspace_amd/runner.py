"""Hot-reload runner for GPU workloads inside a dev pod (the MI355X side of `devspace dev`).

The reference restarts the container process on every synced change (its examples use
nodemon; auto-reload redeploys, cmd/dev.go:285-301). For PyTorch-on-ROCm pods a restart
costs a `import torch` + HIP context creation + weight re-upload to HBM on every edit. This
runner keeps one long-lived process per GPU (one-process-per-GPU, RCCL over xGMI for N>1),
keeps user state (model/optimizer tensors resident in HBM, the process group and its RCCL
communicators) and swaps only the *code* at a step boundary:

    user module (e.g. train.py):
        MARKER = "v1"                 # optional, echoed in the reload line
        def setup(ctx): -> state      # run once (or again when SETUP_VERSION changes)
        def step(ctx, state): -> dict # called repeatedly; re-bound on every edit

    python -m devspace_amd.runner --nproc N --watch /app train.py

On every source change each rank recompiles the module from disk; the ranks agree on the
code generation with one tiny MAX all-reduce per step (so collectives inside `step` stay
matched) over a separate gloo (CPU) group: the control plane never enqueues work on a GPU
stream nor waits for one, so the host keeps running ahead of the GPUs. Rank 0 prints

    [devspace-runner] reloaded gen=3 marker=v1 step=120 loss=... step_ms=... reload_ms=...

A module without `step()` is treated as a plain script and re-executed in the warm
interpreter on each change.

Failure containment (the reference gets it from a fresh process per reload: nodemon in
examples/quickstart/package.json:7, the redeploy loop of cmd/dev.go:225-234,284-302):
  * same bytes on every rank: at each agreed generation rank 0 reads the entry file and
    broadcasts its bytes over the gloo control group; every rank compiles exactly those bytes.
    User modules the entry imports from the synced tree go through a source overlay that records
    the bytes each rank compiled; the ranks compare one code digest, and when a helper changed
    between their reads rank 0's recorded sources are re-sent and compiled everywhere.
  * agreed reload failures: a load that fails on any rank keeps the previous generation on all.
  * agreed step failures: with several ranks, an exception in setup()/step() is fatal for the
    group: the failing rank logs `rank=<r>` with the traceback and exits non-zero; the supervisor
    stops the others (blocked in a collective, or not) and starts a fresh group of child
    processes. A group that fails before its first step completes (the code itself is broken)
    waits for the next edit before starting again, as nodemon does ("app crashed - waiting for
    file changes"). A single rank pauses training after a failed step and resumes with the next
    edit (process, model and optimizer state stay); one rank is supervised as well, so a hard
    crash (segfault, GPU fault, OOM kill) is restarted in the container, not by the kubelet.
  * state survives a group restart: every --rescue-every seconds (60) the ranks snapshot their
    training state into /dev/shm at one agreed step boundary; a restarted group resumes from the
    newest step every rank holds instead of from scratch (`Rescue`).
  * restarts are fast: once a group is up, the supervisor keeps a warm standby group (torch and
    the group's libraries imported, no GPU touched) that replaces a failed one.
  * a stop takes the whole process tree: ranks lead their own sessions and the supervisor is a
    child subreaper (devspace_amd/supervise.py).
  * stuck steps are restarted on evidence only (supervise._GroupWatch.assess; the heartbeat
    thread, _Heartbeat below): a long healthy step (an evaluation, a checkpoint save) is left
    to finish and the edit applies after it.

The supervisor lives in devspace_amd/supervise.py, the snapshots in devspace_amd/rescue.py and
the change detection in devspace_amd/changefeed.py; this module is the rank's loop.

Preemptible steps: a step may call `ctx.preempt_point()` between its phases (e.g. between
forward and backward). The point abandons the rest of the step when a newer version of the
code is waiting — before the optimizer touched any state. With several ranks the decision is
collective (rank 0's view, agreed over the gloo group at the point), so every rank leaves the
step at the same point and the collectives of the next step stay matched. For long steps
(loop period >= --preempt-drain-ms, default 20 ms) the point also drains the GPU work queued
so far while watching the change feed, so an edit waits only for the phase in flight instead
of the whole queued step (the host otherwise runs a full step ahead of the GPU and blocks in
`loss.item()`). The drain costs one launch bubble per point, which on MI355X outweighs the
gain for millisecond steps (measured on the 3.9 ms TinyLM step: p50 6.2-6.4 ms with the drain
vs 6.0-6.06 ms without), hence the threshold.
"""

from __future__ import annotations

import argparse
import hashlib
import importlib.machinery
import importlib.util
import os
import signal
import sys
import threading
import time
import traceback
import types

from devspace_amd.changefeed import (  # noqa: F401  (re-exported: tests and tools use runner.*)
    PREFIX, SYNC_TMP_SUFFIX, ChangeFeed, _IGNORED_DIRS, _ignored, _InotifyWatcher, _log, _PollWatcher, make_watcher)
from devspace_amd.rescue import (  # noqa: F401
    Rescue, RescueSkipped, _default_rescue_dir, _drop_rescue_dir, _in_pod, _rescue_final, _rescue_finish,
    _rescue_restore)

# exit codes of a worker that leaves its group on purpose (the supervisor restarts the group)
EXIT_STEP_FAILED = 3
EXIT_GROUP_LOST = 4
EXIT_LOAD_FAILED = 5


def _status(msg: str) -> None:
    """One line to the supervisor over the status pipe it handed down (DEVSPACE_RUNNER_STATUS_FD):
    `ready <rank>` once the first step ran, `fail <rank> <gen>` before a deliberate exit."""
    fd = os.environ.get("DEVSPACE_RUNNER_STATUS_FD")
    if not fd:
        return
    try:
        os.write(int(fd), (msg + "\n").encode())
    except OSError:  # supervisor gone: PDEATHSIG ends this process anyway
        pass


def _fatal(code: int) -> None:
    """Leave the group now: no destroy_process_group (it would wait on peers that may sit in a
    collective this rank never joins), no atexit hooks that touch the device."""
    try:
        sys.stdout.flush()
        sys.stderr.flush()
    finally:
        os._exit(code)



class Preempted(BaseException):
    """Raised by `Context.preempt_point()` when newer code is waiting: the rest of the old
    step is skipped and the runner swaps the code right away. A BaseException (like
    KeyboardInterrupt) so a user step's generic `except Exception` cannot swallow it and carry
    on into the optimizer update."""


class Agreement:
    """Control plane of a multi-rank group: the code generation at each step boundary and the
    preemption decision at each `preempt_point()`, agreed with MAX all-reduces of CPU tensors
    over a dedicated gloo process group. Nothing here touches a GPU stream or reads a device
    tensor (no `.item()` / `.tolist()` on the device: those would stall the host on every
    step). Every rank must make the same sequence of calls."""

    def __init__(self, dist, group=None, timeout=None):
        import torch

        self.dist = dist
        if group is None:
            # a collective waiting longer than `timeout` raises: a rank stuck in a step (or gone
            # without a trace) ends the group instead of hanging it (the supervisor restarts it)
            group = dist.new_group(backend="gloo", **({"timeout": timeout} if timeout is not None else {}))
        self.group = group
        # [newest generation, helper modules changed, a rank was told to stop (SIGTERM),
        #  a rescue snapshot is due (rank 0's timer), a rank is still writing its snapshot,
        #  a rank's snapshot failed]
        self.ctl = torch.zeros(6, dtype=torch.int64)
        self.flag = torch.zeros(1, dtype=torch.int64)
        self.calls = 0
        # the last boundary's agreed snapshot state: start one / some rank still writing / failed
        self.snap = self.writing = self.write_failed = False

    def boundary(self, pending_gen: int, helper_pending: bool, stop: bool = False, snap: bool = False,
                 writing: bool = False, write_failed: bool = False):
        """(agreed generation, helper modules changed, stop): all ranks leave the loop at the
        same boundary when any of them got SIGTERM, so none is left waiting in a collective
        of a step the others never start. The rescue snapshot's state rides along
        (`self.snap`, `self.writing`, `self.write_failed`)."""
        self.ctl[0] = pending_gen
        self.ctl[1] = int(helper_pending)
        self.ctl[2] = int(stop)
        self.ctl[3] = int(snap)
        self.ctl[4] = int(writing)
        self.ctl[5] = int(write_failed)
        self.dist.all_reduce(self.ctl, op=self.dist.ReduceOp.MAX, group=self.group)
        self.calls += 1
        self.snap, self.writing, self.write_failed = bool(self.ctl[3]), bool(self.ctl[4]), bool(self.ctl[5])
        return int(self.ctl[0]), bool(self.ctl[1]), bool(self.ctl[2])

    def preempt(self, pending: bool) -> bool:
        self.flag[0] = int(pending)
        self.dist.all_reduce(self.flag, op=self.dist.ReduceOp.MAX, group=self.group)
        self.calls += 1
        return bool(self.flag[0])

    def share(self, obj):
        """Rank 0's `obj` on every rank (pickled, over the gloo group): the code bytes of a
        generation, so no rank compiles what it happened to read from disk."""
        box = [obj]
        self.dist.broadcast_object_list(box, src=0, group=self.group)
        self.calls += 1
        return box[0]

    def gather(self, obj) -> list:
        """Every rank's `obj`, in rank order, on every rank (load outcomes and code digests)."""
        out = [None] * self.dist.get_world_size(self.group)
        self.dist.all_gather_object(out, obj, group=self.group)
        self.calls += 1
        return out


class Context:
    """What user code sees: rank/device info, a tiny logging helper and the preemption point."""

    def __init__(self, rank: int, world_size: int, local_rank: int, device):
        self.rank = rank
        self.world_size = world_size
        self.local_rank = local_rank
        self.device = device
        self.step = 0
        self.generation = 0
        self.distributed = world_size > 1
        self._feed = None  # ChangeFeed when preemption is enabled
        self._event = None  # one reusable HIP event for the drain
        self._period_ms = 0.0  # steady-state loop period (set by the runner)
        self._drain_min_ms = 20.0  # drain at preemption points only for steps at least this long
        self._agree = None  # Agreement when world > 1

    def log(self, msg: str) -> None:
        if self.rank == 0:
            _log(msg)

    def error(self, msg: str) -> None:
        """Errors go out from every rank, tagged with it: a failure on rank 5 of 8 must not be
        invisible because only rank 0 prints."""
        _log(f"rank={self.rank} {msg}" if self.world_size > 1 else msg)

    def preempt_point(self) -> None:
        """Cooperative reload point inside `step()`: raises Preempted if a newer version of the
        code is waiting. For long steps it first drains the GPU work queued so far while polling
        the change feed. With several ranks the ranks decide together (rank 0's change feed,
        one gloo all-reduce of a CPU flag) so they all leave the step at the same point; the
        drain then runs to completion before the decision (a decision polled during the drain
        would differ between ranks). No-op when preemption is off."""
        feed = self._feed
        if feed is None:
            return
        long_step = self.device.type == "cuda" and self._period_ms >= self._drain_min_ms
        if self._agree is not None:
            if long_step:
                self._drain(None)
            if self._agree.preempt(self.rank == 0 and feed.pending()):
                raise Preempted()
            return
        if feed.pending():
            raise Preempted()
        if long_step:
            self._drain(feed)

    def _drain(self, feed) -> None:
        import torch

        if self._event is None:
            self._event = torch.cuda.Event()
        ev = self._event
        ev.record()
        while not ev.query():
            if feed is not None and feed.pending():
                raise Preempted()
            time.sleep(0)  # releases the GIL: the change feed thread can post the edit



def purge_user_modules(watch_dir: str) -> list:
    """Drops the modules imported from the synced tree (helpers the entry file imports) from
    sys.modules, so the next exec of the entry file imports their edited versions; packages
    installed in the image, compiled extensions and this runner itself stay. Called only when a
    helper .py file changed: a plain prefix test first, realpath only for the candidates (the
    import cache of a torch process holds thousands of modules)."""
    prefixes = tuple({os.path.abspath(watch_dir) + os.sep, os.path.realpath(watch_dir) + os.sep})
    root = os.path.realpath(watch_dir) + os.sep
    kit = os.path.dirname(os.path.realpath(__file__)) + os.sep  # the runner's own package (in /app in a pod)
    gone = []
    for name, m in list(sys.modules.items()):
        f = getattr(m, "__file__", None)
        if not f or name == "__main__" or not f.endswith(".py") or not f.startswith(prefixes):
            continue
        rf = os.path.realpath(f)
        if rf.startswith(root) and not rf.startswith(kit) and os.sep + "site-packages" + os.sep not in rf:
            del sys.modules[name]
            gone.append(name)
    importlib.invalidate_caches()
    return gone


def load_module(path: str, generation: int, feed=None, src: bytes = None) -> types.ModuleType:
    """Compile the user file into a fresh module object (no import cache involved). `src`: the
    bytes to compile (a multi-rank group passes rank 0's), else the file is read. When the change
    feed already compiled exactly these bytes in the background, that code is used."""
    if src is None:
        with open(path, "rb") as f:
            src = f.read()
    name = f"devspace_user_{generation}"
    mod = types.ModuleType(name)
    mod.__file__ = path
    code = feed.prepared_for(src) if feed is not None else None
    if code is None:
        code = compile(src, path, "exec")
    exec(code, mod.__dict__)  # noqa: S102 - executing the user's own synced code is the point
    mod.__devspace_digest__ = hashlib.sha256(src).hexdigest()[:8]
    return mod


class SourceOverlay:
    """Import hook for the synced tree: every user module (a .py file under the watched
    directory that the entry file imports) is compiled from bytes this hook hands out — rank 0's
    recorded bytes when the group re-sent them (`snap`), else the file as read now — and the
    bytes each load compiled are recorded (`reads`), so the ranks can prove they run one code
    version. Sits in sys.meta_path just before the PathFinder (builtins and frozen modules keep
    precedence, as with a plain `python train.py`); a name not found in the synced tree falls
    through to the normal import system, so other imports pay one cached directory lookup."""

    def __init__(self, root: str):
        self.root = os.path.realpath(root) + os.sep
        self.snap = {}
        self.reads = {}
        self._real = {}
        self.fault = None  # test-only hook, see _FaultHooks

    def install(self):
        mp = sys.meta_path
        if self in mp:
            return self
        at = next((i for i, f in enumerate(mp) if f is importlib.machinery.PathFinder), len(mp))
        mp.insert(at, self)
        return self

    def uninstall(self):
        if self in sys.meta_path:
            sys.meta_path.remove(self)

    def _under(self, p: str) -> bool:
        r = self._real.get(p)
        if r is None:
            r = self._real[p] = os.path.realpath(p or ".") + os.sep
        return r.startswith(self.root)

    def find_spec(self, name, path=None, target=None):
        dirs = [p for p in (path if path is not None else sys.path) if isinstance(p, str) and self._under(p)]
        if not dirs:
            return None
        spec = importlib.machinery.PathFinder.find_spec(name, dirs)
        if spec is None or not spec.origin or not spec.origin.endswith(".py"):
            return None
        if not os.path.realpath(spec.origin).startswith(self.root):
            return None
        spec.loader = _OverlayLoader(name, spec.origin, self)
        return spec

    def source(self, path: str) -> bytes:
        key = os.path.realpath(path)
        data = self.snap.get(key)
        if data is None:
            with open(path, "rb") as f:
                data = f.read()
            if self.fault is not None:
                self.fault.after_helper_read(path)
        self.reads[key] = data
        return data

    def digest(self, src: bytes) -> str:
        """The code of one load: the entry bytes plus every user module it (re)imported."""
        h = hashlib.sha256(src)
        for k in sorted(self.reads):
            h.update(k.encode() + b"\0" + hashlib.sha256(self.reads[k]).digest())
        return h.hexdigest()[:12]


class _OverlayLoader(importlib.machinery.SourceFileLoader):
    """A source loader whose bytes come from the overlay; no .pyc involved (a cached bytecode
    file could be of another version than the bytes the group agreed on)."""

    def __init__(self, fullname, path, overlay):
        super().__init__(fullname, path)
        self._overlay = overlay

    def get_data(self, path):
        if path == self.path:
            return self._overlay.source(path)
        return super().get_data(path)

    def get_code(self, fullname):
        return compile(self.get_data(self.path), self.path, "exec", dont_inherit=True)


class _FaultHooks:
    """Test-only fault injection (DEVSPACE_RUNNER_FAULT): reproduce the races the agreement
    protocol closes, deterministically.
      mutate-entry-after-read  rank 0 rewrites the entry file right after reading it for a
                               reload (a rank reading the file itself would get other bytes)
      skew-helper              rank 0 rewrites each helper module right after reading it, and
                               the other ranks load 0.3 s later (they read the rewritten file)
    Each file is rewritten once (the rewrite is itself an edit: the next generation)."""

    def __init__(self, spec: str, rank: int):
        self.modes = set(filter(None, (spec or "").split(",")))
        self.rank = rank
        self.done = set()
        self.armed = False  # only reloads (generation > 1), not the initial load

    def _rewrite(self, path):
        if path in self.done:
            return
        self.done.add(path)
        with open(path, "ab") as f:
            f.write(b"\n# devspace-fault: rewritten after rank 0 read it\n")

    def after_entry_read(self, path):
        if self.armed and self.rank == 0 and "mutate-entry-after-read" in self.modes:
            self._rewrite(path)

    def after_helper_read(self, path):
        if self.armed and self.rank == 0 and "skew-helper" in self.modes:
            self._rewrite(path)

    def before_load(self):
        if self.armed and self.rank != 0 and "skew-helper" in self.modes:
            time.sleep(0.3)


class LoadFailed(Exception):
    """The group could not load a generation (on some rank); every rank keeps the previous one."""


def _load_generation(entry, gen, feed, overlay, agree, purge, watch_dir, ctx, fault):
    """Load generation `gen` of the entry file, the same bytes on every rank. Returns the module;
    raises LoadFailed (on every rank alike) when any rank failed.

    One rank: read, compile, exec. Several: rank 0 reads the entry and broadcasts the bytes (and
    the purge decision); every rank execs them with the overlay recording the user modules it
    imports; the ranks gather (ok, code digest). Equal digests: done. Different digests (a helper
    module changed between the ranks' reads): rank 0's recorded sources are broadcast, the other
    ranks re-import from them, and the digests are compared again."""
    src = None
    if agree is None or ctx.rank == 0:
        try:
            with open(entry, "rb") as f:
                src = f.read()
            fault.after_entry_read(entry)
        except OSError as e:  # mid-rename, deleted: nothing to load (the ranks still agree on that)
            ctx.error(f"cannot read {entry}: {e}")
    if agree is not None:
        src, purge = agree.share((src, purge))
    if src is None:
        raise LoadFailed(f"{entry} could not be read")
    if purge:
        purge_user_modules(watch_dir)
    overlay.snap, overlay.reads = {}, {}
    fault.before_load()
    mod, err = _try_load(entry, gen, feed, src)
    if agree is None:
        if mod is None:
            raise LoadFailed(err)
        mod.__devspace_code__ = overlay.digest(src)
        return mod
    digest = overlay.digest(src) if mod is not None else None
    outcomes = agree.gather((mod is not None, digest))
    if all(ok for ok, _ in outcomes) and len({d for _, d in outcomes}) > 1:
        if ctx.rank == 0:
            ctx.log(f"gen={gen}: the ranks compiled different helper sources (digests "
                    f"{sorted({d for _, d in outcomes})}): re-sending rank 0's")
        snap = agree.share(dict(overlay.reads) if ctx.rank == 0 else None)
        if ctx.rank != 0:
            purge_user_modules(watch_dir)
            overlay.snap, overlay.reads = snap, {}
            mod, err = _try_load(entry, gen, feed, src)
            digest = overlay.digest(src) if mod is not None else None
            overlay.snap = {}
        outcomes = agree.gather((mod is not None, digest))
    failed = [r for r, (ok, _) in enumerate(outcomes) if not ok]
    digests = {d for _, d in outcomes}
    if err is not None:
        ctx.error(f"load failed gen={gen}:\n{err}")
    if failed or len(digests) != 1:
        why = f"failed on rank(s) {failed}" if failed else f"code digests still differ: {sorted(digests)}"
        raise LoadFailed(why)
    mod.__devspace_code__ = digest
    if os.environ.get("DEVSPACE_RUNNER_DEBUG"):
        _log(f"rank={ctx.rank} loaded gen={gen} digest={mod.__devspace_digest__} code={digest}")
    return mod


def _try_load(entry, gen, feed, src):
    try:
        return load_module(entry, gen, feed, src=src), None
    except (Exception, SystemExit):  # a syntax error, a failing import: reported, the group keeps its code
        return None, traceback.format_exc()


_STANDBY_IMPORTS = ["torch.distributed", "torch.optim", "torch.nn.parallel", "torch._dynamo"]


def _preimport(names) -> None:
    import importlib

    for name in names:
        try:
            importlib.import_module(name)
        except BaseException:  # missing, broken, or exits at import: paid later, if ever used
            pass


def _modules_file():
    d = os.environ.get("DEVSPACE_RESCUE_DIR")
    return os.path.join(d, "imported-modules.txt") if d else None


def _imported_by_group() -> list:
    path = _modules_file()
    try:
        with open(path) as f:
            return [l.strip() for l in f if l.strip()]
    except (OSError, TypeError):
        return []


def _list_imported_modules(watch_dir: str) -> None:
    """Rank 0, once its group is up: the top-level packages its process imported from outside
    the synced tree, for the warm standby to import ahead of a takeover."""
    path = _modules_file()
    if not path:
        return
    root = os.path.realpath(watch_dir) + os.sep
    names = set()
    for name, mod in list(sys.modules.items()):
        top = name.split(".")[0]
        f = getattr(mod, "__file__", None)
        if "." in name or top.startswith("__") or not f or os.path.realpath(f).startswith(root):
            continue
        names.add(top)
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path + ".tmp", "w") as out:
            out.write("\n".join(sorted(names)) + "\n")
        os.replace(path + ".tmp", path)
    except OSError:
        pass


class _Heartbeat:
    """The rank's side of the supervisor's stuck-step rule (supervise._GroupWatch.assess): a
    thread of its own sends, once a second over the status pipe,

        hb <rank> <step> <phase> <in_phase_s> <longest_s> <still_s> <snap_step> <where>

    phase: start (load, setup(), restore, first step) | reload (load, setup() when
    SETUP_VERSION changed, the first step of the new code) | step (a steady-state step) |
    boundary | idle (paused or waiting). still: seconds since the main thread last showed
    progress, sampled 4x a second: its Python position (innermost frame, bytecode offset)
    changed, or it used at least 5 % of a CPU since the last sample outside a call that waits
    (WAIT_CALLS: `.item()`, `synchronize`, collectives, ...). A thread blocked in a deadlock, a
    dead peer's collective (even one whose wait spins the CPU) or a sleep stands still; an eval
    loop, a checkpoint save or a long computation moves. where: the innermost frame of the user's code. From a thread, so a step that runs for
    minutes keeps the beat going (the old beat came from the top of the loop: a long healthy step
    looked stuck). The main thread only sets `phase`/`since`: two attribute writes per step."""

    def __init__(self, rank, ctx, rescue):
        self.rank, self.ctx, self.rescue = rank, ctx, rescue
        self.phase, self.since, self.longest = "start", time.monotonic(), 0.0
        self.main = threading.get_ident()
        extra = os.environ.get("DEVSPACE_RUNNER_WAIT_CALLS", "")
        self.wait_calls = self.WAIT_CALLS | {x.strip() for x in extra.split(",") if x.strip()}
        self.kit = os.path.dirname(os.path.realpath(__file__)) + os.sep
        self.stopped = False
        self.thread = None
        if os.environ.get("DEVSPACE_RUNNER_STATUS_FD"):
            self.thread = threading.Thread(target=self._run, name="devspace-heartbeat", daemon=True)
            self.thread.start()

    def enter(self, phase: str) -> None:
        self.since = time.monotonic()
        self.phase = phase

    def done(self) -> None:
        """A step finished (steady-state, or the first of a start or reload): it counts towards
        the longest step, which scales the stuck threshold."""
        d = time.monotonic() - self.since
        if d > self.longest:
            self.longest = d
        self.enter("boundary")

    def _where(self, f) -> str:
        inner = f
        while f is not None:
            fn = f.f_code.co_filename
            if not fn.startswith(self.kit) and os.sep + "site-packages" + os.sep not in fn and \
                    not fn.startswith(("<", sys.prefix, sys.base_prefix)):
                return f"{os.path.basename(fn)}:{f.f_lineno}"
            f = f.f_back
        return f"{os.path.basename(inner.f_code.co_filename)}:{inner.f_lineno}" if inner is not None else "?"

    # calls that wait on the device or on peers: a thread inside one that burns CPU (HIP's and
    # RCCL's spin/yield waits, a gloo busy-poll) is waiting, not working. DEVSPACE_RUNNER_WAIT_CALLS
    # adds names (comma-separated).
    WAIT_CALLS = frozenset((
        "item", "tolist", "cpu", "numpy", "to", "float", "int", "bool", "synchronize", "wait", "barrier",
        "monitored_barrier", "all_reduce", "all_gather", "all_gather_into_tensor", "all_gather_object",
        "reduce_scatter", "reduce_scatter_tensor", "broadcast", "broadcast_object_list", "all_to_all",
        "all_to_all_single", "reduce", "gather", "scatter", "send", "recv", "backward", "query",
        "_cuda_synchronize"))
    _callee_cache = {}

    @staticmethod
    def _call_table(code) -> dict:
        """{offset of a call instruction: name of the callable it calls} for a code object: walks
        back from each call over its arguments (their stack effects) to the instruction that
        loaded the callable. Calls it cannot resolve (a conditional in the arguments) are left out."""
        import dis

        ins = list(dis.get_instructions(code))
        table = {}
        for k, i in enumerate(ins):
            arg = i.arg or 0
            if i.opname in ("CALL_FUNCTION", "CALL_METHOD", "CALL"):
                need = arg
            elif i.opname in ("CALL_FUNCTION_KW", "CALL_KW"):
                need = arg + 1  # the keyword-names tuple
            elif i.opname == "CALL_FUNCTION_EX":
                need = 1 + (arg & 1)
            else:
                continue
            j = k - 1
            while j >= 0 and need > 0:
                op = ins[j]
                try:
                    need -= dis.stack_effect(op.opcode, op.arg if op.opcode >= dis.HAVE_ARGUMENT else None,
                                             jump=False)
                except (ValueError, TypeError):
                    break
                j -= 1
            if need == 0 and j >= 0 and ins[j].opname.startswith("LOAD") and isinstance(ins[j].argval, str):
                table[i.offset] = ins[j].argval
        return table

    def _callee(self, f):
        """Name of the function the frame is calling right now (`loss.item()` -> item,
        `dist.all_reduce(t)` -> all_reduce), or None when that is not known."""
        code = f.f_code
        table = self._callee_cache.get(code)
        if table is None:
            table = self._call_table(code)
            if len(self._callee_cache) > 4096:
                self._callee_cache.clear()
            self._callee_cache[code] = table
        return table.get(f.f_lasti)

    def _waiting(self, f) -> bool:
        """The main thread is inside a call that waits (see WAIT_CALLS)."""
        if f is None:
            return False
        try:
            name = self._callee(f)
        except Exception:  # an unusual code object: count its CPU time as work, as before
            return False
        return isinstance(name, str) and name in self.wait_calls

    def _cpu(self, clk):
        try:
            return time.clock_gettime(clk) if clk is not None else 0.0
        except OSError:
            return 0.0

    def _run(self) -> None:
        try:
            clk = time.pthread_getcpuclockid(self.main)  # the main thread's CPU-time clock
        except (AttributeError, OSError):
            clk = None
        last, moved, next_beat = None, time.monotonic(), 0.0
        t_prev, cpu_prev = moved, self._cpu(clk)
        while not self.stopped:
            f = sys._current_frames().get(self.main)
            pos = (id(f.f_code), f.f_lasti) if f is not None else None
            now, cpu = time.monotonic(), self._cpu(clk)
            busy = clk is not None and cpu - cpu_prev >= 0.05 * (now - t_prev)
            if busy and pos == last and self._waiting(f):
                busy = False  # CPU spent spinning in a device or collective wait is not progress
            t_prev, cpu_prev = now, cpu
            if pos != last or busy:
                last, moved = pos, now
            if now >= next_beat:
                where = self._where(f).replace(" ", "_") if f is not None else "?"
                snap = self.rescue.last_step if self.rescue is not None else 0
                _status(f"hb {self.rank} {self.ctx.step} {self.phase} {now - self.since:.2f} {self.longest:.3f} "
                        f"{now - moved:.2f} {snap} {where}")
                next_beat = now + 1.0
            del f
            time.sleep(0.25)

    def stop(self) -> None:
        self.stopped = True


def worker_main(args) -> int:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    import torch  # imported once per process; kept warm across reloads

    if args.standby:
        # a warm standby rank: the supervisor hands it the group's rendezvous port when a failed
        # group is replaced, or closes the pipe. Meanwhile it pays what a process start pays
        # before the training code runs, on a thread (an import that hangs never holds up a
        # takeover): `import torch` (done), the modules a setup() first pulls in (creating an
        # optimizer imports torch._dynamo: 1.5 s of a restart on its own) and the libraries the
        # running group's code imported (transformers, datasets, ...: its rank 0 lists them)
        threading.Thread(target=_preimport, args=(_STANDBY_IMPORTS + _imported_by_group(),),
                         name="devspace-standby-imports", daemon=True).start()
        line = sys.stdin.readline().split()
        if len(line) != 2 or line[0] != "go":
            return 0
        os.environ["MASTER_PORT"] = line[1]
    phases, t_phase = [], [time.perf_counter()]

    def phase(name):  # start-up phase times, logged per rank with DEVSPACE_RUNNER_DEBUG
        now = time.perf_counter()
        phases.append(f"{name}={(now - t_phase[0]) * 1000.0:.0f}ms")
        t_phase[0] = now

    device = None
    dist = None
    group_timeout = None
    if args.group_timeout > 0:
        import datetime

        group_timeout = datetime.timedelta(seconds=args.group_timeout)
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    phase("device")
    if world > 1:
        import torch.distributed as dist  # noqa: WPS433

        # nccl == RCCL on ROCm; DEVSPACE_DIST_BACKEND=gloo runs several ranks on one GPU (RCCL
        # refuses two ranks on a device): a 1-GPU rehearsal of the multi-rank pod
        backend = os.environ.get("DEVSPACE_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
        kw = {"timeout": group_timeout} if group_timeout is not None else {}
        if backend == "nccl":
            # the RCCL communicator is created here, eagerly, for this rank's device: a bad device
            # mapping fails before setup(), not inside the first collective of a training step
            kw["device_id"] = device
        t_pg = time.perf_counter()
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
        phase("process_group")
        if rank == 0:
            _log(f"process group up: backend={backend} world={world} in {(time.perf_counter() - t_pg) * 1000.0:.0f} ms"
                 + (f" (RCCL communicator created for {device})" if backend == "nccl" else ""))
    if device.type == "cuda" and args.gemm_tuning != "off":
        try:
            from devspace_amd.ops import gemm_tuning  # noqa: WPS433

            rep = gemm_tuning.apply(args.gemm_tuning, device)
        except ImportError:  # runner vendored without the package
            rep = {"mode": args.gemm_tuning, "active": False, "entries": 0}
        if rank == 0:
            _log(f"gemm tuning mode={rep['mode']} active={rep['active']} entries={rep['entries']}")
    ctx = Context(rank, world, local_rank, device)
    entry = os.path.abspath(args.entry)
    watch_dir = os.path.abspath(args.watch or os.path.dirname(entry))
    if os.path.dirname(entry) not in sys.path:  # `import helper` next to the entry file, as `python train.py`
        sys.path.insert(0, os.path.dirname(entry))
    watcher = make_watcher(watch_dir)
    feed = ChangeFeed(watcher, entry)
    overlay = SourceOverlay(watch_dir).install()
    fault = overlay.fault = _FaultHooks(os.environ.get("DEVSPACE_RUNNER_FAULT"), rank)
    phase("watch")
    # control plane of the group (gloo, CPU tensors): generation, preemption, code agreement
    agree = Agreement(dist, timeout=group_timeout) if world > 1 else None
    phase("control_group")
    # the supervisor of a group hands down a shared-memory directory; one rank alone keeps
    # snapshots only where --rescue-dir says (e.g. a pod volume that outlives the container)
    rescue_dir = os.environ.get("DEVSPACE_RESCUE_DIR") or args.rescue_dir
    # one rank in a pod: kept in the pod's /dev/shm across container restarts, dropped at a clean exit
    own_dir = not rescue_dir and world == 1 and _in_pod()
    if own_dir:
        rescue_dir = _default_rescue_dir(args.entry, 1)
    rescue = None
    if rescue_dir and args.rescue_every > 0:
        # ignored before it exists: its mkdir must not read as an edit (the change feed runs)
        _IGNORED_DIRS.append(os.path.abspath(rescue_dir))
        rescue = Rescue(rescue_dir, rank, args.rescue_every, agree=agree)
    stop = False
    hb = _Heartbeat(rank, ctx, rescue)

    def _term(*_):
        nonlocal stop
        stop = True

    signal.signal(signal.SIGTERM, _term)

    def leave(code, msg):
        """World > 1: this rank cannot go on without desynchronising the group's collectives.
        Say why (from this rank), tell the supervisor, exit; the supervisor restarts the group."""
        if stop:  # the supervisor is already stopping the group: a peer's exit is expected
            _fatal(0)
        ctx.error(msg)
        _status(f"fail {rank} {ctx.generation}")
        _fatal(code)

    try:
        gen = 1
        t_start = time.perf_counter()
        helper_pending = False
        first = {}
        while True:  # startup: load gen 1, setup(), first step
            ctx.generation = gen
            try:
                mod = _load_generation(entry, gen, None, overlay, agree, False, watch_dir, ctx, fault)
                phase("load")
                state = mod.setup(ctx) if hasattr(mod, "setup") else None
                phase("setup")
                if rescue is not None and state is not None and hasattr(mod, "step"):
                    state = _rescue_restore(rescue, agree, mod, ctx, state)
                    phase("restore")
                if hasattr(mod, "step"):
                    hb.enter("start")  # (the first step alone counts towards the longest step)
                    first = mod.step(ctx, state) or {}
                    ctx.step += 1
                    if device.type == "cuda":
                        torch.cuda.synchronize()
                    phase("first_step")
                hb.done()
                break
            except LoadFailed as e:
                if agree is not None:
                    leave(EXIT_LOAD_FAILED, f"startup failed gen={gen}: {e}")
                ctx.error(f"startup failed gen={gen}:\n{e}")
            except Exception:
                if agree is not None:
                    leave(EXIT_STEP_FAILED, f"startup failed gen={gen}:\n{traceback.format_exc()}")
                ctx.error(f"startup failed gen={gen}:\n{traceback.format_exc()}")
            # one rank: wait warm for the next edit, then try again (nodemon's "waiting for file
            # changes before starting"); several ranks left above and the supervisor waits instead
            ctx.log("waiting for a file change before starting again")
            hb.enter("idle")
            while not feed.take(0.5)[0]:
                if stop:
                    return 0
            gen += 1
            hb.enter("start")
        setup_version = getattr(mod, "SETUP_VERSION", None)
        if rescue is not None:
            rescue.steady(device)
        if rank == 0 and os.environ.get("DEVSPACE_RUNNER_STATUS_FD"):  # under a supervisor
            _list_imported_modules(watch_dir)  # before `ready`: the standby is started on it
        _status(f"ready {rank}")
        if os.environ.get("DEVSPACE_RUNNER_DEBUG"):
            _log(f"rank={rank} start-up{' (warm standby)' if args.standby else ''}: {' '.join(phases)}")
        # Preemption only from here on: an edit that lands during setup() or the first step stays
        # pending in the feed and is picked up by the main loop's first check (a Preempted raised
        # there would have had no handler).
        if args.preempt:
            ctx._feed = feed
            ctx._agree = agree
            ctx._drain_min_ms = args.preempt_drain_ms
        # every rank says it is up (one `[rank N]`-prefixed line each in a multi-rank pod's log)
        _log(
            f"started gen={gen} marker={getattr(mod, 'MARKER', '')} digest={mod.__devspace_digest__} "
            f"code={mod.__devspace_code__} "
            f"world={world} device={device} backend={dist.get_backend() if dist is not None else 'none'} "
            f"loss={first.get('loss') if isinstance(first, dict) else None} "
            f"startup_ms={(time.perf_counter() - t_start) * 1000.0:.1f} "
            f"kit={os.path.dirname(os.path.dirname(os.path.abspath(__file__)))}"
        )
        pending_gen = gen
        reload_t0 = None
        period_ema = None  # steady-state loop period (ms), reported with each reload
        t_iter = time.perf_counter()
        last_print_step = 0
        max_steps = args.max_steps
        script_mode = not hasattr(mod, "step")
        fault.armed = True
        paused = False  # one rank: a step of this generation failed; no more steps until an edit
        while agree is not None or not stop:
            if hb.phase not in ("boundary", "idle"):  # a step, reload or start left early (continue)
                hb.enter("boundary")
            # 1. pick up local change notifications (non-blocking while training; blocking when idle)
            timeout = 0 if (not script_mode and args.train and not paused) else 0.05
            n_changes, t_first, helper_changed = feed.take(timeout)
            # Rank 0's feed alone advances the generation: every rank watches the same synced
            # directory, but their feeds post the edit microseconds apart, and a rank that saw it one
            # step late would otherwise bump the group to a second generation (a spurious reload).
            if n_changes and (agree is None or rank == 0):
                pending_gen += 1
                helper_pending = helper_pending or helper_changed
                if reload_t0 is None:
                    reload_t0 = t_first
            # 2. ranks agree on the newest generation (keeps collectives in `step` matched) and on
            #    whether helper modules must be re-imported (rank 0's view, like the generation)
            target = pending_gen
            snap = (rescue is not None and (agree is None or rank == 0) and not paused and not script_mode
                    and rescue.due(ctx.step))
            job = rescue.inflight if rescue is not None else None
            writing = job is not None and not job["done"]
            write_failed = job is not None and job["done"] and job["err"] is not None
            if agree is not None:
                target, agreed_helper, agreed_stop = agree.boundary(pending_gen, helper_pending, stop, snap,
                                                                    writing, write_failed)
                snap, writing, write_failed = agree.snap, agree.writing, agree.write_failed
                if agreed_stop:
                    stop = True
                    break
                pending_gen = max(pending_gen, target)
                helper_pending = helper_pending or agreed_helper
            if job is not None and not writing:
                _rescue_finish(rescue, ctx, write_failed)
            if target > gen:
                t_reload = time.perf_counter()
                hb.enter("reload")
                wait_ms = (t_reload - reload_t0) * 1000.0 if reload_t0 else 0.0
                purge, helper_pending = helper_pending, False
                running = ctx.generation
                gen = target  # consumed, loaded or not: a failed generation is not retried
                try:
                    new_mod = _load_generation(entry, gen, feed, overlay, agree, purge, watch_dir, ctx, fault)
                except LoadFailed as e:
                    reload_t0 = None
                    if agree is None:
                        ctx.error(f"reload failed gen={gen}, keeping gen={running}:\n{e}")
                    else:
                        ctx.log(f"reload failed gen={gen} ({e}), keeping gen={running} on every rank")
                    continue
                new_setup_version = getattr(new_mod, "SETUP_VERSION", None)
                if hasattr(new_mod, "setup") and (state is None or new_setup_version != setup_version):
                    try:
                        state = new_mod.setup(ctx)
                    except Exception:
                        if agree is not None:  # setup() may hold collectives (DDP's broadcast)
                            leave(EXIT_STEP_FAILED, f"setup failed gen={gen}:\n{traceback.format_exc()}")
                        ctx.error(f"reload failed gen={gen} in setup(), keeping gen={running}:\n"
                                  f"{traceback.format_exc()}")
                        reload_t0 = None
                        continue
                    setup_version = new_setup_version
                mod = new_mod
                ctx.generation = gen
                script_mode = not hasattr(mod, "step")  # a script ran in full when it was loaded
                reload_ms = (time.perf_counter() - t_reload) * 1000.0
                # 3. run the first step with the new code and report
                t_step = time.perf_counter()
                hb.enter("reload")  # (the first step alone counts towards the longest step)
                metrics = {}
                try:
                    if not script_mode:
                        metrics = mod.step(ctx, state) or {}
                        ctx.step += 1
                    if device.type == "cuda":
                        torch.cuda.synchronize()
                except Preempted:  # an even newer edit arrived: report that one instead
                    hb.enter("boundary")
                    continue
                except Exception:
                    if agree is not None:
                        leave(EXIT_STEP_FAILED, f"step failed gen={gen} marker={getattr(mod, 'MARKER', '')}: "
                                                f"leaving the group (the supervisor restarts it)\n"
                                                f"{traceback.format_exc()}")
                    ctx.error(f"step failed gen={gen}: training paused until the next edit\n"
                              f"{traceback.format_exc()}")
                    paused = True
                    reload_t0 = None
                    continue
                paused = False
                hb.done()
                step_ms = (time.perf_counter() - t_step) * 1000.0
                since = (time.perf_counter() - reload_t0) * 1000.0 if reload_t0 else 0.0
                reload_t0 = None
                loss = metrics.get("loss") if isinstance(metrics, dict) else None
                ctx.log(
                    f"reloaded gen={gen} marker={getattr(mod, 'MARKER', '')} digest={mod.__devspace_digest__} "
                    f"code={mod.__devspace_code__} ranks={world} "
                    f"step={ctx.step} loss={loss} step_ms={step_ms:.2f} reload_ms={reload_ms:.2f} "
                    f"pickup_ms={since:.2f} inflight_ms={wait_ms:.2f} period_ms={period_ema or 0.0:.2f} "
                    f"t_mono={time.perf_counter():.6f}"
                )
                t_iter = time.perf_counter()
                continue
            if snap and state is not None and rescue.inflight is None:
                rescue.begin(mod, ctx, state, gen, setup_version)
            if script_mode or not args.train or paused:
                if hb.phase != "idle":
                    hb.enter("idle")
                continue
            hb.enter("step")
            try:
                metrics = mod.step(ctx, state) or {}
                ctx.step += 1
            except Preempted:
                hb.enter("boundary")
                continue
            except Exception:
                if agree is not None:
                    leave(EXIT_STEP_FAILED, f"step failed gen={gen} marker={getattr(mod, 'MARKER', '')}: "
                                            f"leaving the group (the supervisor restarts it)\n"
                                            f"{traceback.format_exc()}")
                # one rank (nodemon's "app crashed - waiting for file changes"): no retry loop that
                # prints the same traceback five times a second; the next edit resumes training
                ctx.error(f"step failed gen={gen}: training paused until the next edit\n{traceback.format_exc()}")
                paused = True
                continue
            hb.done()
            now = time.perf_counter()
            dt = (now - t_iter) * 1000.0
            t_iter = now
            period_ema = dt if period_ema is None else 0.9 * period_ema + 0.1 * dt
            ctx._period_ms = period_ema
            if args.log_every and ctx.step - last_print_step >= args.log_every:
                last_print_step = ctx.step
                ctx.log(f"step={ctx.step} gen={gen} loss={metrics.get('loss') if isinstance(metrics, dict) else None} "
                        f"period_ms={period_ema or 0.0:.3f}")
            if max_steps and ctx.step >= max_steps:
                break
        if stop and rescue is not None and args.rescue_dir and state is not None and not script_mode:
            _rescue_final(rescue, agree, mod, ctx, state, gen, setup_version)
    except Exception as e:  # world > 1: a collective of the control plane failed (a peer is gone)
        if agree is None:
            raise
        why = f"{type(e).__name__}: {e}"
        if "timed out" in why.lower() or "timeout" in why.lower():
            why = (f"no answer from every rank within {args.group_timeout:g} s (a rank stuck in a step? "
                   f"--group-timeout): {why}")
        leave(EXIT_GROUP_LOST, f"group failure gen={ctx.generation}: {why}")
    hb.stop()
    feed.close()
    watcher.close()
    overlay.uninstall()
    if own_dir:
        _drop_rescue_dir(rescue_dir)
    if dist is not None and dist.is_initialized():
        dist.destroy_process_group()
    return 0


def parse_args(argv=None):
    p = argparse.ArgumentParser(prog="devspace_amd.runner", description=__doc__.split("\n")[0])
    p.add_argument("entry", help="user module/script (e.g. train.py)")
    p.add_argument("--nproc", type=int, default=int(os.environ.get("DEVSPACE_NPROC", "1")))
    p.add_argument("--watch", default="", help="directory to watch (default: dir of entry)")
    p.add_argument("--port", type=int, default=0)
    p.add_argument("--log-every", type=int, default=0)
    p.add_argument("--max-steps", type=int, default=0)
    p.add_argument("--max-restarts", type=int, default=3)
    p.add_argument("--no-train", dest="train", action="store_false", help="only run a step after each edit")
    p.add_argument("--restart", action="store_true", help="cold-restart on every change (reference behaviour)")
    p.add_argument("--keep-alive", action="store_true", help="in --restart mode, wait for edits after exit")
    p.add_argument("--no-preempt", dest="preempt", action="store_false",
                   default=os.environ.get("DEVSPACE_PREEMPT", "1") != "0",
                   help="ignore ctx.preempt_point() (always finish the in-flight step)")
    p.add_argument("--preempt-drain-ms", type=float,
                   default=float(os.environ.get("DEVSPACE_PREEMPT_DRAIN_MS", "20")),
                   help="drain queued GPU work at preemption points when the step period is at least this")
    p.add_argument("--group-timeout", type=float, default=float(os.environ.get("DEVSPACE_GROUP_TIMEOUT_S", "600")),
                   help="seconds a collective may wait for every rank (control plane and the training "
                        "group); past it the group fails and is restarted (0: torch's defaults)")
    p.add_argument("--gemm-tuning", default=os.environ.get("DEVSPACE_GEMM_TUNING", "off"),
                   choices=("off", "shipped", "online"),
                   help="TunableOp GEMM selection (devspace_amd/ops/gemm_tuning.py)")
    p.add_argument("--rescue-every", type=float, default=float(os.environ.get("DEVSPACE_RESCUE_EVERY_S", "60")),
                   help="seconds between snapshots of the training state in shared memory, from which a "
                        "group restarted after a failure resumes (0: off)")
    p.add_argument("--rescue-dir", default="",
                   help="keep the snapshots here, also after exit, and take a last one at a clean stop (default: "
                        "in a pod, /dev/shm for the pod's lifetime, dropped at a clean stop; elsewhere, /dev/shm "
                        "for the run)")
    p.add_argument("--stuck-after", type=float, default=float(os.environ.get("DEVSPACE_STUCK_AFTER_S", "60")),
                   help="restart a group stuck in a step with the new code when an edit waits in a steady-state "
                        "step longer than this (or 10x the longest step so far), no rank's main thread has moved "
                        "for this long, and a rescue snapshot exists; else the long step is reported once "
                        "(0: never)")
    p.add_argument("--no-warm-standby", dest="warm_standby", action="store_false",
                   default=os.environ.get("DEVSPACE_WARM_STANDBY", "1") != "0",
                   help="do not keep a second set of rank processes with torch imported to replace a failed "
                        "group (a restart then pays the interpreter and torch start-up)")
    p.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--standby", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args(argv)


def die_with_supervisor() -> None:
    """The first thing a rank does: get SIGTERM when its supervisor dies, however it dies (a
    SIGKILLed supervisor must not leave ranks training on the GPU). The supervisor passes its pid
    (DEVSPACE_SUPERVISOR_PID); one that died before this ran left the rank orphaned, and it exits
    at once. Here and not in a preexec_fn: nothing runs in the forked child of a supervisor that
    has threads (the log relay) between fork and exec."""
    pid = os.environ.get("DEVSPACE_SUPERVISOR_PID")
    if not pid:
        return
    try:
        import ctypes

        ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
    except (OSError, AttributeError):  # pragma: no cover - not Linux
        pass
    if os.getppid() != int(pid):
        os._exit(1)


def main(argv=None) -> int:
    args = parse_args(argv)
    if args.worker:
        die_with_supervisor()
    if args.watch == "":
        args.watch = None
    if args.worker:
        return worker_main(args)
    from devspace_amd.supervise import supervisor_main

    return supervisor_main(args)


if __name__ == "__main__":
    sys.exit(main())
