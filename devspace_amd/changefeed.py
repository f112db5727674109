"""Change detection for the hot-reload runner: the synced tree's watcher (the native inotify
binding, inotify through ctypes inside a pod, or polling) and the change feed that pre-compiles
the entry file on a background thread. Shared by the worker loop (devspace_amd/runner.py) and the
supervisor (devspace_amd/supervise.py).

The reference polls the tree every second (pkg/devspace/watch/watch.go:33) and redeploys; the
runner reacts to settled inotify events within a fraction of a millisecond instead.
"""

from __future__ import annotations

import os
import sys
import threading
import time

PREFIX = "[devspace-runner]"


_OUT_LOCK = threading.Lock()  # one line at a time on stdout (the supervisor's LogRelay takes it too)


def _log(msg: str) -> None:
    with _OUT_LOCK:
        sys.stdout.write(f"{PREFIX} {msg}\n")
        sys.stdout.flush()



class _PollWatcher:
    """Fallback watcher when the native inotify binding is unavailable."""

    def __init__(self, path: str):
        self.path = path
        self.state = self._scan()

    def _scan(self):
        out = {}
        for root, dirs, files in os.walk(self.path):
            dirs[:] = [d for d in dirs if d not in ("__pycache__", ".git")]
            for f in files:
                p = os.path.join(root, f)
                try:
                    st = os.stat(p)
                except OSError:
                    continue
                out[p] = (st.st_mtime_ns, st.st_size)
        return out

    def poll(self, timeout_ms: int = 0):
        deadline = time.monotonic() + timeout_ms / 1000.0
        while True:
            now = self._scan()
            changed = [p for p, s in now.items() if self.state.get(p) != s]
            changed += [p for p in self.state if p not in now]
            self.state = now
            if changed or time.monotonic() >= deadline:
                return changed
            time.sleep(0.005)

    def close(self):
        pass


class _InotifyWatcher:
    """inotify through ctypes: what the runner uses inside a pod, where the native module
    (built for the developer machine's Python) is not importable. Recursive, settled events
    only (close-after-write, renames, deletes), so a file still being written triggers nothing."""

    _IN_CLOSE_WRITE, _IN_MOVED_FROM, _IN_MOVED_TO = 0x008, 0x040, 0x080
    _IN_CREATE, _IN_DELETE, _IN_DELETE_SELF, _IN_Q_OVERFLOW = 0x100, 0x200, 0x400, 0x4000
    _IN_ISDIR, _IN_IGNORED, _IN_NONBLOCK, _IN_CLOEXEC = 0x40000000, 0x8000, 0o4000, 0o2000000

    def __init__(self, path: str):
        import ctypes
        import ctypes.util

        self._libc = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6", use_errno=True)
        self.fd = self._libc.inotify_init1(self._IN_NONBLOCK | self._IN_CLOEXEC)
        if self.fd < 0:
            raise OSError(ctypes.get_errno(), "inotify_init1 failed")
        self.mask = (self._IN_CLOSE_WRITE | self._IN_MOVED_FROM | self._IN_MOVED_TO | self._IN_CREATE |
                     self._IN_DELETE | self._IN_DELETE_SELF)
        self.wds = {}
        self._add_tree(path)

    def _add(self, d: str) -> None:
        wd = self._libc.inotify_add_watch(self.fd, os.fsencode(d), self.mask)
        if wd >= 0:
            self.wds[wd] = d

    def _add_tree(self, root: str) -> None:
        for d, dirs, _ in os.walk(root):
            dirs[:] = [x for x in dirs if x not in ("__pycache__", ".git")]
            self._add(d)

    def poll(self, timeout_ms: int = 0):
        import select
        import struct

        out = []
        r, _, _ = select.select([self.fd], [], [], max(0, timeout_ms) / 1000.0)
        if not r:
            return out
        while True:
            try:
                buf = os.read(self.fd, 1 << 16)
            except BlockingIOError:
                break
            off = 0
            while off + 16 <= len(buf):
                wd, mask, _cookie, n = struct.unpack_from("iIII", buf, off)
                name = buf[off + 16:off + 16 + n].split(b"\0", 1)[0].decode(errors="replace")
                off += 16 + n
                if mask & self._IN_IGNORED:
                    self.wds.pop(wd, None)
                    continue
                if mask & self._IN_Q_OVERFLOW:
                    out.append(next(iter(self.wds.values()), ""))  # events were lost: reload
                    continue
                base = self.wds.get(wd)
                if base is None:
                    continue
                p = os.path.join(base, name) if name else base
                if mask & self._IN_ISDIR:
                    if mask & (self._IN_CREATE | self._IN_MOVED_TO):
                        self._add_tree(p)
                    continue
                if mask & self._IN_CREATE:
                    continue  # wait for its close-after-write
                out.append(p)
            # the rest of a burst (an editor's write + rename) lands within microseconds: take
            # what follows within 0.25 ms. (This was 2 ms: a fixed 2 ms on every synced edit,
            # measured as the GPU pod's `other_ms`. The sync helper's own temp file, written
            # before its rename into place, is filtered by name in the change feed instead.)
            r, _, _ = select.select([self.fd], [], [], 0.00025)
            if not r:
                break
        return out

    def close(self):
        if self.fd >= 0:
            os.close(self.fd)
            self.fd = -1


def make_watcher(path: str):
    settled = os.environ.get("DEVSPACE_WATCH_SETTLED", "1") != "0"
    try:
        from devspace_amd import _native  # noqa: WPS433

        # settled events only: a file still being written must not trigger (or preempt) a reload
        return _native.Watcher(path, settled_only=settled)
    except Exception:  # native module missing: a vendored runner inside a pod
        pass
    if settled and sys.platform.startswith("linux"):
        try:
            return _InotifyWatcher(path)
        except OSError:
            pass
    return _PollWatcher(path)


class ChangeFeed:
    """Watches the synced directory on a background thread (the native inotify poll releases
    the GIL) and pre-compiles the entry file as soon as it changes, so the code swap at the next
    step boundary only has to exec it — the compile overlaps the in-flight GPU step."""

    def __init__(self, watcher, entry):
        self.watcher = watcher
        self.entry = entry
        self.cv = threading.Condition()
        self.count = 0
        self.first_t = None
        self.prepared = None
        self.entry_real = os.path.realpath(entry)
        self.helper_changed = False  # a .py file other than the entry changed since the last take
        self.stop = False
        self.thread = threading.Thread(target=self._run, name="devspace-change-feed", daemon=True)
        self.thread.start()

    def _run(self):
        while not self.stop:
            try:
                changed = [p for p in self.watcher.poll(100) if not _ignored(p)]
            except Exception:  # pragma: no cover - watcher died; keep the loop alive
                time.sleep(0.05)
                continue
            if not changed:
                continue
            t = time.perf_counter()
            helper = any(p.endswith(".py") and os.path.realpath(p) != self.entry_real for p in changed)
            # Compile, then post the change. (Posting first so that a step boundary reached
            # during the compile waits for it measured 0.2-0.3 ms slower on MI355X,
            # profiles/r2_feed_order_ab.jsonl.)
            prep = None
            try:
                with open(self.entry, "rb") as f:
                    src = f.read()
                prep = (src, compile(src, self.entry, "exec"))
            except Exception:  # syntax errors surface (with traceback) at the reload itself
                prep = None
            with self.cv:
                self.count += 1
                if self.first_t is None:
                    self.first_t = t
                self.prepared = prep
                self.helper_changed = self.helper_changed or helper
                self.cv.notify_all()

    def pending(self) -> bool:
        """A change batch arrived that the loop has not taken yet (lock-free read)."""
        return self.count > 0

    def take(self, timeout_s=0.0):
        """(number of change batches since the last call, perf_counter of the first one,
        whether a .py file other than the entry file changed in them)."""
        with self.cv:
            if self.count == 0 and timeout_s > 0:
                self.cv.wait(timeout_s)
            n, t, helper = self.count, self.first_t, self.helper_changed
            self.count, self.first_t, self.helper_changed = 0, None, False
            return n, t, helper

    def prepared_for(self, src):
        with self.cv:
            p = self.prepared
        return p[1] if p is not None and p[0] == src else None

    def close(self):
        self.stop = True
        self.thread.join(1.0)


# the in-pod sync helper writes `<name>.devspace-tmp` and renames it into place
# (src/helper/helper.cc kTmpSuffix): only the rename is the edit
SYNC_TMP_SUFFIX = ".devspace-tmp"


_IGNORED_DIRS = []  # what the runner itself writes under the watched tree (a --rescue-dir there)


def _ignored(p: str) -> bool:
    base = os.path.basename(p)
    return ("__pycache__" in p or base.endswith((".pyc", ".swp", "~", SYNC_TMP_SUFFIX)) or
            base.startswith(".#") or any(p == d or p.startswith(d + os.sep) for d in _IGNORED_DIRS))
