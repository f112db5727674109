"""The POSIX sync protocols in a container that has only the reference's documented toolset
(`sh tar find stat mkdir rm cat printf echo kill sleep`, plus the `gzip` GNU tar
execs for -z; busybox tar has it built in). No `head`, `touch`, `mv`, `dd` or `wc`: fast mode
must fall back to the cat/stat upload and still probe for downstream changes.

The "container" is the LocalShellTransport shell started with PATH = a directory holding only
those tools (reference: docs/pages/development/synchronization.md:83)."""

import os
import shutil
import time

import pytest

_native = pytest.importorskip("devspace_amd._native")

TOOLS = ["sh", "tar", "find", "stat", "mkdir", "rm", "cat", "printf", "echo", "kill", "sleep", "gzip"]


def _wait(pred, timeout, what):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if pred():
            return
        time.sleep(0.02)
    raise AssertionError(f"timed out: {what}")


@pytest.fixture()
def minimal_path(tmp_path):
    bindir = tmp_path / "minbin"
    bindir.mkdir()
    for t in TOOLS:
        src = shutil.which(t)
        assert src, t
        os.symlink(src, bindir / t)
    old = os.environ["PATH"]
    yield str(bindir), old
    os.environ["PATH"] = old


@pytest.mark.parametrize("mode", ["fast", "compat"])
def test_sync_with_only_reference_tools(minimal_path, mode, tmp_path):
    bindir, old_path = minimal_path
    src, dst = tmp_path / "src", tmp_path / "pod" / "app"
    (src / "lib").mkdir(parents=True)
    dst.mkdir(parents=True)
    (src / "main.py").write_text("print('hi')\n")
    (src / "lib" / "blob.bin").write_bytes(os.urandom(3 << 20))
    logs = tmp_path / "logs"
    sess = _native.SyncSession(str(src), str(dst), mode=mode, log_dir=str(logs), pod_name=f"min-{mode}")
    os.environ["PATH"] = bindir  # the shells the session starts now see only the minimal tools
    try:
        sess.start()
    finally:
        os.environ["PATH"] = old_path
    try:
        assert sess.wait_initial_sync(120000), sess.error()
        assert (dst / "main.py").read_text() == "print('hi')\n"
        assert (dst / "lib" / "blob.bin").read_bytes() == (src / "lib" / "blob.bin").read_bytes()
        # upstream edit
        time.sleep(1.1)  # compat compares whole-second mtimes
        (src / "main.py").write_text("print('edited')\n")
        _wait(lambda: (dst / "main.py").read_text() == "print('edited')\n", 30, "upstream edit")
        # downstream create + delete
        (dst / "lib" / "from_pod.txt").write_text("pod")
        _wait(lambda: (src / "lib" / "from_pod.txt").exists(), 30, "downstream create")
        (dst / "lib" / "from_pod.txt").unlink()
        _wait(lambda: not (src / "lib" / "from_pod.txt").exists(), 30, "downstream delete")
        assert sess.running(), sess.error()
        st = sess.stats()
        if mode == "fast":
            assert st["probes"] > 0, st  # change probes work without touch/mv/head
            log = (logs / "sync.log").read_text()
            assert "`head` not found in the container" in log, log[-2000:]
    finally:
        sess.stop()
