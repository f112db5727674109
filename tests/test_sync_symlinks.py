"""Local symlinks are followed upstream, as the reference does (sync/upstream.go:261-304,
sync/symlink.go): a link to a file or directory outside the synced tree uploads the target's
content, edits of the target (and new files in a linked directory) sync, removing the link
removes the copy in the container, and the target itself is never touched."""

import os
import time

import pytest

_native = pytest.importorskip("devspace_amd._native")

from conftest import ROOT  # noqa: E402


def _wait(pred, timeout, what):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if pred():
            return
        time.sleep(0.02)
    raise AssertionError(f"timed out: {what}")


def _read(p):
    try:
        with open(p) as f:
            return f.read()
    except OSError:
        return None


@pytest.mark.parametrize("mode", ["fast", "compat", "helper"])
def test_symlinks_followed_upstream(tmp_path, mode):
    src, dst, ext = tmp_path / "src", tmp_path / "pod", tmp_path / "ext"
    for d in (src, dst, ext / "sub"):
        d.mkdir(parents=True)
    (ext / "target.txt").write_text("t1")
    (ext / "sub" / "inner.txt").write_text("i1")
    os.symlink(ext / "target.txt", src / "link.txt")
    os.symlink(ext / "sub", src / "linkdir")
    helper = os.path.join(ROOT, "bin", "devspace-helper") if mode == "helper" else ""
    sess = _native.SyncSession(str(src), str(dst), mode="fast" if mode == "helper" else mode, helper_path=helper,
                               log_dir=str(tmp_path / "logs"), pod_name=f"links-{mode}")
    sess.start()
    try:
        assert sess.wait_initial_sync(60000), sess.error()
        assert _read(dst / "link.txt") == "t1" and not os.path.islink(dst / "link.txt")
        assert _read(dst / "linkdir" / "inner.txt") == "i1"
        time.sleep(1.1)  # compat compares whole-second mtimes
        (ext / "target.txt").write_text("t2")
        (ext / "sub" / "inner.txt").write_text("i2")
        (ext / "sub" / "new.txt").write_text("n")
        _wait(lambda: _read(dst / "link.txt") == "t2", 30, "edit of a linked file")
        _wait(lambda: _read(dst / "linkdir" / "inner.txt") == "i2", 30, "edit inside a linked directory")
        _wait(lambda: _read(dst / "linkdir" / "new.txt") == "n", 30, "new file inside a linked directory")
        os.unlink(src / "link.txt")
        _wait(lambda: not (dst / "link.txt").exists(), 30, "link removal")
        assert _read(ext / "target.txt") == "t2"
        assert sess.running(), sess.error()
    finally:
        sess.stop()
