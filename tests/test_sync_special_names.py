"""File names that need quoting in the shell protocols (spaces, quotes, `$`, backticks, glob
characters, a leading dash, tabs, backslashes, non-ASCII) through every sync protocol: initial
sync, upstream edit, downstream create and upstream delete."""

import os
import time

import pytest

_native = pytest.importorskip("devspace_amd._native")

from conftest import ROOT  # noqa: E402

NAMES = ["with space.txt", "it's.txt", 'dq"uote.txt', "dollar$HOME.txt", "back`tick`.txt", "ünïcödé.txt",
         "-leading-dash.txt", "star*glob?.txt", "br[ack]et.txt", "semi;colon.txt", "amp&er.txt", "tab\there.txt",
         "dir with space/nested 'q'.txt", "percent%d.txt", "back\\slash.txt"]


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
def test_special_file_names_all_protocols(tmp_path, mode):
    src, dst = tmp_path / "src", tmp_path / "pod"
    src.mkdir()
    dst.mkdir()
    for n in NAMES:
        p = src / n
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text("v1 " + n)
    helper = os.path.join(ROOT, "bin", "devspace-helper") if mode == "helper" else ""
    sess = _native.SyncSession(str(src), str(dst), mode="fast" if mode == "helper" else mode, helper_path=helper,
                               log_dir=str(tmp_path / "logs"), pod_name=f"names-{mode}")
    sess.start()
    try:
        assert sess.wait_initial_sync(60000), sess.error()
        assert [n for n in NAMES if _read(dst / n) != "v1 " + n] == []
        time.sleep(1.1)  # compat compares whole-second mtimes
        for n in NAMES:
            (src / n).write_text("v2 " + n)
        _wait(lambda: all(_read(dst / n) == "v2 " + n for n in NAMES), 30, "upstream edits")
        for n in NAMES:
            (dst / ("pod-" + n.replace("/", "_"))).write_text("pod")
        _wait(lambda: all((src / ("pod-" + n.replace("/", "_"))).exists() for n in NAMES), 30, "downstream creates")
        for n in NAMES:
            (src / n).unlink()
        _wait(lambda: not any((dst / n).exists() for n in NAMES), 30, "upstream deletes")
        assert sess.running(), sess.error()
    finally:
        sess.stop()
