"""pybind11 module (devspace_amd._native) — YAML, matchers, config parsing, sync session."""
import os
import time

import pytest

from devspace_amd import _native


def test_yaml_roundtrip():
    d = _native.yaml_parse("a: 1\nb:\n- x\n- {y: true}\n")
    assert d == {"a": 1, "b": ["x", {"y": True}]}
    assert _native.yaml_parse(_native.yaml_dump(d)) == d


def test_matchers():
    assert _native.gitignore_match(["*.pyc"], "/a/b/c.pyc")
    assert not _native.gitignore_match(["/build"], "/src/build")
    assert _native.dockerignore_match(["node_modules"], "node_modules/x/y")
    assert _native.glob_match("chart/**", "chart/templates/a.yaml")


def test_parse_config_upgrade():
    cfg = _native.parse_config({"version": "v1alpha1", "devSpace": {"services": [{"name": "s"}]}})
    assert cfg["version"] == "v1alpha2"
    assert cfg["dev"]["selectors"][0]["name"] == "s"
    with pytest.raises(Exception):
        _native.parse_config({"version": "v1alpha2", "bogus": 1})


@pytest.mark.parametrize("mode", ["fast", "helper", "compat"])
def test_sync_session_roundtrip(tmp_path, mode):
    local, remote = tmp_path / "local", tmp_path / "remote"
    local.mkdir()
    remote.mkdir()
    (local / "a.txt").write_text("one")
    helper = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin", "devspace-helper")
    s = _native.SyncSession(str(local), str(remote), mode=mode, helper_path=helper, log_dir=str(tmp_path / "logs"))
    s.start()
    assert s.wait_initial_sync(20000), s.error()

    def wait(pred, timeout=15):
        t0 = time.time()
        while time.time() - t0 < timeout:
            if pred():
                return True
            time.sleep(0.02)
        return False

    assert wait(lambda: (remote / "a.txt").exists() and (remote / "a.txt").read_text() == "one")
    (remote / "b.txt").write_text("from-pod")
    assert wait(lambda: (local / "b.txt").exists())
    (local / "a.txt").write_text("two!")
    assert wait(lambda: (remote / "a.txt").read_text() == "two!")
    # the counters move after the remote ack (and its log line), i.e. just after the bytes
    # landed: wait for them instead of reading them the moment the file changed
    assert wait(lambda: s.stats()["upstream_changes"] >= 2 and s.stats()["downstream_changes"] >= 1), s.stats()
    s.stop()
