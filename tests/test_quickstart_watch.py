"""examples/quickstart/watch.js — the restart-on-change runner of the headline benchmark's app.
Each edit must restart the server as a fresh process running the new code as its main module
(what nodemon does), whether the restart goes through the pre-booted standby or a cold spawn."""

import os
import shutil
import signal
import socket
import subprocess
import time
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")

APP = """const http = require('http');
const port = process.env.PORT;
const main = require.main === module;
// nothing of the standby's hand-off may leak into the app: no IPC channel, no SIGUSR2 listener
const st = typeof process.send + '/' + typeof process.connected + '/' + process.listenerCount('SIGUSR2');
http.createServer((req, res) => {
  res.end(JSON.stringify({tag: 'TAG', pid: process.pid, main, send: st, argv1: process.argv[1]}));
}).listen(port);
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _get(port):
    import json
    try:
        return json.loads(urllib.request.urlopen(f"http://127.0.0.1:{port}/", timeout=2).read())
    except Exception:
        return None


def _wait(pred, timeout=30):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        v = pred()
        if v:
            return v
        time.sleep(0.01)
    raise AssertionError("timed out")


@pytest.mark.skipif(NODE is None, reason="node not installed")
@pytest.mark.parametrize("standby", ["2", "1", "0"])
def test_watch_restarts_fresh_main_module(tmp_path, standby):
    shutil.copy(os.path.join(ROOT, "examples", "quickstart", "watch.js"), tmp_path / "watch.js")
    app = tmp_path / "index.js"
    app.write_text(APP.replace("TAG", "v0"))
    port = _port()
    p = subprocess.Popen([NODE, "watch.js", "index.js"], cwd=tmp_path, start_new_session=True,
                         env=dict(os.environ, PORT=str(port), WATCH_STANDBY=standby),
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        first = _wait(lambda: _get(port))
        pids = {first["pid"]}
        for i in range(1, 4):
            time.sleep(0.4)  # let the next standby boot
            tmp = tmp_path / ".index.js.tmp"
            tmp.write_text(APP.replace("TAG", f"v{i}"))
            os.rename(tmp, app)  # how devspace sync lands a file
            r = _wait(lambda: (lambda b: b if b and b["tag"] == f"v{i}" else None)(_get(port)))
            assert r["main"] is True, r  # require.main === module, as under `node index.js`
            assert r["send"] == "undefined/undefined/0", r
            assert r["argv1"] == str(app), r
            assert r["pid"] not in pids, r  # a fresh process per edit
            pids.add(r["pid"])
    finally:
        os.killpg(p.pid, signal.SIGTERM)
        out, _ = p.communicate(timeout=10)
    assert "[watch] started gen=4" in out, out
    if standby != "0":
        assert "(standby)" in out, out  # restarts went through a booted standby
    else:
        assert "standby" not in out, out
    # no process of the tree outlives the watcher (the standby exits with its parent channel)
    time.sleep(0.5)
    for pid in pids:
        assert not os.path.exists(f"/proc/{pid}") or open(f"/proc/{pid}/stat").read().split()[2] == "Z"


def test_standbys_exit_when_the_watcher_is_killed(tmp_path):
    """A standby holds only its status pipe to the watcher: SIGKILL of the watcher alone (no
    process-group signal) closes that pipe and every standby exits."""
    import psutil

    app = tmp_path / "index.js"
    app.write_text("require('http').createServer((q, r) => r.end('v0')).listen(0);\n")
    shutil.copy(os.path.join(ROOT, "examples", "quickstart", "watch.js"), tmp_path / "watch.js")
    p = subprocess.Popen(["node", str(tmp_path / "watch.js"), str(app)], cwd=tmp_path, stdout=subprocess.DEVNULL,
                         stderr=subprocess.STDOUT, env=dict(os.environ, WATCH_STANDBY="3"), start_new_session=True)
    try:
        deadline = time.time() + 20
        standbys = []
        while time.time() < deadline and len(standbys) < 3:
            time.sleep(0.2)
            standbys = [c for c in psutil.Process(p.pid).children() if "-e" in c.cmdline()]
        assert len(standbys) == 3, standbys
        p.kill()
        p.wait(10)
        gone, alive = psutil.wait_procs(standbys, timeout=10)
        assert not alive, alive
    finally:
        try:
            os.killpg(p.pid, signal.SIGKILL)  # the app the watcher started, and anything left
        except ProcessLookupError:
            pass


def test_standby_pool_shrinks_after_a_quiet_period(tmp_path):
    """After a burst grew the pool, a restart after a quiet period gives one standby back."""
    import psutil

    app = tmp_path / "index.js"
    app.write_text("require('http').createServer((q, r) => r.end('v0')).listen(0);\n")
    shutil.copy(os.path.join(ROOT, "examples", "quickstart", "watch.js"), tmp_path / "watch.js")
    p = subprocess.Popen(["node", str(tmp_path / "watch.js"), str(app)], cwd=tmp_path, stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True,
                         env=dict(os.environ, WATCH_STANDBY="1", WATCH_STANDBY_MAX="4", WATCH_STANDBY_SHRINK_MS="1500"))
    try:
        time.sleep(1.0)
        for i in range(12):
            app.write_text(f"require('http').createServer((q, r) => r.end('v{i + 1}')).listen(0);\n")
            time.sleep(0.02)
        time.sleep(2.5)  # settle, and longer than the shrink period
        grown = len(psutil.Process(p.pid).children())
        app.write_text("require('http').createServer((q, r) => r.end('quiet')).listen(0);\n")
        time.sleep(2.0)
        after = len(psutil.Process(p.pid).children())
        assert after == grown - 1, (grown, after)
    finally:
        p.terminate()
        p.wait(10)


def test_standby_pool_grows_under_back_to_back_edits(tmp_path):
    """Edits faster than node boots exhaust the standby pool: the watcher adds standbys (up to
    WATCH_STANDBY_MAX) instead of handing restarts to processes still booting."""
    import psutil

    app = tmp_path / "index.js"
    app.write_text("require('http').createServer((q, r) => r.end('v0')).listen(0);\n")
    shutil.copy(os.path.join(ROOT, "examples", "quickstart", "watch.js"), tmp_path / "watch.js")
    p = subprocess.Popen(["node", str(tmp_path / "watch.js"), str(app)], cwd=tmp_path, stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True, env=dict(os.environ, WATCH_STANDBY="1",
                                                                         WATCH_STANDBY_MAX="4"))
    try:
        time.sleep(1.0)
        for i in range(12):  # back to back: no time for a standby to boot in between
            app.write_text(f"require('http').createServer((q, r) => r.end('v{i + 1}')).listen(0);\n")
            time.sleep(0.02)
        time.sleep(2.0)  # let the pool settle
        kids = psutil.Process(p.pid).children()
        # the running app + the grown pool (1 standby at start, at most 4)
        assert 3 <= len(kids) <= 5, [k.cmdline()[:3] for k in kids]
    finally:
        p.terminate()
        p.wait(10)


def test_restart_handed_to_a_booting_standby_serves(tmp_path):
    """Edits landing faster than standbys boot hand the script to a standby whose warm-up has
    not finished: the warm-up must stop there (no message on the removed IPC channel, no stray
    exception in the app) and the last version must serve."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    app = tmp_path / "index.js"

    def write(v):
        app.write_text("require('http').createServer((q, r) => r.end('%s')).listen(%d, '127.0.0.1');\n" % (v, port))

    write("v0")
    shutil.copy(os.path.join(ROOT, "examples", "quickstart", "watch.js"), tmp_path / "watch.js")
    p = subprocess.Popen(["node", str(tmp_path / "watch.js"), str(app)], cwd=tmp_path, stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True, env=dict(os.environ, WATCH_STANDBY="1"))
    try:
        assert "started gen=1" in p.stdout.readline()
        time.sleep(0.05)  # the standby started with gen 1 is still booting
        for i in range(1, 9):
            write(f"v{i}")
            time.sleep(0.03)
        deadline = time.time() + 15
        body = None
        while time.time() < deadline:
            try:
                body = urllib.request.urlopen(f"http://127.0.0.1:{port}/", timeout=1).read().decode()
                if body == "v8":
                    break
            except OSError:
                pass
            time.sleep(0.05)
        assert body == "v8", body
    finally:
        p.terminate()
        out = p.communicate(timeout=10)[0]
    assert "TypeError" not in out and "Error" not in out.replace("[watch]", ""), out
