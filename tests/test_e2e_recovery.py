"""Dev services survive pod restarts (the reference exits or keeps talking to the
dead pod, services/port_forwarding.go:18-95, services/attach.go:18, services/terminal.go:18):

* port-forward: new connections follow the selector to the replacement pod;
* attach (`dev --terminal=false`): re-attaches to the replacement pod;
* terminal: an interactive session whose pod is deleted reconnects to the new pod;
* forwarders torn down by a dev auto-reload while connections are open (round-1 UAF).
"""

import os
import pty
import re
import select
import signal
import socket
import subprocess
import time
import urllib.request

import yaml

from test_e2e_cli import running, wait_for


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stop(p):
    try:
        os.killpg(p.pid, signal.SIGINT)
        out, _ = p.communicate(timeout=30)
    except Exception:
        os.killpg(p.pid, signal.SIGKILL)
        out, _ = p.communicate()
    return out


def _app_project(lk, name, ns, remote, local, log_ticks=False):
    proj = lk.project("quickstart", name)
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["cluster"]["namespace"] = ns
    cfg["dev"].pop("overrideImages")
    cfg["dev"]["ports"][0]["portMappings"] = [{"localPort": local, "remotePort": remote}]
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    values = os.path.join(proj, "chart", "values.yaml")
    v = yaml.safe_load(open(values))
    v["components"][0]["containers"][0]["env"] = [{"name": "PORT", "value": str(remote)}]
    open(values, "w").write(yaml.safe_dump(v))
    return proj


def _fetch(local):
    try:
        return urllib.request.urlopen(f"http://127.0.0.1:{local}/", timeout=3).read().decode()
    except Exception:
        return None


def _replace_pod(lk, ns):
    first = running(lk.pods(ns))[0]["metadata"]["name"]
    lk.cluster.store.mark_deleting("", "pods", ns, first)
    return first, wait_for(lambda: [p for p in running(lk.pods(ns)) if p["metadata"]["name"] != first],
                           timeout=60, what="replacement pod")[0]["metadata"]["name"]


def test_port_forward_and_attach_follow_pod_restart(localkube):
    lk = localkube
    ns = "rec-pf"
    remote, local = _free_port(), _free_port()
    proj = _app_project(lk, "qs-rec-pf", ns, remote, local)
    dev = lk.popen(["dev", "--terminal=false", "--sync=false"], proj)
    try:
        wait_for(lambda: running(lk.pods(ns)), timeout=60, what="pod")
        body = wait_for(lambda: _fetch(local), timeout=30, what="forwarded response")
        first, second = _replace_pod(lk, ns)
        assert first in body, body
        body2 = wait_for(lambda: (_fetch(local) or "") if second in (_fetch(local) or "") else None, timeout=60,
                         what="response from the replacement pod")
        assert second in body2
    finally:
        out = _stop(dev)
    assert f"now targets pod {second}" in out, out
    assert re.search(rf"Attached to container \S+ of pod {second}", out), out
    lk.run(["purge"], proj)


def test_terminal_reconnects_after_pod_restart(localkube):
    lk = localkube
    ns = "rec-tty"
    proj = lk.project("quickstart", "qs-rec-tty")
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["cluster"]["namespace"] = ns
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    lk.run(["deploy"], proj)
    wait_for(lambda: running(lk.pods(ns)), what="pod")
    master, slave = pty.openpty()
    p = subprocess.Popen([lk.bin, "enter"], cwd=proj, env=lk.env, stdin=slave, stdout=slave, stderr=slave,
                         start_new_session=True)
    os.close(slave)
    buf = b""

    def read_until(pat, timeout=30):
        nonlocal buf
        deadline = time.time() + timeout
        while time.time() < deadline:
            if re.search(pat, buf):
                return True
            r, _, _ = select.select([master], [], [], 0.2)
            if r:
                try:
                    buf += os.read(master, 65536)
                except OSError:
                    break
        return re.search(pat, buf) is not None

    try:
        time.sleep(1.0)
        os.write(master, b"echo first-$((20+1))\n")
        assert read_until(rb"first-21"), buf
        first, second = _replace_pod(lk, ns)
        assert read_until(rb"reconnecting the terminal"), buf
        time.sleep(1.0)
        os.write(master, b"echo second-$HOSTNAME\n")
        assert read_until(rb"second-" + second.encode()), buf
        os.write(master, b"exit 0\n")
        assert p.wait(20) == 0
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
        os.close(master)
    lk.run(["purge"], proj)


def test_port_forward_follows_a_statefulset_pod_replaced_under_the_same_name(localkube):
    """A StatefulSet's replacement pod keeps its name: the multiplexed tunnel of the old pod
    answers every stream with the kubelet's missing-sandbox error (no 404 at an upgrade to
    notice), so the forward compares uids, drops the tunnel and replays on the new pod's."""
    lk = localkube
    ns = "rec-sts"
    remote, local = _free_port(), _free_port()
    proj = lk.project("quickstart-kubectl", "qsk-rec-sts")
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["cluster"]["namespace"] = ns
    cfg["dev"].pop("overrideImages")
    cfg["dev"]["ports"][0]["portMappings"] = [{"localPort": local, "remotePort": remote}]
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    man_path = os.path.join(proj, "kube", "deployment.yaml")
    man = yaml.safe_load(open(man_path))
    man["kind"] = "StatefulSet"
    man["spec"]["serviceName"] = "quickstart"
    man["spec"]["template"]["spec"]["containers"][0]["env"] = [{"name": "PORT", "value": str(remote)}]
    open(man_path, "w").write(yaml.safe_dump(man))
    dev = lk.popen(["dev", "--terminal=false", "--sync=false"], proj)
    try:
        first = wait_for(lambda: running(lk.pods(ns)), timeout=60, what="pod")[0]
        assert first["metadata"]["name"] == "quickstart-0"
        assert wait_for(lambda: _fetch(local), timeout=30, what="forwarded response")
        lk.cluster.store.mark_deleting("", "pods", ns, "quickstart-0")
        wait_for(lambda: [p for p in running(lk.pods(ns))
                          if p["metadata"]["uid"] != first["metadata"]["uid"]], timeout=60, what="replacement pod")
        assert wait_for(lambda: _fetch(local), timeout=30, what="response from the replacement pod")
    finally:
        out = _stop(dev)
    assert "now targets pod quickstart-0 (replaced)" in out, out
    lk.run(["purge"], proj)


def test_reload_with_open_forwarded_connections(localkube):
    """dev auto-reload destroys the forwarders while connections are still open: every
    connection thread is owned and joined (round 1 detached them with a dangling `this`)."""
    lk = localkube
    ns = "rec-reload"
    remote, local = _free_port(), _free_port()
    proj = _app_project(lk, "qs-rec-reload", ns, remote, local)
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["dev"]["autoReload"] = {"paths": ["reload.txt"]}
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    open(os.path.join(proj, "reload.txt"), "w").write("0")
    dev = lk.popen(["dev", "--terminal=false", "--sync=false"], proj)
    socks = []
    try:
        wait_for(lambda: running(lk.pods(ns)), timeout=60, what="pod")
        wait_for(lambda: _fetch(local), timeout=30, what="forwarded response")
        time.sleep(1.5)  # the auto-reload poll watcher takes its baseline
        for _ in range(8):  # idle keep-alive connections held open through the forwarder
            s = socket.create_connection(("127.0.0.1", local))
            s.sendall(b"GET / HTTP/1.1\r\nHost: x\r\n\r\n")
            socks.append(s)
        open(os.path.join(proj, "reload.txt"), "w").write("1")
        # after the reload the forwarder is rebuilt and serves again
        wait_for(lambda: dev.poll() is None and _fetch(local), timeout=60, what="forwarding after reload")
        time.sleep(3.5)  # reload message + 2 s + redeploy
        assert dev.poll() is None, "devspace dev died during the reload"
        assert wait_for(lambda: _fetch(local), timeout=30, what="forwarding after the reload")
    finally:
        for s in socks:
            s.close()
        out = _stop(dev)
    assert "Change detected, will reload in 2 seconds" in out, out
    assert out.count("Port forwarding started") >= 2, out
    lk.run(["purge"], proj)
