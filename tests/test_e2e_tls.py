"""The Kubernetes transports over TLS: server verified against certificate-authority-data,
client authenticated with client-certificate-data/client-key-data (mTLS), for REST, exec
WebSocket (wss) with stdin, dev sync in all three protocols, port-forward and log streaming.

Every streaming path here writes to the remote side while a reader thread is parked on the
same TLS connection — the case that deadlocked in round 1 (a blocking SSL_read held the SSL
lock that the stdin writer needed)."""

import os
import signal
import socket
import time
import urllib.request

import pytest
import yaml

from conftest import DevspaceEnv
from test_e2e_cli import container_root, running, wait_for


@pytest.fixture(scope="module")
def tls_kube(tmp_path_factory):
    from devspace_amd.localkube import LocalCluster

    base = str(tmp_path_factory.mktemp("lktls"))
    cluster = LocalCluster(os.path.join(base, "state"), gpus=0, tls=True).start()
    try:
        yield DevspaceEnv(cluster, base)
    finally:
        cluster.stop()


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


def _project(lk, name, ns):
    proj = lk.project("quickstart", name)
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["cluster"]["namespace"] = ns
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    return proj


def test_deploy_enter_logs_over_mtls(tls_kube):
    lk = tls_kube
    assert lk.cluster.server.startswith("https://")
    proj = lk.project("quickstart", "quickstart-tls")
    lk.run(["deploy"], proj)
    wait_for(lambda: running(lk.pods("quickstart")), what="pod")
    out = lk.run(["enter", "--", "cat", "package.json"], proj).stdout
    assert '"name": "quickstart"' in out
    logs = wait_for(lambda: "listening" in lk.run(["logs"], proj).stdout and lk.run(["logs"], proj).stdout,
                    what="logs")
    assert "Example app listening" in logs
    lk.run(["purge"], proj)


def test_enter_with_piped_stdin_over_wss(tls_kube):
    lk = tls_kube
    proj = _project(lk, "qs-tls-stdin", "tlsstdin")
    lk.run(["deploy"], proj)
    wait_for(lambda: running(lk.pods("tlsstdin")), what="pod")
    p = lk.run(["enter", "--", "sh", "-c", "read x; echo got-$x"], proj, input="hello\n", timeout=30)
    assert "got-hello" in p.stdout, p.stdout + p.stderr
    # a larger stdin stream through the same TLS connection while stdout flows back
    blob = "".join(f"line-{i:06d}\n" for i in range(40000))  # ~480 KB
    p = lk.run(["enter", "--", "sh", "-c", "wc -l; echo end"], proj, input=blob, timeout=60)
    assert "40000" in p.stdout and "end" in p.stdout, p.stdout + p.stderr
    lk.run(["purge"], proj)


def _upload_4mib(lk, proj, root, name):
    data = os.urandom(4 << 20)
    dst = os.path.join(root, "app", name)
    t0 = time.perf_counter()
    with open(os.path.join(proj, name), "wb") as f:
        f.write(data)

    def arrived():
        try:
            return os.path.getsize(dst) == len(data) and open(dst, "rb").read() == data
        except OSError:
            return False

    wait_for(arrived, timeout=60, interval=0.01, what=f"4 MiB upload {name}")
    return time.perf_counter() - t0


def _dev_sync_roundtrip(lk, proj, ns, mode):
    env = dict(lk.env, DEVSPACE_SYNC_MODE=mode)
    import subprocess

    dev = subprocess.Popen([lk.bin, "dev", "--terminal=false", "--portforwarding=false"], cwd=proj, env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, text=True,
                           start_new_session=True)
    out = ""
    try:
        pods = wait_for(lambda: running(lk.pods(ns)), timeout=60, what="dev pod")
        root = container_root(lk, pods[0])
        wait_for(lambda: os.path.exists(os.path.join(root, "app", "index.js")), timeout=60, what="initial sync")
        # small edit upstream
        with open(os.path.join(proj, "index.js"), "a") as f:
            f.write(f"// tls edit {mode}\n")
        wait_for(lambda: f"// tls edit {mode}" in open(os.path.join(root, "app", "index.js")).read(),
                 timeout=30, what="small upstream edit")
        up_s = _upload_4mib(lk, proj, root, f"big-{mode}.bin")
        # downstream: a file written inside the container
        lk.run(["enter", "--", "sh", "-c", f"echo from-pod-{mode} > pod_{mode}.txt"], proj, timeout=30)
        wait_for(lambda: os.path.exists(os.path.join(proj, f"pod_{mode}.txt")), timeout=30, what="downstream")
        assert open(os.path.join(proj, f"pod_{mode}.txt")).read().strip() == f"from-pod-{mode}"
        # a 4 MiB file created in the container comes back too
        lk.run(["enter", "--", "sh", "-c", f"head -c 4194304 /dev/urandom > big_pod_{mode}.bin"], proj, timeout=30)
        wait_for(lambda: os.path.exists(os.path.join(proj, f"big_pod_{mode}.bin")) and
                 os.path.getsize(os.path.join(proj, f"big_pod_{mode}.bin")) == 4 << 20,
                 timeout=60, what="4 MiB downstream")
    finally:
        out = _stop(dev)
    assert "Sync started" in out, out
    return up_s, out


@pytest.mark.parametrize("mode", ["helper", "fast", "compat"])
def test_dev_sync_over_wss(tls_kube, mode):
    lk = tls_kube
    ns = f"tlssync-{mode}"
    proj = _project(lk, f"qs-tls-sync-{mode}", ns)
    up_s, out = _dev_sync_roundtrip(lk, proj, ns, mode)
    if mode != "compat":
        assert up_s < 10, up_s
    if mode == "helper":
        assert "falling back" not in out.lower(), out
    lk.run(["purge"], proj)


def test_wss_upload_within_2x_of_plain(tls_kube, localkube):
    """4 MiB upstream over wss vs ws (helper protocol), same host."""
    times = {}
    for label, lk in (("plain", localkube), ("tls", tls_kube)):
        ns = f"cmp-{label}"
        proj = _project(lk, f"qs-cmp-{label}", ns)
        up_s, _ = _dev_sync_roundtrip(lk, proj, ns, "helper")
        times[label] = up_s
        lk.run(["purge"], proj)
    assert times["tls"] <= 2 * times["plain"] + 0.25, times


def test_port_forward_over_wss(tls_kube):
    lk = tls_kube
    proj = _project(lk, "qs-tls-pf", "tlspf")
    remote, local = _free_port(), _free_port()
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["dev"].pop("overrideImages")
    cfg["dev"]["ports"][0]["portMappings"] = [{"localPort": local, "remotePort": remote}]
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    values = os.path.join(proj, "chart", "values.yaml")
    v = yaml.safe_load(open(values))
    v["components"][0]["containers"][0]["env"] = [{"name": "PORT", "value": str(remote)}]
    open(values, "w").write(yaml.safe_dump(v))
    dev = lk.popen(["dev", "--terminal=false", "--sync=false"], proj)
    try:
        wait_for(lambda: running(lk.pods("tlspf")), timeout=60, what="pod")

        def fetch():
            try:
                return urllib.request.urlopen(f"http://127.0.0.1:{local}/", timeout=3).read().decode()
            except Exception:
                return None

        body = wait_for(fetch, timeout=30, what="forwarded response")
        assert body.startswith("Hello from"), body
        for _ in range(10):
            assert (fetch() or "").startswith("Hello from")
    finally:
        out = _stop(dev)
    assert f"Port forwarding started on {local}:{remote}" in out, out
    lk.run(["purge"], proj)


def test_logs_follow_over_wss(tls_kube):
    lk = tls_kube
    proj = _project(lk, "qs-tls-logs", "tlslogs")
    values = os.path.join(proj, "chart", "values.yaml")
    v = yaml.safe_load(open(values))
    v["components"][0]["containers"][0]["command"] = ["sh", "-c",
                                                       "i=0; while true; do echo tick-$i; i=$((i+1)); sleep 0.2; done"]
    open(values, "w").write(yaml.safe_dump(v))
    lk.run(["deploy"], proj)
    wait_for(lambda: running(lk.pods("tlslogs")), what="pod")
    p = lk.popen(["logs", "-f", "--lines", "1"], proj)
    try:
        seen = []
        deadline = time.time() + 20
        while time.time() < deadline and len(seen) < 5:
            line = p.stdout.readline()
            if line.startswith("tick-"):
                seen.append(int(line.strip().split("-")[1]))
        assert len(seen) >= 5, seen
        assert seen == sorted(seen) and seen[-1] - seen[0] == len(seen) - 1
    finally:
        _stop(p)
    lk.run(["purge"], proj)


def test_untrusted_or_anonymous_clients_are_rejected(tls_kube):
    lk = tls_kube
    proj = lk.project("quickstart", "quickstart-tls-bad")
    kc = yaml.safe_load(open(lk.kubeconfig))
    good = yaml.safe_dump(kc)
    try:
        # no client certificate: the server refuses the handshake
        kc["users"][0]["user"] = {"token": "x"}
        open(lk.kubeconfig, "w").write(yaml.safe_dump(kc))
        p = lk.run(["deploy"], proj, check=False)
        assert p.returncode != 0
        # wrong CA: the client refuses the server
        kc = yaml.safe_load(good)
        kc["clusters"][0]["cluster"]["certificate-authority-data"] = kc["users"][0]["user"]["client-certificate-data"]
        open(lk.kubeconfig, "w").write(yaml.safe_dump(kc))
        p = lk.run(["deploy"], proj, check=False)
        assert p.returncode != 0
        assert "certificate" in (p.stdout + p.stderr).lower() or "tls" in (p.stdout + p.stderr).lower()
    finally:
        open(lk.kubeconfig, "w").write(good)
