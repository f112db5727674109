"""kubeconfig / auth / transport fidelity against the local cluster (client-go parity,
/root/reference/pkg/util/kubeconfig/kubeconfig.go:17-69, pkg/devspace/kubectl/client.go:63-142):

* exec credential plugins: re-run on expiry (status.expirationTimestamp) and on 401, including
  mid-`dev` (the token expires, the pod restarts, the sync reconnects with a fresh token);
* HTTPS_PROXY (HTTP CONNECT tunnel) and NO_PROXY;
* keep-alive: one TLS handshake serves every REST call of a `devspace deploy`;
* a ':'-separated multi-file KUBECONFIG.
"""

import datetime
import json
import os
import select
import signal
import socket
import subprocess
import sys
import threading
import time

import pytest
import yaml

from conftest import DevspaceEnv
from test_e2e_cli import container_root, running, wait_for

PLUGIN = r'''
import datetime, json, os, sys, time
cnt = os.environ["PLUGIN_COUNT"]
n = (int(open(cnt).read() or 0) if os.path.exists(cnt) else 0) + 1
open(cnt, "w").write(str(n))
ttl = int(os.environ.get("PLUGIN_TTL", "0"))
info = json.loads(os.environ.get("KUBERNETES_EXEC_INFO", "{}"))
assert info.get("kind") == "ExecCredential", info
exp = int(time.time()) + ttl if ttl else 0
st = {"token": "tok-%d-%d" % (exp, n)}
if ttl:
    st["expirationTimestamp"] = datetime.datetime.utcfromtimestamp(exp).strftime("%Y-%m-%dT%H:%M:%SZ")
print(json.dumps({"apiVersion": "client.authentication.k8s.io/v1beta1", "kind": "ExecCredential", "status": st}))
'''


class TokenPolicy:
    """tok-<expiry>-<n>: valid until <expiry> (0 = never) unless revoked (n <= revoked_upto)."""

    def __init__(self):
        self.revoked_upto = 0

    def __call__(self, token):
        try:
            _, exp, n = token.split("-")
            exp, n = int(exp), int(n)
        except ValueError:
            return False
        if n <= self.revoked_upto:
            return False
        return exp == 0 or exp > time.time()


def _plugin_cluster(tmp_path, ttl, policy):
    from devspace_amd.localkube import LocalCluster

    cluster = LocalCluster(str(tmp_path / "state"), gpus=0, token_validator=policy).start()
    lk = DevspaceEnv(cluster, str(tmp_path))
    plugin = tmp_path / "plugin.py"
    plugin.write_text(PLUGIN)
    count = tmp_path / "count"
    kc = yaml.safe_load(open(lk.kubeconfig))
    kc["users"][0]["user"] = {"exec": {
        "apiVersion": "client.authentication.k8s.io/v1beta1", "command": sys.executable, "args": [str(plugin)],
        "env": [{"name": "PLUGIN_COUNT", "value": str(count)}, {"name": "PLUGIN_TTL", "value": str(ttl)}],
        "provideClusterInfo": True}}
    open(lk.kubeconfig, "w").write(yaml.safe_dump(kc))
    return cluster, lk, count


def test_exec_plugin_refreshes_on_401(tmp_path):
    policy = TokenPolicy()
    policy.revoked_upto = 1  # the first token the plugin hands out is already revoked
    cluster, lk, count = _plugin_cluster(tmp_path, 0, policy)
    try:
        proj = lk.project("quickstart", "qs-401")
        lk.run(["deploy"], proj)
        assert int(count.read_text()) == 2
        assert cluster.api.auth_failures >= 1
        lk.run(["purge"], proj)
    finally:
        cluster.stop()


def test_token_expires_mid_dev_and_sync_reconnects(tmp_path):
    policy = TokenPolicy()
    cluster, lk, count = _plugin_cluster(tmp_path, 3, policy)
    dev = None
    try:
        proj = lk.project("quickstart", "qs-expiry")
        dev = lk.popen(["dev", "--terminal=false", "--portforwarding=false"], proj)
        pods = wait_for(lambda: running(lk.pods("quickstart")), timeout=60, what="dev pod")
        root = container_root(lk, pods[0])
        wait_for(lambda: os.path.exists(os.path.join(root, "app", "index.js")), timeout=30, what="initial sync")
        first = pods[0]["metadata"]["name"]
        time.sleep(4.0)  # the token the sync started with is expired now
        cluster.store.mark_deleting("", "pods", "quickstart", first)
        new = wait_for(lambda: [p for p in running(lk.pods("quickstart")) if p["metadata"]["name"] != first],
                       timeout=60, what="replacement pod")[0]
        new_root = container_root(lk, new)
        with open(os.path.join(proj, "index.js"), "a") as f:
            f.write("// after token expiry\n")
        wait_for(lambda: os.path.exists(os.path.join(new_root, "app", "index.js")) and
                 "// after token expiry" in open(os.path.join(new_root, "app", "index.js")).read(),
                 timeout=60, what="sync into the replacement pod")
        assert int(count.read_text()) >= 2
    finally:
        if dev is not None:
            os.killpg(dev.pid, signal.SIGINT)
            try:
                dev.communicate(timeout=30)
            except Exception:
                os.killpg(dev.pid, signal.SIGKILL)
        cluster.stop()


def test_token_file_rotated_mid_dev_is_read_again(tmp_path):
    """A kubeconfig `tokenFile` (a projected service-account token, rotated by the kubelet):
    when the file gets a new token and the old one is revoked mid-`dev`, the next request that
    gets a 401 reads the file again and goes on, as client-go's cached token source does; the
    sync reconnects into the replacement pod with the new token."""
    from devspace_amd.localkube import LocalCluster

    policy = TokenPolicy()
    cluster = LocalCluster(str(tmp_path / "state"), gpus=0, token_validator=policy).start()
    lk = DevspaceEnv(cluster, str(tmp_path))
    token = tmp_path / "sa-token"
    token.write_text("tok-0-1\n")
    kc = yaml.safe_load(open(lk.kubeconfig))
    kc["users"][0]["user"] = {"tokenFile": str(token)}
    open(lk.kubeconfig, "w").write(yaml.safe_dump(kc))
    dev = None
    try:
        proj = lk.project("quickstart", "qs-tokenfile")
        dev = lk.popen(["dev", "--terminal=false", "--portforwarding=false"], proj)
        pods = wait_for(lambda: running(lk.pods("quickstart")), timeout=60, what="dev pod")
        root = container_root(lk, pods[0])
        wait_for(lambda: os.path.exists(os.path.join(root, "app", "index.js")), timeout=30, what="initial sync")
        first = pods[0]["metadata"]["name"]
        failures = cluster.api.auth_failures
        token.write_text("tok-0-2\n")  # rotated; the old token stops working at once
        policy.revoked_upto = 1
        cluster.store.mark_deleting("", "pods", "quickstart", first)
        new = wait_for(lambda: [p for p in running(lk.pods("quickstart")) if p["metadata"]["name"] != first],
                       timeout=60, what="replacement pod")[0]
        new_root = container_root(lk, new)
        with open(os.path.join(proj, "index.js"), "a") as f:
            f.write("// after token rotation\n")
        wait_for(lambda: os.path.exists(os.path.join(new_root, "app", "index.js")) and
                 "// after token rotation" in open(os.path.join(new_root, "app", "index.js")).read(),
                 timeout=60, what="sync into the replacement pod")
        assert cluster.api.auth_failures > failures  # the old token was refused, then replaced
    finally:
        if dev is not None:
            os.killpg(dev.pid, signal.SIGINT)
            try:
                out, _ = dev.communicate(timeout=30)
                print(out[-4000:])
            except Exception:
                os.killpg(dev.pid, signal.SIGKILL)
            log = os.path.join(proj, ".devspace", "logs", "sync.log")
            if os.path.exists(log):
                print(open(log).read()[-4000:])
        cluster.stop()


class ConnectProxy(threading.Thread):
    """Minimal HTTP CONNECT proxy (what HTTPS_PROXY points at in corporate networks)."""

    def __init__(self):
        super().__init__(daemon=True)
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(64)
        self.port = self.sock.getsockname()[1]
        self.targets = []
        self.stop = False

    def run(self):
        while not self.stop:
            r, _, _ = select.select([self.sock], [], [], 0.2)
            if not r:
                continue
            c, _ = self.sock.accept()
            threading.Thread(target=self.handle, args=(c,), daemon=True).start()

    def handle(self, c):
        head = b""
        while b"\r\n\r\n" not in head:
            d = c.recv(4096)
            if not d:
                c.close()
                return
            head += d
        line = head.split(b"\r\n")[0].decode()
        method, target, _ = line.split(" ", 2)
        if method != "CONNECT":
            c.sendall(b"HTTP/1.1 405 Method Not Allowed\r\n\r\n")
            c.close()
            return
        self.targets.append(target)
        host, port = target.rsplit(":", 1)
        up = socket.create_connection((host, int(port)))
        c.sendall(b"HTTP/1.1 200 Connection established\r\n\r\n")
        socks = [c, up]
        try:
            while True:
                r, _, _ = select.select(socks, [], [], 30)
                if not r:
                    break
                for s in r:
                    d = s.recv(65536)
                    if not d:
                        return
                    (up if s is c else c).sendall(d)
        except OSError:
            pass
        finally:
            c.close()
            up.close()


@pytest.fixture(scope="module")
def tls_cluster(tmp_path_factory):
    from devspace_amd.localkube import LocalCluster

    base = str(tmp_path_factory.mktemp("lkauth"))
    cluster = LocalCluster(os.path.join(base, "state"), gpus=0, tls=True).start()
    try:
        yield DevspaceEnv(cluster, base)
    finally:
        cluster.stop()


def _net_span(proj):
    spans = [json.loads(l) for l in open(os.path.join(proj, ".devspace", "logs", "trace.jsonl"))]
    return [s for s in spans if s["span"] == "net"][-1]


def test_https_proxy_and_no_proxy(tls_cluster):
    lk = tls_cluster
    proxy = ConnectProxy()
    proxy.start()
    try:
        proj = lk.project("quickstart", "qs-proxy")
        env = dict(lk.env, HTTPS_PROXY=f"http://127.0.0.1:{proxy.port}", NO_PROXY="", no_proxy="")
        env.pop("https_proxy", None)
        p = subprocess.run([lk.bin, "deploy"], cwd=proj, env=env, capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stdout + p.stderr
        wait_for(lambda: running(lk.pods("quickstart")), what="pod")
        p = subprocess.run([lk.bin, "enter", "--", "cat", "package.json"], cwd=proj, env=env, capture_output=True,
                           text=True, timeout=60)
        assert '"name": "quickstart"' in p.stdout, p.stdout + p.stderr
        assert proxy.targets and all(t == f"127.0.0.1:{lk.cluster.port}" for t in proxy.targets), proxy.targets
        assert int(_net_span(proj)["proxied"]) >= 1
        n = len(proxy.targets)
        env["NO_PROXY"] = "localhost,127.0.0.0/8"
        p = subprocess.run([lk.bin, "enter", "--", "true"], cwd=proj, env=env, capture_output=True, text=True,
                           timeout=60)
        assert p.returncode == 0, p.stdout + p.stderr
        assert len(proxy.targets) == n, proxy.targets
        lk.run(["purge"], proj)
    finally:
        proxy.stop = True


def test_keepalive_one_handshake_for_all_rest_calls(tls_cluster):
    lk = tls_cluster
    proj = lk.project("quickstart", "qs-keepalive")
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["cluster"]["namespace"] = "keepalive"
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    lk.run(["deploy"], proj)
    net = _net_span(proj)
    assert int(net["requests"]) >= 8, net
    # REST rides pooled keep-alive connections; watches hold their own while they run
    assert int(net["tls_handshakes"]) <= 3, net
    assert int(net["reused"]) >= int(net["requests"]) - int(net["tls_handshakes"]) - 2, net
    lk.run(["purge"], proj)


def test_multi_file_kubeconfig(tls_cluster, tmp_path):
    lk = tls_cluster
    kc = yaml.safe_load(open(lk.kubeconfig))
    a = {"apiVersion": "v1", "kind": "Config", "current-context": kc["current-context"], "users": kc["users"],
         "clusters": [], "contexts": []}
    b = {"apiVersion": "v1", "kind": "Config", "clusters": kc["clusters"], "contexts": kc["contexts"], "users": [
        {"name": kc["users"][0]["name"], "user": {"token": "shadowed-by-first-file"}}]}
    fa, fb = tmp_path / "a.yaml", tmp_path / "b.yaml"
    fa.write_text(yaml.safe_dump(a))
    fb.write_text(yaml.safe_dump(b))
    proj = lk.project("quickstart", "qs-multikc")
    env = dict(lk.env, KUBECONFIG=f"{fa}:{fb}")
    p = subprocess.run([lk.bin, "deploy"], cwd=proj, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    p = subprocess.run([lk.bin, "purge"], cwd=proj, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
