"""The Kubernetes transports over TLS: server verified against certificate-authority-data,
client authenticated with client-certificate-data/client-key-data (mTLS), for REST, exec
WebSocket (wss) and log streaming."""

import os

import pytest
import yaml

from conftest import DevspaceEnv
from test_e2e_cli import running, wait_for


@pytest.fixture(scope="module")
def tls_kube(tmp_path_factory):
    from devspace_amd.localkube import LocalCluster

    base = str(tmp_path_factory.mktemp("lktls"))
    cluster = LocalCluster(os.path.join(base, "state"), gpus=0, tls=True).start()
    try:
        yield DevspaceEnv(cluster, base)
    finally:
        cluster.stop()


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
