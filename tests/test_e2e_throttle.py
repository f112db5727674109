"""The CLI against a throttling API server: API Priority and Fairness answers
`429 Too Many Requests` + `Retry-After` on busy clusters. client-go (the reference's transport,
/root/reference/pkg/devspace/kubectl/client.go:34-51) waits and retries; so must every call of the
rebuild: REST CRUD, server-side apply, list+watch, logs, and the exec / port-forward upgrades
behind sync and port-forwarding.

The local cluster's fault switch answers the first request of every (verb, resource) with 429
Retry-After: 1, afresh for each command."""

import os
import socket
import urllib.request

import pytest
import yaml

from conftest import DevspaceEnv
from test_e2e_cli import container_root, running, wait_for
from test_e2e_services import _stop

THROTTLE_LOG = "The API server is throttling requests"


@pytest.fixture(scope="module")
def throttled(tmp_path_factory):
    from devspace_amd.localkube import LocalCluster

    base = str(tmp_path_factory.mktemp("lk-throttle"))
    cluster = LocalCluster(os.path.join(base, "state"), gpus=0).start()
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


def _throttle(lk):
    lk.cluster.api.reset_throttle(first=1, retry_after=1)


def _verbs(lk):
    return {verb for verb, _ in lk.cluster.api.throttled}


def test_deploy_dev_logs_purge_complete_under_429(throttled):
    lk = throttled
    proj = lk.project("quickstart", "quickstart-429")
    remote, local = _free_port(), _free_port()
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["dev"].pop("overrideImages")  # the app itself runs: port-forwarding has a server to reach
    cfg["dev"]["ports"][0]["portMappings"] = [{"localPort": local, "remotePort": remote}]
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    values = os.path.join(proj, "chart", "values.yaml")
    v = yaml.safe_load(open(values))
    v["components"][0]["containers"][0]["env"] = [{"name": "PORT", "value": str(remote)}]
    open(values, "w").write(yaml.safe_dump(v))

    _throttle(lk)
    out = lk.run(["deploy"], proj, timeout=300).stdout
    assert "Successfully deployed!" in out, out
    assert out.count(THROTTLE_LOG) == 1, out  # logged once, not per retry
    assert {"create", "get", "patch"} & _verbs(lk), lk.cluster.api.throttled
    wait_for(lambda: running(lk.pods("quickstart")), timeout=60, what="pod")

    _throttle(lk)
    dev = lk.popen(["dev", "--terminal=false"], proj)
    try:
        pods = wait_for(lambda: running(lk.pods("quickstart")), timeout=120, what="dev pod")

        def fetch():
            try:
                return urllib.request.urlopen(f"http://127.0.0.1:{local}/", timeout=2).read().decode()
            except Exception:
                return None

        assert wait_for(fetch, timeout=120, what="forwarded response").startswith("Hello")
        root = container_root(lk, running(lk.pods("quickstart"))[0])
        with open(os.path.join(proj, "index.js"), "a") as f:
            f.write("// edit under throttling\n")
        wait_for(lambda: "// edit under throttling" in open(os.path.join(root, "app", "index.js")).read(),
                 timeout=60, what="upstream sync")
        # the exec (sync) and port-forward upgrades were throttled and retried
        assert "connect" in _verbs(lk), lk.cluster.api.throttled
        assert any(r.startswith("pods/portforward") for _, r in lk.cluster.api.throttled), lk.cluster.api.throttled
        assert any(r.startswith("pods/exec") for _, r in lk.cluster.api.throttled), lk.cluster.api.throttled
    finally:
        out = _stop(dev)
    assert "Sync started" in out and "Port forwarding started" in out, out
    assert out.count(THROTTLE_LOG) == 1, out

    _throttle(lk)
    out = lk.run(["logs"], proj, timeout=120).stdout
    assert "listening" in out, out
    assert ("get", "pods/log") in lk.cluster.api.throttled, lk.cluster.api.throttled

    _throttle(lk)
    lk.run(["purge"], proj, timeout=300)
    assert "delete" in _verbs(lk) or "deletecollection" in _verbs(lk), lk.cluster.api.throttled
    wait_for(lambda: not lk.pods("quickstart"), timeout=60, what="pods deleted")
    lk.cluster.api.reset_throttle(first=0)
