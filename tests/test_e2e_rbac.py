"""A namespace-scoped user (RBAC: a Role + RoleBinding in one namespace, as DevSpace.cloud Spaces
and most multi-tenant clusters hand out): no access to nodes, namespaces or anything else at the
cluster scope. deploy / dev (sync + port-forward) / logs / analyze / purge must work with only
that, degrading the cluster-scoped extras (GPU capacity checks, namespace creation) instead of
failing. The local cluster's RBAC mode answers 403 Forbidden like a real API server."""

import os
import socket
import urllib.request

import pytest
import yaml

from conftest import DevspaceEnv
from test_e2e_cli import container_root, running, wait_for
from test_e2e_services import _stop

NS = "team-a"
TOKEN = "team-a-developer-token"


@pytest.fixture(scope="module")
def scoped(tmp_path_factory):
    from devspace_amd.localkube import LocalCluster

    base = str(tmp_path_factory.mktemp("lk-rbac"))
    cluster = LocalCluster(os.path.join(base, "state"), gpus=0).start()
    try:
        # the cluster admin created the namespace and bound the developer to it
        cluster.store.create("", "namespaces", "", {"apiVersion": "v1", "kind": "Namespace",
                                                    "metadata": {"name": NS}}, "v1")
        cluster.api.scoped_tokens[TOKEN] = NS
        env = DevspaceEnv(cluster, base)
        kc = yaml.safe_load(open(env.kubeconfig))
        for u in kc["users"]:
            u["user"] = {"token": TOKEN}
        for c in kc["contexts"]:
            c["context"]["namespace"] = NS
        open(env.kubeconfig, "w").write(yaml.safe_dump(kc))
        yield env
    finally:
        cluster.stop()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_namespace_scoped_user_deploys_develops_and_purges(scoped):
    lk = scoped
    proj = lk.project("quickstart", "quickstart-rbac")
    remote, local = _free_port(), _free_port()
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["cluster"]["namespace"] = NS
    cfg["dev"].pop("overrideImages")
    cfg["dev"]["ports"][0]["portMappings"] = [{"localPort": local, "remotePort": remote}]
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    values = os.path.join(proj, "chart", "values.yaml")
    v = yaml.safe_load(open(values))
    v["components"][0]["containers"][0]["env"] = [{"name": "PORT", "value": str(remote)}]
    open(values, "w").write(yaml.safe_dump(v))

    out = lk.run(["deploy"], proj, timeout=300).stdout
    assert "Successfully deployed!" in out, out
    assert "Created namespace" not in out  # it could not even read it: not an error
    wait_for(lambda: running(lk.pods(NS)), timeout=60, what="pod")

    dev = lk.popen(["dev", "--terminal=false"], proj)
    try:
        def fetch():
            try:
                return urllib.request.urlopen(f"http://127.0.0.1:{local}/", timeout=2).read().decode()
            except Exception:
                return None

        assert wait_for(fetch, timeout=60, what="forwarded response").startswith("Hello")
        root = container_root(lk, running(lk.pods(NS))[0])
        with open(os.path.join(proj, "index.js"), "a") as f:
            f.write("// scoped edit\n")
        wait_for(lambda: "// scoped edit" in open(os.path.join(root, "app", "index.js")).read(), timeout=30,
                 what="upstream sync")
    finally:
        out = _stop(dev)
    assert "Sync started" in out and "Port forwarding started" in out, out

    assert "listening" in lk.run(["logs"], proj, timeout=60).stdout
    assert '"name": "quickstart"' in lk.run(["enter", "--", "cat", "package.json"], proj, timeout=60).stdout
    out = lk.run(["analyze", "--wait=false"], proj, timeout=60).stdout
    assert "No problems found" in out, out
    lk.run(["purge"], proj, timeout=120)
    wait_for(lambda: not lk.pods(NS), timeout=60, what="pods deleted")
    # the API server did refuse the cluster-scoped reads along the way
    assert lk.cluster.api.forbidden > 0


def test_namespace_scoped_user_sees_a_clear_error_outside_its_namespace(scoped):
    """Deploying into a namespace the user has no rights in fails with the API server's reason,
    not a crash or a silent success."""
    lk = scoped
    proj = lk.project("quickstart", "quickstart-rbac-other")
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["cluster"]["namespace"] = "someone-else"
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    r = lk.run(["deploy"], proj, timeout=120, check=False)
    out = r.stdout + r.stderr
    assert r.returncode != 0, out
    assert "forbidden" in out.lower(), out
