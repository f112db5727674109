"""Server-side apply against an API server that enforces immutable fields, PV binding and
pvc-protection (devspace_amd.localkube): redeploys keep PersistentVolumeClaims (same UID, the
binder's spec.volumeName intact), Services keep their clusterIP, immutable changes fail with a
hint unless --force-recreate, and a claim in use survives its own deletion until the pod goes.

Reference behaviour: `kubectl apply --force` (deploy/kubectl/kubectl.go:79-160) and Helm
upgrade (helm/install.go:100-166) — both merge into live objects instead of replacing them."""

import json
import os
import urllib.request

import yaml

from test_e2e_cli import running, wait_for


def _ns_project(lk, example, name, ns, wait=True):
    proj = lk.project(example, name)
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["cluster"]["namespace"] = ns
    if not wait:  # php-mysql's mysql:8 image is not in the offline local registry: do not wait
        for d in cfg["deployments"]:
            d["helm"]["wait"] = False
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    return proj


def _pvcs(lk, ns):
    return lk.cluster.store.list("", "persistentvolumeclaims", ns)


def test_redeploy_keeps_pvc_and_service_identity(localkube):
    lk = localkube
    ns = "ssa-php"
    proj = _ns_project(lk, "php-mysql-example", "php-ssa", ns, wait=False)
    lk.run(["deploy"], proj)
    wait_for(lambda: lk.pods(ns), timeout=60, what="pods")
    pvc = wait_for(lambda: [p for p in _pvcs(lk, ns) if (p["spec"] or {}).get("volumeName")], what="bound pvc")[0]
    uid, vol = pvc["metadata"]["uid"], pvc["spec"]["volumeName"]
    svc = lk.cluster.store.list("", "services", ns)[0]
    svc_uid, cluster_ip = svc["metadata"]["uid"], svc["spec"]["clusterIP"]
    assert cluster_ip

    # change the workload and force a redeploy: the PVC spec re-rendered without volumeName
    values = os.path.join(proj, "chart", "values.yaml")
    v = yaml.safe_load(open(values))
    v["components"][0]["containers"][0]["env"].append({"name": "REDEPLOY", "value": "1"})
    open(values, "w").write(yaml.safe_dump(v))
    for _ in range(2):
        lk.run(["deploy", "-d"], proj)
    pvc2 = [p for p in _pvcs(lk, ns) if p["metadata"]["name"] == pvc["metadata"]["name"]][0]
    assert pvc2["metadata"]["uid"] == uid
    assert pvc2["spec"]["volumeName"] == vol
    assert not pvc2["metadata"].get("deletionTimestamp")
    mf = {m["manager"] for m in pvc2["metadata"].get("managedFields") or []}
    assert "devspace" in mf, pvc2["metadata"]
    svc2 = lk.cluster.store.get("", "services", ns, svc["metadata"]["name"])
    assert svc2["metadata"]["uid"] == svc_uid and svc2["spec"]["clusterIP"] == cluster_ip
    lk.run(["purge"], proj)


def test_fields_dropped_from_the_chart_are_removed(localkube):
    lk = localkube
    ns = "ssa-prune"
    proj = _ns_project(lk, "quickstart", "qs-ssa-prune", ns)
    values = os.path.join(proj, "chart", "values.yaml")
    v = yaml.safe_load(open(values))
    v["components"][0]["containers"][0]["env"] = [{"name": "KEEP", "value": "1"}, {"name": "DROP", "value": "2"}]
    open(values, "w").write(yaml.safe_dump(v))
    lk.run(["deploy"], proj)
    wait_for(lambda: running(lk.pods(ns)), timeout=60, what="pod")
    v["components"][0]["containers"][0]["env"] = [{"name": "KEEP", "value": "1"}]
    open(values, "w").write(yaml.safe_dump(v))
    lk.run(["deploy", "-d"], proj)
    dep = lk.cluster.store.list("apps", "deployments", ns)[0]
    env = dep["spec"]["template"]["spec"]["containers"][0]["env"]
    assert [e["name"] for e in env] == ["KEEP"], env
    lk.run(["purge"], proj)


def test_immutable_change_needs_force_recreate(localkube):
    lk = localkube
    ns = "ssa-immut"
    proj = _ns_project(lk, "quickstart-kubectl", "qsk-immut", ns)
    lk.run(["deploy"], proj)
    wait_for(lambda: running(lk.pods(ns)), timeout=60, what="pod")
    dep = lk.cluster.store.list("apps", "deployments", ns)[0]
    old_uid = dep["metadata"]["uid"]
    # change the Deployment's selector (immutable in apps/v1)
    kdir = os.path.join(proj, "kube")
    for fn in os.listdir(kdir):
        p = os.path.join(kdir, fn)
        docs = list(yaml.safe_load_all(open(p)))
        for d in docs:
            if d and d.get("kind") == "Deployment":
                d["spec"]["selector"]["matchLabels"]["tier"] = "web"
                d["spec"]["template"]["metadata"]["labels"]["tier"] = "web"
        open(p, "w").write(yaml.safe_dump_all(docs))
    p = lk.run(["deploy", "-d"], proj, check=False)
    assert p.returncode != 0
    assert "immutable" in (p.stdout + p.stderr) and "--force-recreate" in (p.stdout + p.stderr), p.stdout + p.stderr
    assert lk.cluster.store.list("apps", "deployments", ns)[0]["metadata"]["uid"] == old_uid
    lk.run(["deploy", "-d", "--force-recreate"], proj)
    dep = lk.cluster.store.list("apps", "deployments", ns)[0]
    assert dep["metadata"]["uid"] != old_uid
    assert dep["spec"]["selector"]["matchLabels"]["tier"] == "web"
    lk.run(["purge", "-d", "devspace-default"], proj)


def test_pvc_protection_holds_claim_while_pod_uses_it(localkube):
    """The fake API server's pvc-protection (what a real cluster does to a deleted claim)."""
    lk = localkube
    ns = "ssa-protect"
    proj = _ns_project(lk, "php-mysql-example", "php-protect", ns, wait=False)
    lk.run(["deploy"], proj)
    wait_for(lambda: lk.pods(ns), timeout=60, what="pods")
    pvc = wait_for(lambda: _pvcs(lk, ns), what="pvc")[0]
    name = pvc["metadata"]["name"]
    base = lk.cluster.server
    req = urllib.request.Request(f"{base}/api/v1/namespaces/{ns}/persistentvolumeclaims/{name}", method="DELETE",
                                 headers={"Authorization": "Bearer x"})
    json.loads(urllib.request.urlopen(req).read())
    still = lk.cluster.store.try_get("", "persistentvolumeclaims", ns, name)
    assert still and still["metadata"].get("deletionTimestamp"), still
    lk.run(["purge"], proj)
    wait_for(lambda: not lk.pods(ns), timeout=60, what="pods gone")
    wait_for(lambda: not lk.cluster.store.try_get("", "persistentvolumeclaims", ns, name), timeout=30,
             what="claim released")
