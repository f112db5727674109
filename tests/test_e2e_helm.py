"""Helm 3 semantics end to end through `devspace deploy` / `purge` on the local cluster:
lifecycle hooks (pre-install Job that must complete, post-install hooks with delete policies,
`test` hooks never run), failed hooks rolling an upgrade back, release records stored as real
Helm 3 Secrets (decoded here against the pkg/release/release.go schema), and dependency
conditions / .Files / .Capabilities from the API server's discovery on a live cluster.

Reference: helm/install.go:54-166 (install/upgrade via Tiller, Helm 2), which this replaces with
native Helm 3 semantics (SURVEY §2.3 helm adapter)."""

import base64
import gzip
import json
import os
import shutil

import yaml

from conftest import ROOT
from test_e2e_cli import wait_for

CHARTS = os.path.join(ROOT, "tests", "fixtures", "charts")


def _helm_project(lk, chart, name, ns, values=None):
    proj = os.path.join(lk.base, name)
    if os.path.exists(proj):
        shutil.rmtree(proj)
    os.makedirs(os.path.join(proj, ".devspace"))
    shutil.copytree(os.path.join(CHARTS, chart), os.path.join(proj, "chart"), symlinks=True)
    dep = {"name": "rel", "helm": {"chartPath": "./chart", "timeout": 60}}
    if values:
        dep["helm"]["overrideValues"] = values
    cfg = {"version": "v1alpha2", "cluster": {"kubeContext": "devspace-local", "namespace": ns},
           "deployments": [dep]}
    with open(os.path.join(proj, ".devspace", "config.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    return proj


def _releases(lk, ns, name="rel"):
    out = []
    for s in lk.cluster.store.list("", "secrets", ns, f"owner=helm,name={name}"):
        raw = base64.b64decode(base64.b64decode(s["data"]["release"]))
        rel = json.loads(gzip.decompress(raw))
        out.append((s, rel))
    return sorted(out, key=lambda x: x[1]["version"])


def _cm(lk, ns, name):
    return lk.cluster.store.try_get("", "configmaps", ns, name)


def test_hooks_run_in_order_and_release_is_helm3(localkube):
    lk = localkube
    ns = "helm-hooks"
    proj = _helm_project(lk, "hooks-chart", "helm-hooks", ns)
    out = lk.run(["deploy"], proj).stdout
    assert "Running pre-install hook Job/rel-migrate" in out, out
    job = lk.cluster.store.get("batch", "jobs", ns, "rel-migrate")
    assert any(c["type"] == "Complete" and c["status"] == "True" for c in job["status"]["conditions"]), job["status"]
    assert _cm(lk, ns, "rel-app")["data"]["revision"] == "1"
    # hook-succeeded deletes the post hook; the marker (default before-hook-creation) stays
    assert _cm(lk, ns, "rel-post") is None
    assert _cm(lk, ns, "rel-marker")["data"]["installed-at-revision"] == "1"
    # `test` hooks only run under `helm test`
    assert lk.cluster.store.try_get("", "pods", ns, "rel-test") is None

    (secret, rel), = _releases(lk, ns)
    assert secret["type"] == "helm.sh/release.v1"
    assert secret["metadata"]["name"] == "sh.helm.release.v1.rel.v1"
    labels = secret["metadata"]["labels"]
    assert labels["owner"] == "helm" and labels["status"] == "deployed" and labels["version"] == "1"
    # pkg/release/release.go + pkg/chart/chart.go JSON layout
    assert set(rel) >= {"name", "info", "chart", "manifest", "hooks", "version", "namespace"}
    assert rel["name"] == "rel" and rel["namespace"] == ns and rel["version"] == 1
    info = rel["info"]
    assert set(info) >= {"first_deployed", "last_deployed", "deleted", "description", "status"}
    assert info["status"] == "deployed" and info["description"] == "Install complete"
    chart = rel["chart"]
    assert set(chart) >= {"metadata", "lock", "templates", "values", "schema", "files"}
    assert chart["metadata"]["name"] == "hooks-chart" and chart["metadata"]["apiVersion"] == "v2"
    names = sorted(t["name"] for t in chart["templates"])
    assert names == ["templates/app.yaml", "templates/data-pvc.yaml", "templates/migrate-job.yaml",
                     "templates/post-hook.yaml", "templates/test-pod.yaml"], names
    src = {t["name"]: base64.b64decode(t["data"]).decode() for t in chart["templates"]}
    assert "helm.sh/hook" in src["templates/migrate-job.yaml"]
    assert chart["values"] == {"migrate": {"exitCode": 0}}
    # hooks are recorded with events, weights, policies and their last run; not in the manifest
    hooks = {h["name"]: h for h in rel["hooks"]}
    assert set(hooks) == {"rel-migrate", "rel-post", "rel-marker", "rel-test"}
    assert hooks["rel-migrate"]["events"] == ["pre-install", "pre-upgrade"]
    assert hooks["rel-migrate"]["weight"] == -5
    assert hooks["rel-migrate"]["last_run"]["phase"] == "Succeeded"
    assert hooks["rel-post"]["delete_policies"] == ["hook-succeeded"]
    assert hooks["rel-test"]["last_run"] == {}
    assert "rel-migrate" not in rel["manifest"] and "name: rel-app" in rel["manifest"]

    # upgrade: pre-upgrade re-runs the Job (before-hook-creation replaces it), superseded record
    lk.run(["deploy", "-d"], proj)
    rels = _releases(lk, ns)
    assert [r["version"] for _, r in rels] == [1, 2]
    assert rels[0][1]["info"]["status"] == "superseded" and rels[0][0]["metadata"]["labels"]["status"] == "superseded"
    assert rels[1][1]["info"]["status"] == "deployed" and rels[1][1]["info"]["description"] == "Upgrade complete"
    assert rels[1][1]["info"]["first_deployed"] == rels[0][1]["info"]["first_deployed"]
    assert _cm(lk, ns, "rel-app")["data"]["revision"] == "2"
    job2 = lk.cluster.store.get("batch", "jobs", ns, "rel-migrate")
    assert job2["metadata"]["uid"] != job["metadata"]["uid"]

    pvc = lk.cluster.store.get("", "persistentvolumeclaims", ns, "rel-data")
    out = lk.run(["purge"], proj).stdout
    wait_for(lambda: not _releases(lk, ns), timeout=30, what="release secrets purged")
    assert _cm(lk, ns, "rel-app") is None
    # helm.sh/resource-policy: keep survives the uninstall (same object, not recreated)
    kept = lk.cluster.store.try_get("", "persistentvolumeclaims", ns, "rel-data")
    assert kept and kept["metadata"]["uid"] == pvc["metadata"]["uid"], out
    assert "resource-policy: keep" in out, out


def test_failed_pre_upgrade_hook_rolls_back(localkube):
    lk = localkube
    ns = "helm-hookfail"
    proj = _helm_project(lk, "hooks-chart", "helm-hookfail", ns)
    lk.run(["deploy"], proj)
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["deployments"][0]["helm"]["overrideValues"] = {"migrate": {"exitCode": 3}}
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    p = lk.run(["deploy", "-d"], proj, check=False)
    assert p.returncode != 0
    assert "pre-upgrade hook Job/rel-migrate failed" in p.stdout + p.stderr, p.stdout + p.stderr
    rels = _releases(lk, ns)
    st = [(r["version"], r["info"]["status"]) for _, r in rels]
    # rev 2 failed, rev 3 is the rollback to rev 1
    assert st == [(1, "superseded"), (2, "failed"), (3, "deployed")], st
    assert rels[2][1]["info"]["description"] == "Rollback to 1"
    assert _cm(lk, ns, "rel-app")["data"]["revision"] == "1"
    lk.run(["purge"], proj)


def test_dependencies_files_and_capabilities_on_cluster(localkube):
    lk = localkube
    ns = "helm-deps"
    proj = _helm_project(lk, "deps-chart", "helm-deps", ns, values={"workerB": {"enabled": True}})
    lk.run(["deploy"], proj)
    assert _cm(lk, ns, "rel-db") and _cm(lk, ns, "rel-cache") and _cm(lk, ns, "rel-worker-a")
    assert _cm(lk, ns, "rel-worker-b")["data"]["queue"] == "default"
    assert _cm(lk, ns, "must-not-render") is None
    assert _cm(lk, ns, "rel-deps-chart")["data"]["db-exported-user"] == "admin"
    lk.run(["purge"], proj)

    ns = "helm-files"
    proj = _helm_project(lk, "files-chart", "helm-files", ns)
    lk.run(["deploy"], proj)
    caps = _cm(lk, ns, "rel-caps")["data"]
    # from the API server's /version and /apis (localkube reports v1.29.0-devspace-local)
    assert caps["kube"] == "v1.29.0-devspace-local", caps
    assert caps["has-apps"] == "true" and caps["has-bogus"] == "false"
    conf = _cm(lk, ns, "rel-conf")["data"]
    assert conf["a.conf"] == "listen 80\nworkers 4\n" and conf["ignored"] == ""
    (_, rel), = _releases(lk, ns)
    assert rel["info"]["notes"] == "hello from rel in helm-files.\n"
    files = sorted(f["name"] for f in rel["chart"]["files"])
    assert files == ["README.md", "conf/a.conf", "conf/b.conf", "data/lines.txt", "data/token.txt"], files
    lk.run(["purge"], proj)


def test_lookup_keeps_generated_secret_across_upgrades(localkube):
    """Helm 3 `lookup` reads the live cluster during install/upgrade: the chart reuses the
    password it generated on the first install instead of rotating it on every deploy."""
    lk = localkube
    ns = "helm-lookup"
    proj = _helm_project(lk, "lookup-chart", "helm-lookup", ns)
    lk.run(["deploy"], proj)
    pw1 = lk.cluster.store.get("", "secrets", ns, "rel-auth")["data"]["password"]
    assert _cm(lk, ns, "rel-lookup")["data"]["found-before"] == "no"
    lk.run(["deploy", "-d"], proj)
    assert lk.cluster.store.get("", "secrets", ns, "rel-auth")["data"]["password"] == pw1
    cm = _cm(lk, ns, "rel-lookup")["data"]
    assert cm["found-before"] == "yes" and int(cm["configmaps-seen"]) >= 1, cm
    lk.run(["purge"], proj)


def test_values_schema_rejects_invalid_values_before_anything_is_applied(localkube):
    lk = localkube
    ns = "helm-schema"
    proj = _helm_project(lk, "schema-chart", "helm-schema", ns, values={"replicas": 99})
    p = lk.run(["deploy"], proj, check=False)
    out = p.stdout + p.stderr
    assert p.returncode != 0 and "values don't meet the specifications of the schema(s)" in out, out
    assert "replicas: Must be less than or equal to 16" in out, out
    assert _cm(lk, ns, "rel-schema") is None and not _releases(lk, ns)
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["deployments"][0]["helm"]["overrideValues"] = {"replicas": 2}
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    lk.run(["deploy"], proj)
    assert _cm(lk, ns, "rel-schema")["data"]["replicas"] == "2"
    lk.run(["purge"], proj)


def test_release_history_is_pruned(localkube):
    """Helm 3's --history-max: each revision is a Secret with the gzipped chart; a dev session that
    redeploys on every chart edit keeps only the newest `maxHistory` (default 10), never dropping
    the deployed one."""
    lk = localkube
    ns = "helm-history"
    proj = _helm_project(lk, "hooks-chart", "helm-history", ns)
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    cfg["deployments"][0]["helm"]["maxHistory"] = 3
    with open(cfg_path, "w") as f:
        yaml.safe_dump(cfg, f)
    for _ in range(5):
        lk.run(["deploy", "-d"], proj)
    rels = _releases(lk, ns)
    assert [r["version"] for _, r in rels] == [3, 4, 5], [r["version"] for _, r in rels]
    assert rels[-1][1]["info"]["status"] == "deployed"
    assert all(r["info"]["status"] == "superseded" for _, r in rels[:-1])
    lk.run(["purge"], proj)
