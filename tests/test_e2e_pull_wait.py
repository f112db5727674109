"""Pull-aware rollout wait. A first `rocm/pytorch` pull onto a fresh MI355X node
routinely outlasts the 300 s GPU rollout timeout; the original purges a first install on timeout
(/root/reference/pkg/devspace/helm/install.go:155-161), deleting the pod mid-pull. Here a pod
whose kubelet reports `Pulling` extends the wait (up to DEVSPACE_PULL_TIMEOUT), pods that can
never start fail within seconds with the analyze report, and a first install whose pull is still
going when the budget runs out is kept.

Time-scaled on the local cluster's slow-pull mode: an 8 s pull against a 4 s rollout timeout
stands for a 600 s pull against the 300 s GPU default."""

import os
import time

import yaml

from conftest import DevspaceEnv


def _cluster(tmp_path, pull_seconds, gpus=1):
    from devspace_amd.localkube import LocalCluster

    cluster = LocalCluster(str(tmp_path / "state"), gpus=gpus).start()
    cluster.kubelet.pull_seconds = pull_seconds
    return cluster, DevspaceEnv(cluster, str(tmp_path))


def _set_timeout(proj, seconds):
    p = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(p))
    cfg["deployments"][0]["helm"]["timeout"] = seconds
    open(p, "w").write(yaml.safe_dump(cfg))


def _releases(cluster, ns):
    return sorted((s["metadata"]["labels"].get("version"), s["metadata"]["labels"].get("status"))
                  for s in cluster.store.list("", "secrets", ns, "owner=helm"))


def _events(cluster, ns, reason):
    return [e for e in cluster.store.list("", "events", ns) if e["reason"] == reason]


def test_gpu_chart_waits_out_a_long_image_pull(tmp_path):
    cluster, lk = _cluster(tmp_path, pull_seconds=8.0)
    try:
        proj = lk.project("rocm-pytorch")
        _set_timeout(proj, 4)
        t0 = time.time()
        r = lk.run(["deploy"], proj, timeout=120, check=False)
        took = time.time() - t0
        out = r.stdout + r.stderr
        assert r.returncode == 0, out
        assert "Successfully deployed!" in out, out
        assert took >= 8.0, (took, out)  # it did wait for the pull, past the 4 s timeout
        assert "waiting for the pull" in out, out
        # one install, never purged: one revision, deployed; one pod, pulled once
        assert _releases(cluster, "rocm-pytorch") == [("1", "deployed")], _releases(cluster, "rocm-pytorch")
        pods = cluster.store.list("", "pods", "rocm-pytorch")
        assert len(pods) == 1 and pods[0]["status"]["phase"] == "Running", pods
        assert len(_events(cluster, "rocm-pytorch", "Pulling")) == 1
        assert "Keeping release" not in out
    finally:
        cluster.stop()


def test_image_pull_backoff_fails_within_seconds_with_report(tmp_path):
    cluster, lk = _cluster(tmp_path, pull_seconds=8.0, gpus=0)
    try:
        proj = lk.project("quickstart")
        values = os.path.join(proj, "chart", "values.yaml")
        v = yaml.safe_load(open(values))
        v["components"][0]["containers"][0]["image"] = "registry.invalid/team/missing:1.0"
        open(values, "w").write(yaml.safe_dump(v))
        t0 = time.time()
        r = lk.run(["deploy"], proj, timeout=120, check=False)
        took = time.time() - t0
        out = r.stdout + r.stderr
        assert r.returncode != 0, out
        assert took < 15, (took, out)  # not the 40 s rollout timeout
        assert "rollout failed" in out and ("ErrImagePull" in out or "ImagePullBackOff" in out), out
        assert "Problems" in out and "registry.invalid/team/missing" in out, out  # the analyze report
    finally:
        cluster.stop()


def test_first_install_still_pulling_at_the_budget_is_kept(tmp_path):
    """The pull budget runs out with the pull still going: the command fails, says why, and keeps
    the release and its pod (the pull goes on); the next deploy picks the wait up and succeeds."""
    cluster, lk = _cluster(tmp_path, pull_seconds=10.0)
    try:
        proj = lk.project("rocm-pytorch")
        _set_timeout(proj, 2)
        lk.env["DEVSPACE_PULL_TIMEOUT"] = "4"
        r = lk.run(["deploy"], proj, timeout=120, check=False)
        out = r.stdout + r.stderr
        assert r.returncode != 0, out
        assert "is still in progress" in out and "Keeping release" in out, out
        assert _releases(cluster, "rocm-pytorch") == [("1", "failed")], _releases(cluster, "rocm-pytorch")
        pods = cluster.store.list("", "pods", "rocm-pytorch")
        assert len(pods) == 1, pods
        first_pod = pods[0]["metadata"]["uid"]
        lk.env["DEVSPACE_PULL_TIMEOUT"] = "60"
        r = lk.run(["deploy"], proj, timeout=120, check=False)
        out = r.stdout + r.stderr
        assert r.returncode == 0, out
        pods = cluster.store.list("", "pods", "rocm-pytorch")
        assert [p["metadata"]["uid"] for p in pods] == [first_pod]  # the same pod, its pull never restarted
        assert ("2", "deployed") in _releases(cluster, "rocm-pytorch"), _releases(cluster, "rocm-pytorch")
        assert len(_events(cluster, "rocm-pytorch", "Pulling")) == 1
    finally:
        cluster.stop()


def test_a_transient_pull_error_is_waited_out(tmp_path):
    """an ErrImagePull the kubelet can get past (the registry timed out) is not fatal
    at the first look: the wait goes on while the kubelet retries, and the deploy succeeds."""
    cluster, lk = _cluster(tmp_path, pull_seconds=0.0, gpus=0)
    try:
        proj = lk.project("quickstart")
        cluster.kubelet.pull_flaky[""] = time.monotonic() + 5.0
        t0 = time.time()
        r = lk.run(["deploy"], proj, timeout=120, check=False)
        took = time.time() - t0
        out = r.stdout + r.stderr
        assert r.returncode == 0, out
        assert took >= 4.0, (took, out)
        assert "i/o timeout" in out and "the kubelet retries the pull" in out, out
    finally:
        cluster.stop()


def test_a_pull_error_that_lasts_fails_after_the_grace(tmp_path):
    cluster, lk = _cluster(tmp_path, pull_seconds=0.0, gpus=0)
    try:
        proj = lk.project("quickstart")
        cluster.kubelet.pull_flaky[""] = time.monotonic() + 120.0
        lk.env["DEVSPACE_PULL_ERROR_GRACE_S"] = "3"
        t0 = time.time()
        r = lk.run(["deploy"], proj, timeout=120, check=False)
        took = time.time() - t0
        out = r.stdout + r.stderr
        assert r.returncode != 0, out
        assert 3.0 <= took < 20, (took, out)  # the grace, not the 40 s rollout timeout
        assert "rollout failed" in out and "i/o timeout" in out, out
    finally:
        cluster.stop()
