"""MI355X nodes as the AMD GPU device plugin and node labeller present them, end to
end through the CLI against the local cluster (CPU only: no device is opened here).

* CPX compute partitioning: 8 MI355X become 64 schedulable `amd.com/gpu` devices with an even
  36 GB share of HBM each; `devspace init` offers up to 64 and sizes CPU/memory per partition.
* Unhealthy devices (capacity > allocatable) are reported by `devspace analyze`.
* A pod that cannot get its devices is told who holds them.

The reference's counterparts: the chart's per-container resources block
(/root/reference/examples/quickstart/chart/templates/deployments.yaml:63-82) and the pod checks of
analyze (/root/reference/pkg/devspace/analyze/pods.go:158).
"""
import os

import yaml

from conftest import DevspaceEnv


def _cluster(tmp_path, **kw):
    from devspace_amd.localkube import LocalCluster

    c = LocalCluster(str(tmp_path / "state"), **kw).start()
    return c, DevspaceEnv(c, str(tmp_path))


def test_init_on_a_cpx_node_offers_64_partitions_with_their_hbm_share(tmp_path):
    cluster, lk = _cluster(tmp_path, gpus=8, gpu_partition="cpx", memory_partition="nps2")
    try:
        node = cluster.store.list("", "nodes", "")[0]
        assert node["status"]["allocatable"]["amd.com/gpu"] == "64"

        def project(name):
            proj = os.path.join(lk.base, name)
            os.makedirs(proj, exist_ok=True)
            with open(os.path.join(proj, "train.py"), "w") as f:
                f.write("import torch\nprint(torch.__version__)\n")
            return proj

        # 65 is past the node's 64 devices: refused
        r = lk.run(["init"], project("init-cpx65"), input="\n65\n", check=False)
        assert r.returncode != 0 and "answer '65' does not match" in r.stdout + r.stderr, r.stdout + r.stderr
        proj = project("init-cpx")
        answers = "\n16\ncpx-ns\n\nlocal.registry\nlocal.registry/cpx\nno\n"
        out = lk.run(["init"], proj, input=answers).stdout
        assert "Project successfully initialized" in out, out
        assert "Sizing the pod for 16 device(s) (node devspace-local: 8 x AMD_Instinct_MI355X, CPX/NPS2: 64 " \
               "schedulable amd.com/gpu of 36 GB HBM each" in out, out
        assert "HBM per device: 36 GB (CPX/NPS2 partition)" in out, out
        values_text = open(os.path.join(proj, "chart", "values.yaml")).read()
        assert "CPX/NPS2 partition with an even" in values_text and "36 GB (576 GB for the 16 devices)" in values_text
        values = yaml.safe_load(values_text)
        res = values["components"][0]["containers"][0]["resources"]
        assert res["limits"]["gpu"] == 16
        # a 64th of the node per device (os.cpu_count() cores, 64 Gi), not an 8th; with fewer CPUs
        # than devices the pod gets its share of 90 % of them, never one CPU per device
        share = (os.cpu_count() or 1) * 0.9 / 64
        want = str(16 * int(share)) if share >= 1 else (str(int(16 * share)) if 16 * share >= 1
                                                           else f"{max(100, int(16 * share * 10) * 100)}m")
        assert res["limits"]["cpu"] == want and res["requests"]["cpu"] == want, res
        if share < 1:
            assert "fewer than one CPU each" in out, out
    finally:
        cluster.stop()


def _wait_false(proj, namespace=None):
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    raw = open(cfg_path).read().replace("chartPath: ./chart", "chartPath: ./chart\n    wait: false")
    if namespace:
        raw = raw.replace("namespace: rocm-pytorch", f"namespace: {namespace}")
    open(cfg_path, "w").write(raw)


def test_analyze_reports_an_unhealthy_gpu(tmp_path):
    cluster, lk = _cluster(tmp_path, gpus=2, unhealthy_gpus=1)
    try:
        proj = lk.project("rocm-pytorch")
        _wait_false(proj)
        lk.run(["deploy"], proj, timeout=180)
        report = lk.run(["analyze", "--wait=false", "-n", "rocm-pytorch"], proj, check=False).stdout
        assert "node devspace-local: 1 of 2 amd.com/gpu unhealthy (capacity 2, allocatable 1)" in report, report
        lk.run(["purge"], proj, check=False)
    finally:
        cluster.stop()


def test_analyze_names_the_pods_holding_the_gpus(tmp_path):
    """One device on the node, held by a pod of another namespace: the second pod's report names
    the holder instead of leaving "Insufficient amd.com/gpu" to guesswork."""
    cluster, lk = _cluster(tmp_path, gpus=1)
    try:
        a = lk.project("rocm-pytorch", "proj-a")
        _wait_false(a, "team-a")
        lk.run(["deploy"], a, timeout=180)
        b = lk.project("rocm-pytorch", "proj-b")
        _wait_false(b, "team-b")
        lk.run(["deploy"], b, timeout=180, check=False)
        holder = [p["metadata"]["name"] for p in cluster.store.list("", "pods", "team-a")][0]
        from test_e2e_cli import wait_for  # noqa: WPS433

        wait_for(lambda: [p for p in cluster.store.list("", "pods", "team-b")
                          if any(c.get("reason") == "Unschedulable" for c in (p.get("status") or {}).get("conditions") or [])],
                 what="unschedulable pod")
        report = lk.run(["analyze", "--wait=false", "-n", "team-b"], b, check=False).stdout
        assert f"waits for 1 GPU device(s); node devspace-local (1 amd.com/gpu) has them held by team-a/{holder} (1)" \
            in report, report
        lk.run(["purge"], b, check=False)
        lk.run(["purge"], a, check=False)
    finally:
        cluster.stop()
