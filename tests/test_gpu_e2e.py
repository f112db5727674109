"""MI355X end to end: a GPU-enabled local cluster (amd.com/gpu from the KFD topology) runs the
examples/rocm-pytorch training pod through `devspace deploy`; `devspace analyze --gpu-probe`
runs the gfx950 probe kernels inside the pod."""

import json
import os
import time

import pytest

from conftest import DevspaceEnv


def _wait(fn, timeout, what):
    deadline = time.time() + timeout
    while time.time() < deadline:
        v = fn()
        if v:
            return v
        time.sleep(0.2)
    raise AssertionError("timed out waiting for " + what)


@pytest.mark.gpu
def test_rocm_pytorch_pod_trains_on_gpu(tmp_path):
    from devspace_amd.localkube import LocalCluster, detect_gpus

    gpus = detect_gpus()
    assert gpus >= 1, "no GPU in the KFD topology"
    cluster = LocalCluster(str(tmp_path / "state"), gpus=gpus).start()
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        proj = lk.project("rocm-pytorch")
        node = cluster.store.get("", "nodes", "", "devspace-local")
        assert node["status"]["allocatable"]["amd.com/gpu"] == str(gpus)
        out = lk.run(["deploy"], proj, timeout=600).stdout
        assert "Successfully deployed!" in out
        pod = _wait(lambda: [p for p in lk.pods("rocm-pytorch") if p["status"].get("phase") == "Running"], 120,
                    "running pod")[0]
        root = json.loads(pod["metadata"]["annotations"]["devspace.sh/local-roots"])[
            pod["spec"]["containers"][0]["name"]]
        log = _wait(lambda: (open(root + ".log").read() if os.path.exists(root + ".log") else "")
                    if "started gen=" in (open(root + ".log").read() if os.path.exists(root + ".log") else "")
                    else None, 300, "runner start")
        assert "device=cuda:0" in log, log
        report = lk.run(["analyze", "--wait=false", "--gpu-probe", "-n", "rocm-pytorch"], proj, timeout=300).stdout
        assert "GPU" not in report or "No problems found" in report, report
        lk.run(["purge"], proj, timeout=120)
    finally:
        cluster.stop()
