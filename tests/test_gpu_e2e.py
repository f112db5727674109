"""MI355X end to end: a GPU-enabled local cluster (amd.com/gpu from the KFD topology) runs the
examples/rocm-pytorch training pod through `devspace deploy`; `devspace analyze --gpu-probe`
runs the gfx950 probe kernels inside the pod."""

import glob
import json
import os
import re
import shutil
import sys
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
        prof = os.environ.get("DEVSPACE_E2E_POD_PROFILE")
        if prof:
            # profile the workload inside the pod, as one would on a real node: the container
            # command runs the image's entrypoint under rocprofv3 (kernel trace, written when
            # the runner exits on the pod's SIGTERM at purge)
            import yaml

            rocprof = shutil.which("rocprofv3")
            assert rocprof, "rocprofv3 not on PATH"
            prof = os.path.realpath(prof)
            os.makedirs(prof, exist_ok=True)
            vpath = os.path.join(proj, "chart", "values.yaml")
            v = yaml.safe_load(open(vpath))
            v["components"][0]["containers"][0]["command"] = [
                rocprof, "--kernel-trace", "--stats", "-d", prof, "-o", "pod", "--",
                sys.executable, "-m", "devspace_amd.runner", "--watch", "/app", "train.py"]
            with open(vpath, "w") as f:
                yaml.safe_dump(v, f, sort_keys=False)
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
        # the pod runs the workload kit vendored into the project (no devspace checkout on its
        # Python path, as in a real image) and the gfx950 kernels, not an eager fallback
        assert re.search(r"kit=" + re.escape(root), log), log
        assert "[devspace-runner] fused=hip" in log, log
        r = lk.run(["analyze", "--wait=false", "--gpu-probe", "-n", "rocm-pytorch"], proj, timeout=300)
        report = r.stdout + r.stderr
        # the probe ran inside the pod and exercised every granted device (MFMA self-test)
        assert "No problems found" in report, report
        m = re.search(r"GPU probe of pod \S+: (\d+) device\(s\) checked by the (\w+) probe: (.*)", report)
        assert m, report
        granted = int(pod["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"])
        assert int(m.group(1)) == granted and m.group(2) in ("devspace", "torch"), report
        assert "gfx950" in m.group(3), report
        if m.group(2) == "devspace":
            assert re.search(r"MFMA self-test err 0(\.0)?(,|$)", m.group(3)), report
        workload = []
        if prof:
            import psutil

            for pr in psutil.process_iter(["cmdline"]):
                try:
                    if "devspace_amd.runner" in " ".join(pr.info["cmdline"] or []) and \
                            pr.environ().get("DEVSPACE_CONTAINER_ROOT") == root:
                        workload.append(pr)
                except (psutil.Error, OSError):
                    pass
            assert workload, "profiled runner process not found"
        lk.run(["purge"], proj, timeout=120)
        if prof:
            # the trace is written when the runner exits (SIGTERM from the pod deletion)
            _, alive = psutil.wait_procs(workload, timeout=90)
            assert not alive, alive
            dbs = _wait(lambda: glob.glob(os.path.join(prof, "**", "*.db"), recursive=True) or
                        glob.glob(os.path.join(prof, "**", "*kernel_stats.csv"), recursive=True), 60,
                        "the pod's rocprofv3 output")
            print("pod profile:", dbs)
    finally:
        cluster.stop()


@pytest.mark.gpu
def test_two_rank_gpu_pod_contains_a_rank_failure_and_analyze_explains_it(tmp_path):
    """The rocm-pytorch pod with amd.com/gpu: 2 (both ranks on the box's one MI355X, joined over
    gloo), through `devspace deploy`: an edit that breaks rank 1 stops and parks the training
    group, `devspace analyze` names the failing rank and its exception, and the fix brings the
    group back on the GPU."""
    from devspace_amd.localkube import LocalCluster

    cluster = LocalCluster(str(tmp_path / "state"), gpus=2).start()
    cluster.kubelet.extra_env["DEVSPACE_DIST_BACKEND"] = "gloo"  # RCCL refuses two ranks on one GPU
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        proj = lk.project("rocm-pytorch")
        vpath = os.path.join(proj, "chart", "values.yaml")
        v = open(vpath).read()
        with open(vpath, "w") as f:
            f.write(re.sub(r"gpu: \d+", "gpu: 2", v))
        assert "Successfully deployed!" in lk.run(["deploy"], proj, timeout=600).stdout
        pod = _wait(lambda: [p for p in lk.pods("rocm-pytorch") if p["status"].get("phase") == "Running"], 120,
                    "running pod")[0]
        root = json.loads(pod["metadata"]["annotations"]["devspace.sh/local-roots"])[
            pod["spec"]["containers"][0]["name"]]

        def log():
            return open(root + ".log").read() if os.path.exists(root + ".log") else ""

        _wait(lambda: "started gen=1" in log(), 300, "runner start")
        assert re.search(r"started gen=1 .*world=2 device=cuda", log()), log()[-3000:]
        train = os.path.join(root, "app", "train.py")  # what `devspace dev` syncs into the pod
        good = open(train).read()
        bad = good.replace("def step(ctx, state):\n",
                           "def step(ctx, state):\n    if ctx.rank == 1:\n"
                           "        raise ValueError('rank 1 sees a bad batch')\n", 1)
        assert bad != good
        with open(train + ".tmp", "w") as f:
            f.write(bad)
        os.rename(train + ".tmp", train)
        _wait(lambda: "waiting for a file change before starting the group again" in log(), 180, "group parked")
        r = lk.run(["analyze", "--wait=false", "-n", "rocm-pytorch"], proj, timeout=120, check=False)
        report = r.stdout + r.stderr
        assert "training group is down after rank=1" in report, report
        assert "ValueError: rank 1 sees a bad batch" in report, report
        n_started = log().count("started gen=1")
        with open(train + ".tmp", "w") as f:
            f.write(good.replace('MARKER = "v0"', 'MARKER = "fixed"'))
        os.rename(train + ".tmp", train)
        _wait(lambda: log().count("started gen=1") > n_started and "marker=fixed" in log(), 240, "group back")
        assert re.search(r"started gen=1 marker=fixed .*world=2 device=cuda", log()), log()[-3000:]
        r = lk.run(["analyze", "--wait=false", "-n", "rocm-pytorch"], proj, timeout=120, check=False)
        assert "training group is down" not in r.stdout, r.stdout
    finally:
        cluster.stop()
