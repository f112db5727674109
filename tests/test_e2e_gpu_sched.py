"""GPU scheduling failures and interrupts through the real CLI on a GPU-less local cluster (CPU).

A chart requesting amd.com/gpu that no node can satisfy is reported at once (analyze report
with the FailedScheduling event, repeated scheduler attempts aggregated into one event), not
waited out for the rollout timeout; Ctrl-C ends a one-shot command right away."""

import signal
import subprocess
import threading
import time

from conftest import DevspaceEnv


def test_unschedulable_gpu_chart_fails_fast_with_report(tmp_path):
    from devspace_amd.localkube import LocalCluster

    cluster = LocalCluster(str(tmp_path / "state"), gpus=0).start()
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        proj = lk.project("rocm-pytorch")
        t0 = time.time()
        r = lk.run(["deploy"], proj, timeout=120, check=False)
        elapsed = time.time() - t0
        out = r.stdout + r.stderr
        assert r.returncode != 0, out
        assert elapsed < 30, (elapsed, out)  # not the 300 s GPU rollout timeout
        assert "no node advertises amd.com/gpu" in out, out
        assert "Events (1 potential issue(s))" in out, out
        assert "Insufficient amd.com/gpu" in out, out
        # the scheduler's retries are one Event with a count, as an API server's correlator keeps them
        evs = [e for e in cluster.store.list("", "events", "rocm-pytorch") if e["reason"] == "FailedScheduling"]
        assert len(evs) == 1, evs
    finally:
        cluster.stop()


def test_interrupt_ends_one_shot_command(tmp_path):
    """SIGINT while `deploy` waits on the rollout exits with 130 at once (a Go binary's default);
    before, the flag was only read by the dev loop and the wait ran to its end."""
    from devspace_amd.localkube import LocalCluster

    cluster = LocalCluster(str(tmp_path / "state"), gpus=0).start()
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        proj = lk.project("rocm-pytorch")  # unschedulable here: the rollout wait lasts 5 s
        p = subprocess.Popen([lk.bin, "deploy"], cwd=proj, env=lk.env, stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, text=True)
        deadline = time.time() + 60
        while time.time() < deadline and not cluster.store.list("apps", "deployments", "rocm-pytorch"):
            time.sleep(0.02)
        time.sleep(0.3)
        assert p.poll() is None
        t0 = time.time()
        p.send_signal(signal.SIGINT)
        out, _ = p.communicate(timeout=20)
        assert p.returncode == 130, out
        assert time.time() - t0 < 2, out
    finally:
        cluster.stop()


def test_rocm_pytorch_example_runs_from_a_clean_clone(tmp_path):
    """the example's workload kit (devspace_amd/) is written by the checkout's build
    and git-ignored, so a clean clone has none. `devspace deploy` adds the kit it ships to the
    build context (with a notice) and the pod starts the runner — built from `git ls-files` only."""
    import os
    import shutil

    from conftest import ROOT
    from devspace_amd.localkube import LocalCluster

    files = subprocess.run(["git", "ls-files", "examples/rocm-pytorch"], cwd=ROOT, capture_output=True, text=True,
                           check=True).stdout.split()
    assert files and not [f for f in files if "/devspace_amd/" in f]
    proj = tmp_path / "clone" / "rocm-pytorch"
    for f in files:
        dst = proj / os.path.relpath(f, "examples/rocm-pytorch")
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy2(os.path.join(ROOT, f), dst)
    cluster = LocalCluster(str(tmp_path / "state"), gpus=1).start()
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        r = lk.run(["deploy"], str(proj), timeout=300, check=False)
        out = r.stdout + r.stderr
        assert r.returncode == 0, out
        assert "has no devspace_amd/" in out, out
        assert not (proj / "devspace_amd").exists()  # the project tree is left alone
        pods = cluster.wait_pods_running("rocm-pytorch", timeout=120)
        import json

        root = next(iter(json.loads(pods[0]["metadata"]["annotations"]["devspace.sh/local-roots"]).values()))
        assert os.path.exists(os.path.join(root, "app", "devspace_amd", "runner.py"))
        deadline = time.time() + 240
        log = ""
        while time.time() < deadline:
            log = open(root + ".log").read() if os.path.exists(root + ".log") else ""
            if "[devspace-runner] started gen=1" in log or "Traceback" in log:
                break
            time.sleep(0.5)
        assert "[devspace-runner] started gen=1" in log, log[-3000:]
    finally:
        cluster.stop()


def test_analyze_reports_a_training_group_that_is_down(tmp_path):
    """A rank of the pod's training group fails on a bad edit: the runner stops the group and
    waits for the next edit, the pod stays Running, and `devspace analyze` says why the GPUs are
    idle (the failing rank and its exception) instead of "No problems found"."""
    import os
    import re

    from devspace_amd.localkube import LocalCluster

    cluster = LocalCluster(str(tmp_path / "state"), gpus=2).start()
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        proj = lk.project("rocm-pytorch")
        train = os.path.join(proj, "train.py")
        src = open(train).read()
        for k, v in (("VOCAB", 128), ("DIM", 64), ("HEADS", 4), ("LAYERS", 1), ("SEQ", 16), ("BATCH", 2)):
            src = re.sub(rf"^{k} = \d+$", f"{k} = {v}", src, flags=re.M)
        src = src.replace("def step(ctx, state):\n",
                          "def step(ctx, state):\n    if ctx.rank == 1:\n"
                          "        raise ValueError('shapes (4,8) and (9,8) not aligned')\n", 1)
        open(train, "w").write(src)
        values = os.path.join(proj, "chart", "values.yaml")
        v = open(values).read()
        open(values, "w").write(re.sub(r"gpu: \d+", "gpu: 2", v))  # two ranks
        r = lk.run(["deploy"], proj, timeout=300, check=False)
        assert r.returncode == 0, r.stdout + r.stderr
        pods = cluster.wait_pods_running("rocm-pytorch", timeout=120)
        import json

        root = next(iter(json.loads(pods[0]["metadata"]["annotations"]["devspace.sh/local-roots"]).values()))
        deadline = time.time() + 180
        log = ""
        while time.time() < deadline and "waiting for a file change" not in log:
            log = open(root + ".log").read() if os.path.exists(root + ".log") else ""
            time.sleep(0.5)
        assert "waiting for a file change" in log, log[-3000:]
        out = lk.run(["analyze", "--wait=false"], proj, timeout=120, check=False).stdout
        assert "training group is down after rank=1" in out, out
        assert "ValueError: shapes (4,8) and (9,8) not aligned" in out, out
    finally:
        cluster.stop()


def test_unschedulable_while_the_autoscaler_adds_a_gpu_node_is_waited_out(tmp_path):
    """GPU node pools often scale from zero. A pod that is Unschedulable while the
    cluster autoscaler says it triggered a scale-up is waited for (up to the rollout timeout),
    not failed at the first look; the deploy succeeds once the node's GPUs appear."""
    from devspace_amd.localkube import LocalCluster

    cluster = LocalCluster(str(tmp_path / "state"), gpus=0).start()
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        proj = lk.project("rocm-pytorch")
        lk.env["DEVSPACE_UNSCHEDULABLE_GRACE_S"] = "1"

        def autoscaler():
            deadline = time.time() + 60
            pods = []
            while time.time() < deadline and not pods:
                pods = cluster.store.list("", "pods", "rocm-pytorch")
                time.sleep(0.05)
            if not pods:
                return
            md = pods[0]["metadata"]
            cluster.store.create("", "events", "rocm-pytorch", {
                "metadata": {"name": md["name"] + ".scaleup", "namespace": "rocm-pytorch"},
                "involvedObject": {"kind": "Pod", "name": md["name"], "namespace": "rocm-pytorch", "uid": md["uid"]},
                "reason": "TriggeredScaleUp", "type": "Normal", "count": 1,
                "message": "pod triggered scale-up: [{mi355x-pool 0->1 (max: 4)}]",
                "source": {"component": "cluster-autoscaler"}}, "v1")
            time.sleep(4.0)  # the node boots
            cluster.kubelet.add_gpus(1)

        t = threading.Thread(target=autoscaler, daemon=True)
        t.start()
        t0 = time.time()
        r = lk.run(["deploy"], proj, timeout=120, check=False)
        took = time.time() - t0
        out = r.stdout + r.stderr
        assert r.returncode == 0, out
        assert took >= 4.0, (took, out)
        assert "the cluster autoscaler is adding a node" in out, out
    finally:
        cluster.stop()
