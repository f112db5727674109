"""GPU scheduling failures and interrupts through the real CLI on a GPU-less local cluster (CPU).

A chart requesting amd.com/gpu that no node can satisfy is reported at once (analyze report
with the FailedScheduling event, repeated scheduler attempts aggregated into one event), not
waited out for the rollout timeout; Ctrl-C ends a one-shot command right away."""

import signal
import subprocess
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
