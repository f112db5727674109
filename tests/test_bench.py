"""bench.py contract: one JSON line with the driver's fields."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(args, timeout):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = r.stdout.strip().splitlines()[-1]
    return json.loads(line)


def test_bench_cpu_tiny():
    """The full contract on CPU: the headline is the quickstart loop (BASELINE configs[0], the
    metric's named config) with its same-box reference-equivalent column; extras cover the
    deploy (both columns), the GPU-pod loop and BASELINE configs[1-3] (both columns)."""
    # three reference samples: one compat-protocol sample can ride on a batch window an echo of
    # the previous upload opened (it then lands early), which a single sample cannot outvote
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--ref-steps",
                        "3", "--gpu-steps", "2", "--example-steps", "2", "--tiny"], capture_output=True, text=True,
                       timeout=1200, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    # every failed extra, with its message, in any assertion below that fails
    errs = d.get("extra_errors", {})
    assert "reference_equivalent" in d and "wan" in d and "deploy" in d, (errs, r.stderr[-3000:])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["metric"].endswith("quickstart") and d["higher_is_better"] is False
    assert d["value"] > 0 and d["steps"] == 3 and d["value"] == d["p50_ms"]
    cfg = d["config"]
    assert cfg["app"] == "examples/quickstart"
    assert cfg["transport"].startswith("https + wss") and "RUN steps not executed" in cfg["builder"]
    # same-box reference column of the headline (compat protocol + reference waits)
    assert d["reference_equivalent"]["p50_ms"] > d["value"], r.stderr[-3000:]
    assert d["reference_equivalent"]["sync_p50_ms"] > d["sync_p50_ms"]
    assert 0 < d["dev_start_s"] < d["reference_equivalent"]["dev_start_s"], (d["dev_start_s"], d["reference_equivalent"])
    # the headline is the tool's own loop: cold restarts (nodemon), not the example's standby pool
    assert cfg["restart"] == "cold" and "WATCH_STANDBY=0" in cfg["sample"] and d["dtype"] is None
    pool = d["standby_pool"]
    assert pool["n"] >= 10 and pool["p50_ms"] > 0 and "app-side" in pool["what"], pool
    # the same loops behind a 30 ms RTT link: every edit pays at least the one-way delay
    wan = d["wan"]
    assert wan["rtt_ms"] == 30 and wan["n"] >= 5 and wan["link_connections"] > 0, wan
    # each edit's GET reached the restarted app once (no hedged duplicates by default)
    assert wan["app_requests_per_edit"] == 1.0 and d["app_requests_per_edit"] == 1.0, (wan, errs)
    assert wan["sync_p50_ms"] >= 15 and wan["p50_ms"] > wan["sync_p50_ms"], wan
    assert wan["reference_equivalent"]["p50_ms"] > wan["p50_ms"], wan
    # deploy across the link: kept-alive connections vs a dial (+ TLS) per request
    wd = wan["deploy"]
    assert wd["net"]["tcp_dials"] < wd["reference_equivalent"]["net"]["tcp_dials"], wd
    assert wd["reference_equivalent"]["wall_clock_s"] > wd["wall_clock_s"], wd
    dep = d["deploy"]
    # the image build ran the Dockerfile's RUN (npm install); an edit rebuilt from the layer cache
    assert dep["control_plane_only"] is False and dep["run_steps_executed"] is True, dep
    assert dep["net"]["tls_handshakes"] >= 1 and dep["phases_ms"]["image.build"] > 100, dep
    assert dep["edit_redeploy_s"] < dep["wall_clock_s"], dep
    # reference timing: no kept-alive connections, 5 s rollout polls
    assert dep["reference_equivalent"]["wall_clock_s"] > dep["wall_clock_s"], dep
    # the reference's rollout wait polls every 5 s, the first check after one interval
    assert dep["reference_equivalent"]["wall_clock_s"] >= 4.5, dep
    assert dep["reference_equivalent"]["net"]["reused"] == 0, dep
    g = d["gpu_pod"]
    assert g["n"] == 2 and g["reload_p50_ms"] > 0 and g["fused_ops"].startswith("eager (no GPU)"), g
    assert g["reference_equivalent"]["p50_ms"] > g["reload_p50_ms"]
    # the same GPU-pod loop with the cluster 30 ms away: the edit crosses the link one way
    gw = g["wan"]
    assert "error" not in gw and gw["n"] == 10 and gw["sync_p50_ms"] >= 15, gw
    assert gw["reload_p50_ms"] > gw["sync_p50_ms"], gw
    # one rank: the drill's hard crash is replaced from the warm standby, resuming from a snapshot
    drill = g["fault_drill"]
    assert drill.get("recovered") is True and drill["ranks"] == 1 and drill["warm_standby"], drill
    assert drill["resumed_from_step"], drill
    for key in ("php_mysql", "microservices", "kaniko"):
        e = d[key]
        assert "error" not in e, (key, e, r.stderr[-3000:])
        assert e["n"] == 2 and e["edit_to_pod_p50_ms"] > 0 and e["deploy_cold_s"] > 0, (key, e)
        assert e["reference_equivalent"]["edit_to_pod_p50_ms"] > e["edit_to_pod_p50_ms"], (key, e)
    assert d["microservices"]["sync_paths"] == 2 and d["microservices"]["port_forwards"] == 2


def test_bench_torchrun_two_ranks_cpu():
    """The driver's N>1 launch shape (torchrun, one rank per GPU) on CPU with gloo: rank 0
    drives the CLI, rank 1 joins the timing barriers; exactly one JSON line, and the GPU-pod
    extra ran one training rank per bench rank."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29655", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--tiny", "--ref-steps", "0", "--gpu-steps", "2", "--example-steps", "0",
           "--no-deploy-bench"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["steps"] == 2 and d["value"] > 0
    assert d["n_gpus"] == 2 and d["gpu_pod"]["parallelism"] == "dp2", d
    assert d["gpu_pod"]["ranks"] == 2 and d["gpu_pod"]["ranks_agreed_on_code"] is True, d["gpu_pod"]
    # the 2-rank pod's failure path: rank 1 raises once, the group is replaced and trains again
    drill = d["gpu_pod"]["fault_drill"]
    assert drill.get("recovered") is True, drill
    assert drill["failure_to_training_s"] < 60, drill


@pytest.mark.slow
def test_bench_torchrun_eight_ranks_cpu():
    """the driver's 8-GPU launch (torchrun, 8 bench ranks) rehearsed on CPU with
    gloo: the GPU pod starts 8 runner ranks, every reload is confirmed by all 8 (one code digest,
    `ranks=8` in the runner's line), and the run stays within the extras budget."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", "29657", os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "2",
           "--warmup", "1", "--tiny", "--ref-steps", "0", "--gpu-steps", "3", "--example-steps", "0",
           "--no-deploy-bench", "--extras-budget-s", "400"]
    env = dict(os.environ, DEVSPACE_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["steps"] == 2 and d["value"] > 0
    g = d.get("gpu_pod")
    assert isinstance(g, dict) and "error" not in g, (g, r.stderr[-3000:])
    assert g["parallelism"] == "dp8" and g["ranks"] == 8 and g["ranks_agreed_on_code"] is True, g
    assert g["n"] == 3 and g["reload_p50_ms"] > 0, g
    assert g["fault_drill"].get("recovered") is True, g["fault_drill"]  # 8 ranks: fail, replace, resume


def test_bench_extras_budget_keeps_the_headline():
    """A hung extra (here: no time left at all) ends that extra, not the run: the headline line
    is still printed, and the extras that could not finish are left out."""
    d = _run(["--steps", "2", "--warmup", "1", "--ref-steps", "1", "--gpu-steps", "2", "--example-steps", "0",
              "--no-deploy-bench", "--tiny", "--extras-budget-s", "0.001"], 600)
    assert d["value"] > 0 and d["steps"] == 2
    assert "gpu_pod" not in d and "cold_restart" not in d and "reference_equivalent" not in d, d


def test_a_failed_extra_is_named_with_its_message():
    """An extra that raises is reported in `extra_errors` with its message (it used to vanish and
    surface later as a KeyError in the caller's assertions)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--ref-steps",
                        "0", "--gpu-steps", "0", "--example-steps", "0", "--tiny"], capture_output=True, text=True,
                       timeout=600, cwd=ROOT, env=dict(os.environ, DEVSPACE_BENCH_FAIL_EXTRA="deploy"))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["value"] > 0 and "deploy" not in d, d
    assert "forced failure of deploy" in d["extra_errors"]["deploy"], d.get("extra_errors")


@pytest.mark.gpu
def test_bench_gpu_short():
    d = _run(["--steps", "3", "--warmup", "1", "--ref-steps", "1"], 900)
    assert d["n_gpus"] >= 1 and d["value"] > 0
