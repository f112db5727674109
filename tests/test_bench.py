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
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--ref-steps",
                        "1", "--qs-steps", "3", "--tiny"], capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    # the extras are best-effort inside bench.py (logged, not fatal): show why one is missing
    assert "quickstart" in d and "tool_attributable" in d, r.stderr[-3000:]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "config"):
        assert k in d
    assert d["higher_is_better"] is False
    assert d["value"] > 0
    # the config names what was measured: app, transport, builder fidelity
    assert d["config"]["app"] == "examples/rocm-pytorch"
    assert d["config"]["transport"].startswith("https + wss")
    assert "RUN steps not executed" in d["config"]["builder"]
    assert d["deploy"]["control_plane_only"] is True
    assert d["deploy"]["net"]["tls_handshakes"] >= 1
    assert d["reference_equivalent"]["p50_ms"] > d["value"]
    # Node.js quickstart loop through sync + port-forward, and the sync-protocol comparison
    assert d["quickstart"]["n"] == 3 and d["quickstart"]["reload_p50_ms"] > d["quickstart"]["sync_p50_ms"] > 0
    assert d["tool_attributable"]["reference_protocol_sync_p50_ms"] > d["tool_attributable"]["sync_p50_ms"]


def test_bench_torchrun_two_ranks_cpu():
    """The driver's N>1 launch shape (torchrun, one rank per GPU) on CPU with gloo: rank 0
    drives the dev loop, rank 1 joins the timing barriers; exactly one JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29655", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--tiny", "--ref-steps", "0", "--qs-steps", "0", "--no-deploy-bench"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["steps"] == 2 and d["value"] > 0
    # the pod ran one training rank per bench rank (the runner's N-rank generation agreement)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"


@pytest.mark.gpu
def test_bench_gpu_short():
    d = _run(["--steps", "3", "--warmup", "1", "--ref-steps", "1"], 900)
    assert d["n_gpus"] >= 1 and d["value"] > 0
