"""Hot-reload runner (workload side): code swap without losing state."""
import os
import re
import subprocess
import sys
import time

import pytest

from conftest import ROOT

TRAIN = os.path.join(ROOT, "examples", "rocm-pytorch", "train.py")


def _tiny_copy(tmp_path):
    src = open(TRAIN).read()
    for k, v in (("VOCAB", 128), ("DIM", 64), ("HEADS", 4), ("LAYERS", 1), ("SEQ", 16), ("BATCH", 2)):
        src = re.sub(rf"^{k} = \d+$", f"{k} = {v}", src, flags=re.M)
    p = tmp_path / "train.py"
    p.write_text(src)
    return p


def _run_reload(tmp_path, extra_env=None, nproc=1):
    p = _tiny_copy(tmp_path)
    env = dict(os.environ, PYTHONPATH=ROOT, **(extra_env or {}))
    proc = subprocess.Popen([sys.executable, "-u", "-m", "devspace_amd.runner", "--nproc", str(nproc), "--watch",
                             str(tmp_path), str(p)],
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True)
    lines = []
    try:
        t0 = time.time()
        while time.time() - t0 < 180:
            line = proc.stdout.readline()
            lines.append(line)
            if "started gen=1" in line:
                break
        assert any("started gen=1" in l for l in lines), "".join(lines)
        p.write_text(p.read_text().replace('MARKER = "v0"', 'MARKER = "edited"'))
        t0 = time.time()
        while time.time() - t0 < 60:
            line = proc.stdout.readline()
            lines.append(line)
            if "marker=edited" in line:
                break
        reload_line = [l for l in lines if "marker=edited" in l]
        assert reload_line, "".join(lines[-20:])
        # a broken edit keeps the previous version running
        p.write_text(p.read_text() + "\nthis is not python\n")
        t0 = time.time()
        while time.time() - t0 < 60:
            line = proc.stdout.readline()
            lines.append(line)
            if "reload failed" in line:
                break
        assert any("reload failed" in l for l in lines)
        assert proc.poll() is None
        return reload_line[0] + "".join(l for l in lines if "started gen=1" in l)
    finally:
        proc.terminate()
        proc.wait(10)


def test_runner_hot_reload_cpu(tmp_path):
    line = _run_reload(tmp_path, {"HIP_VISIBLE_DEVICES": "-1", "CUDA_VISIBLE_DEVICES": "-1"})
    assert "gen=2" in line


def test_runner_hot_reload_two_ranks_cpu(tmp_path):
    """The N>1 path of the pod (one process per GPU, DDP, generation agreement by all-reduce),
    rehearsed with two gloo ranks on the CPU."""
    line = _run_reload(tmp_path, {"HIP_VISIBLE_DEVICES": "-1", "CUDA_VISIBLE_DEVICES": "-1"}, nproc=2)
    assert "gen=2" in line and "world=2" in line


@pytest.mark.gpu
def test_runner_hot_reload_gpu(tmp_path):
    line = _run_reload(tmp_path)
    assert "gen=2" in line
