"""Compile the HIP sources in this directory for gfx950 (in-tree .so, travels with the repo)."""

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise FileNotFoundError("hipcc not found")


def lib_path(name="gpuprobe"):
    return os.path.join(HERE, f"lib{name}.so")


def build(verbose=False, force=False):
    src = os.path.join(HERE, "gpuprobe.hip")
    out = lib_path()
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    cmd = [hipcc(), "-O3", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wno-unused-value", "-o", out, src]
    if verbose:
        print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return out
