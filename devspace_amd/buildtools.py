"""Build helpers: configure + compile the native tree in-place (bin/ and devspace_amd/*.so)."""

from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD_DIR = os.path.join(ROOT, "build")


def _run(cmd, verbose):
    if verbose:
        print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=ROOT, stdout=None if verbose else subprocess.DEVNULL)


def native_ready() -> bool:
    return (
        os.path.exists(os.path.join(ROOT, "bin", "devspace"))
        and os.path.exists(os.path.join(ROOT, "bin", "devspace-helper"))
        and bool(glob.glob(os.path.join(ROOT, "devspace_amd", "_native*.so")))
    )


def build_cpp(verbose=False, jobs=None):
    jobs = jobs or min(16, os.cpu_count() or 4)
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    _run(["cmake", "-S", ROOT, "-B", BUILD_DIR, "-DCMAKE_BUILD_TYPE=RelWithDebInfo",
          f"-DPython3_EXECUTABLE={sys.executable}"] + gen, verbose)
    _run(["cmake", "--build", BUILD_DIR, "-j", str(jobs)], verbose)


def build_hip(verbose=False):
    """gfx950 GPU probe library (devspace_amd/ops/gpuprobe.hip)."""
    from devspace_amd.ops import build as ops_build

    return ops_build.build(verbose=verbose)


def write_example_kit(verbose=False):
    """examples/rocm-pytorch carries the workload kit like a `devspace init`'d project does
    (devspace_amd/kit.py; not tracked in git), with the in-tree gfx950 build in place of the
    image build's cached one."""
    from devspace_amd import kit

    written = kit.write_kit(os.path.join(ROOT, "examples", "rocm-pytorch"), prebuilt=True)
    if verbose and written:
        print("+ workload kit -> examples/rocm-pytorch/devspace_amd: " + ", ".join(written), flush=True)


def build_all(verbose=False):
    build_cpp(verbose=verbose)
    try:
        build_hip(verbose=verbose)
    except FileNotFoundError as e:  # hipcc missing: CPU-only environments still get the tool
        print(f"skipping HIP build: {e}", flush=True)
    write_example_kit(verbose=verbose)


def ensure_built():
    if not native_ready():
        build_cpp(verbose=False)
    write_example_kit()
