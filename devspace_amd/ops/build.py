"""Compile the HIP sources in this directory for gfx950 (in-tree .so files that travel with the repo).

* gpuprobe.hip  -> libgpuprobe.so           C ABI, loaded with ctypes by devspace_amd.gpucheck
* fused_ops.hip -> _fused_ops<EXT_SUFFIX>   PyTorch extension (ATen + pybind11), compiled directly
                                            with hipcc against the installed torch headers/libs
"""

import os
import shutil
import subprocess
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise FileNotFoundError("hipcc not found")


def lib_path(name="gpuprobe"):
    return os.path.join(HERE, f"lib{name}.so")


def fused_path():
    return os.path.join(HERE, "_fused_ops" + sysconfig.get_config_var("EXT_SUFFIX"))


def _stale(out, *srcs):
    return not os.path.exists(out) or any(os.path.getmtime(out) < os.path.getmtime(s) for s in srcs)


def _run(cmd, verbose):
    if verbose:
        print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build_probe(verbose=False, force=False):
    src = os.path.join(HERE, "gpuprobe.hip")
    out = lib_path()
    if force or _stale(out, src):
        _run([hipcc(), "-O3", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wno-unused-value", "-o", out, src],
             verbose)
    return out


def source_sha(path=None) -> str:
    """SHA-256 of the fused-ops source, compiled into the extension (`_fused_ops.source_sha`)."""
    import hashlib

    with open(path or os.path.join(HERE, "fused_ops.hip"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _fused_tag():
    """Cache key of a fused-ops build: source bytes, torch build, target arch, Python ABI."""
    import hashlib

    import torch

    h = hashlib.sha256(open(os.path.join(HERE, "fused_ops.hip"), "rb").read())
    h.update(f"{torch.__version__}|{torch.version.hip}|{ARCH}|{sysconfig.get_config_var('EXT_SUFFIX')}".encode())
    return h.hexdigest()[:16]


def fused_cache_path():
    """Where a vendored copy (a project made by `devspace init`, running in its pod) keeps the
    extension it compiled: $DEVSPACE_OPS_CACHE or ~/.cache/devspace_amd, keyed by _fused_tag()."""
    base = os.environ.get("DEVSPACE_OPS_CACHE") or os.path.join(os.path.expanduser("~"), ".cache", "devspace_amd")
    return os.path.join(base, "fused-" + _fused_tag(), "_fused_ops" + sysconfig.get_config_var("EXT_SUFFIX"))


def ensure_fused_cached(verbose=True):
    """Compiles the extension into the cache unless it is there (minutes: done at image build by
    the rocm-pytorch Dockerfile, else once on the first pod start). Returns its path."""
    out = fused_cache_path()
    if not os.path.exists(out):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        tmp = out + f".tmp{os.getpid()}"
        if verbose:
            print(f"[devspace_amd] compiling the fused gfx950 ops ({ARCH}) into {out} ...", flush=True)
        build_fused(verbose=False, force=True, out=tmp)
        os.replace(tmp, out)  # concurrent ranks: whoever finishes first wins, the rest overwrite
    return out


def build_fused(verbose=False, force=False, out=None):
    import torch  # headers + libraries of the torch this extension is loaded into

    src = os.path.join(HERE, "fused_ops.hip")
    out = out or fused_path()
    if not (force or _stale(out, src)):
        return out
    troot = os.path.dirname(torch.__file__)
    tlib = os.path.join(troot, "lib")
    cxx11 = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [hipcc(), "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared",
           "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_fused_ops", "-DTORCH_API_INCLUDE_EXTENSION_H",
           f'-DDEVSPACE_SOURCE_SHA="{source_sha(src)}"',
           f"-D_GLIBCXX_USE_CXX11_ABI={cxx11}", "-Wno-unused-result",
           "-I" + os.path.join(troot, "include"), "-I" + os.path.join(troot, "include", "torch", "csrc", "api", "include"),
           "-I" + sysconfig.get_paths()["include"], src,
           "-L" + tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
           "-Wl,-rpath," + tlib, "-o", out]
    _run(cmd, verbose)
    return out


def build(verbose=False, force=False):
    out = build_probe(verbose=verbose, force=force)
    build_fused(verbose=verbose, force=force)
    return out


def main(argv=None):
    import argparse

    p = argparse.ArgumentParser(prog="devspace_amd.ops.build", description=__doc__.split("\n")[0])
    p.add_argument("--fused", action="store_true", help="the fused training ops")
    p.add_argument("--probe", action="store_true", help="the GPU probe library")
    p.add_argument("--cache", action="store_true",
                   help="build the fused ops into the cache (image build of a vendored copy) instead of in place")
    a = p.parse_args(argv)
    if a.probe:
        print(build_probe(verbose=True))
    if a.fused:
        print(ensure_fused_cached() if a.cache else build_fused(verbose=True))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
