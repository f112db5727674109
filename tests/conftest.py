import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.hookimpl(tryfirst=True)
def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")
    # every `devspace` this test run starts ends with it, even when pytest itself is killed (a
    # timeout's os._exit, SIGKILL): the CLI ties itself to this pid (PR_SET_PDEATHSIG,
    # src/platform/linux.cc tie_to_parent) when it is its parent
    os.environ["DEVSPACE_PARENT_PID"] = str(os.getpid())
    # a hung test ends the run with every thread's stack (pytest-timeout) instead of stalling it:
    # the longest test takes about 5 minutes; an explicit --timeout wins
    if getattr(config.option, "timeout", None) is None and config.pluginmanager.hasplugin("timeout"):
        config.option.timeout = 1800
        config.option.timeout_method = "thread"


@pytest.fixture(scope="session", autouse=True)
def native_build():
    """Build the native tree once per session if the in-tree artefacts are missing."""
    from devspace_amd import buildtools

    buildtools.ensure_built()
    return ROOT


@pytest.fixture
def devspace_bin():
    return os.path.join(ROOT, "bin", "devspace")


class DevspaceEnv:
    """A running local cluster plus an isolated HOME/KUBECONFIG for `devspace` invocations."""

    def __init__(self, cluster, base):
        import subprocess  # noqa: F401

        self.cluster = cluster
        self.base = base
        self.home = os.path.join(base, "home")
        os.makedirs(self.home, exist_ok=True)
        self.kubeconfig = cluster.write_kubeconfig(os.path.join(self.home, ".kube", "config"))
        self.env = dict(os.environ)
        self.env.update(cluster.env(self.kubeconfig))
        self.env.update(HOME=self.home, DEVSPACE_NONINTERACTIVE="1", PYTHONPATH=ROOT)
        # DEVSPACE_BIN: run the e2e suite against another build (e.g. build/asan/bin/devspace)
        self.bin = os.environ.get("DEVSPACE_BIN") or os.path.join(ROOT, "bin", "devspace")

    def run(self, args, cwd, input=None, timeout=120, check=True):
        import subprocess

        env = self.env
        if input is not None:
            # answers scripted over the pipe: DEVSPACE_NONINTERACTIVE=1 never reads stdin
            env = {k: v for k, v in self.env.items() if k != "DEVSPACE_NONINTERACTIVE"}
        p = subprocess.run([self.bin] + list(args), cwd=cwd, env=env, input=input, capture_output=True,
                           text=True, timeout=timeout)
        if check and p.returncode != 0:
            raise AssertionError(f"devspace {' '.join(args)} failed rc={p.returncode}\n{p.stdout}\n{p.stderr}")
        return p

    def popen(self, args, cwd, env=None):
        import subprocess

        return subprocess.Popen([self.bin] + list(args), cwd=cwd, env=dict(self.env, **(env or {})),
                                stdout=subprocess.PIPE,
                                stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, text=True,
                                start_new_session=True)

    def pods(self, namespace, selector=""):
        return self.cluster.store.list("", "pods", namespace, selector)

    def project(self, example, dst_name=None):
        import shutil

        dst = os.path.join(self.base, dst_name or example)
        if os.path.exists(dst):
            shutil.rmtree(dst)
        shutil.copytree(os.path.join(ROOT, "examples", example), dst, symlinks=True)
        return dst


@pytest.fixture(scope="module")
def localkube(tmp_path_factory):
    from devspace_amd.localkube import LocalCluster

    base = str(tmp_path_factory.mktemp("lk"))
    cluster = LocalCluster(os.path.join(base, "state"), gpus=int(os.environ.get("LK_GPUS", "0"))).start()
    try:
        yield DevspaceEnv(cluster, base)
    finally:
        cluster.stop()
