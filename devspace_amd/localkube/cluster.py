"""Local single-node cluster: API server + process kubelet + Docker-API builder + registry.

This is the "local-pod backend" of SURVEY.md §7.4: the GPU box has no Kubernetes, Docker or
network, so `devspace deploy/dev/enter/logs/analyze` run against this cluster through the
exact same wire protocols they use against a real MI355X node (REST, WebSocket exec/attach/
port-forward, Docker Engine API over a unix socket). The node advertises `amd.com/gpu`
capacity equal to the visible GPUs (KFD topology), like the AMD GPU device plugin.

    python -m devspace_amd.localkube up --state /tmp/lk [--gpus N] [--kubeconfig PATH]
"""

from __future__ import annotations

import asyncio
import glob
import os
import socket
import threading
import time

from aiohttp import web

from .apiserver import ApiServer
from .dockerd import ImageStore, make_app
from .kubelet import Kubelet
from .store import Store

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def detect_gpus():
    """Counts GPU agents in the KFD topology (CPU nodes report simd_count 0)."""
    n = 0
    for props in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(props) as f:
                kv = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            if int(kv.get("simd_count", "0")) > 0:
                n += 1
        except (OSError, ValueError):
            continue
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        ids = [v for v in vis.split(",") if v.strip() and v.strip() != "-1"]
        n = min(n, len(ids)) if n else 0
    return n


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class LocalCluster:
    def __init__(self, state_dir, port=0, gpus=None, context="devspace-local", extra_env=None):
        self.state_dir = os.path.abspath(state_dir)
        os.makedirs(self.state_dir, exist_ok=True)
        self.port = port or free_port()
        self.gpus = detect_gpus() if gpus is None else gpus
        self.context = context
        self.store = Store()
        self.images = ImageStore(os.path.join(self.state_dir, "docker"))
        env = {"PYTHONPATH": ROOT + os.pathsep + os.environ.get("PYTHONPATH", "")}
        env.update(extra_env or {})
        self.kubelet = Kubelet(self.store, self.images, self.state_dir, gpus=self.gpus, extra_env=env)
        self.api = ApiServer(self.store, self.kubelet)
        self.docker_sock = os.path.join(self.state_dir, "docker.sock")
        self.loop = None
        self.thread = None
        self._runners = []
        self._ready = threading.Event()
        self._kubelet_task = None

    @property
    def server(self):
        return f"http://127.0.0.1:{self.port}"

    def kubeconfig_yaml(self, namespace="default"):
        return (
            "apiVersion: v1\nkind: Config\n"
            f"current-context: {self.context}\n"
            "clusters:\n"
            f"- name: {self.context}\n  cluster:\n    server: {self.server}\n"
            "contexts:\n"
            f"- name: {self.context}\n  context:\n    cluster: {self.context}\n    user: {self.context}\n"
            f"    namespace: {namespace}\n"
            "users:\n"
            f"- name: {self.context}\n  user:\n    token: devspace-local-token\n"
            "preferences: {}\n"
        )

    def write_kubeconfig(self, path, namespace="default"):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            f.write(self.kubeconfig_yaml(namespace))
        return path

    def env(self, kubeconfig_path):
        """Environment for devspace processes targeting this cluster."""
        return {"KUBECONFIG": kubeconfig_path, "DOCKER_HOST": f"unix://{self.docker_sock}"}

    async def _amain(self):
        api_runner = web.AppRunner(self.api.app(), access_log=None)
        await api_runner.setup()
        await web.TCPSite(api_runner, "127.0.0.1", self.port).start()
        if os.path.exists(self.docker_sock):
            os.unlink(self.docker_sock)
        d_runner = web.AppRunner(make_app(self.images), access_log=None)
        await d_runner.setup()
        await web.UnixSite(d_runner, self.docker_sock).start()
        self._runners = [api_runner, d_runner]
        self._kubelet_task = asyncio.create_task(self.kubelet.run())
        try:
            self.store.create("", "namespaces", "", {"metadata": {"name": "default"}}, "v1")
        except Exception:
            pass
        self._ready.set()

    def start(self):
        def run():
            self.loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self.loop)
            self.loop.run_until_complete(self._amain())
            self.loop.run_forever()

        self.thread = threading.Thread(target=run, daemon=True, name="localkube")
        self.thread.start()
        if not self._ready.wait(30):
            raise RuntimeError("local cluster failed to start")
        return self

    def stop(self):
        if not self.loop:
            return

        async def shutdown():
            await self.kubelet.shutdown()
            if self._kubelet_task:
                self._kubelet_task.cancel()
            for r in self._runners:
                await r.cleanup()

        fut = asyncio.run_coroutine_threadsafe(shutdown(), self.loop)
        try:
            fut.result(30)
        finally:
            self.loop.call_soon_threadsafe(self.loop.stop)
            self.thread.join(10)
            self.loop = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def wait_pods_running(self, namespace, selector="", timeout=120):
        t0 = time.time()
        while time.time() - t0 < timeout:
            pods = self.store.list("", "pods", namespace, selector)
            if pods and all((p.get("status") or {}).get("phase") == "Running" for p in pods):
                return pods
            time.sleep(0.05)
        raise TimeoutError(f"pods {selector} not running in {namespace}")
