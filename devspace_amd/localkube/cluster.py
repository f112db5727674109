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
import base64
import glob
import os
import socket
import ssl
import subprocess
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


def make_pki(d):
    """Self-signed CA + server cert (127.0.0.1/localhost) + client cert, via the openssl CLI."""
    os.makedirs(d, exist_ok=True)

    def ossl(*args):
        subprocess.run(["openssl"] + list(args), check=True, capture_output=True)

    ossl("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "2", "-subj", "/CN=devspace-local-ca",
         "-keyout", f"{d}/ca.key", "-out", f"{d}/ca.crt")
    ext = f"{d}/san.ext"
    with open(ext, "w") as f:
        f.write("subjectAltName=IP:127.0.0.1,DNS:localhost\n")
    for name, subj, extra in (("server", "/CN=127.0.0.1", ["-extfile", ext]),
                              ("client", "/CN=devspace-user/O=system:masters", [])):
        ossl("req", "-newkey", "rsa:2048", "-nodes", "-subj", subj, "-keyout", f"{d}/{name}.key",
             "-out", f"{d}/{name}.csr")
        ossl("x509", "-req", "-in", f"{d}/{name}.csr", "-CA", f"{d}/ca.crt", "-CAkey", f"{d}/ca.key",
             "-CAcreateserial", "-days", "2", "-out", f"{d}/{name}.crt", *extra)
    return d


def _b64file(path):
    with open(path, "rb") as f:
        return base64.b64encode(f.read()).decode()


class LocalCluster:
    def __init__(self, state_dir, port=0, gpus=None, context="devspace-local", extra_env=None, tls=False,
                 token_validator=None, gpu_partition="spx", memory_partition="nps1", gpu_strategy="single",
                 unhealthy_gpus=0, run_steps=False, portforward_tunnel=True):
        self.state_dir = os.path.abspath(state_dir)
        self.tls = tls
        self.pki = make_pki(os.path.join(self.state_dir, "pki")) if tls else None
        os.makedirs(self.state_dir, exist_ok=True)
        self.port = port or free_port()
        self.gpus = detect_gpus() if gpus is None else gpus
        self.context = context
        self.store = Store()
        self.images = ImageStore(os.path.join(self.state_dir, "docker"))
        self.images.run_steps = run_steps  # the image builder executes RUN (host runtime)
        env = {"PYTHONPATH": ROOT + os.pathsep + os.environ.get("PYTHONPATH", "")}
        env.update(extra_env or {})
        self.kubelet = Kubelet(self.store, self.images, self.state_dir, gpus=self.gpus, extra_env=env)
        # SPX/DPX/QPX/CPX compute partitions, NPS memory mode, single/mixed resource naming and
        # devices the device plugin marked unhealthy, as an MI355X node would advertise them
        self.kubelet.set_gpu_topology(gpu_partition, memory_partition, gpu_strategy, unhealthy_gpus)
        self.api = ApiServer(self.store, self.kubelet, token_validator=token_validator)
        # False: an API server older than Kubernetes 1.30 (no SPDY-over-WebSocket port-forward)
        self.api.portforward_tunnel = portforward_tunnel
        self.docker_sock = os.path.join(self.state_dir, "docker.sock")
        self.loop = None
        self.thread = None
        self._runners = []
        self._ready = threading.Event()
        self._kubelet_task = None

    @property
    def server(self):
        return f"{'https' if self.tls else 'http'}://127.0.0.1:{self.port}"

    def kubeconfig_yaml(self, namespace="default"):
        cluster = f"    server: {self.server}\n"
        user = "    token: devspace-local-token\n"
        if self.tls:  # verify the server against our CA and authenticate with a client cert
            cluster += f"    certificate-authority-data: {_b64file(os.path.join(self.pki, 'ca.crt'))}\n"
            user = (f"    client-certificate-data: {_b64file(os.path.join(self.pki, 'client.crt'))}\n"
                    f"    client-key-data: {_b64file(os.path.join(self.pki, 'client.key'))}\n")
        return (
            "apiVersion: v1\nkind: Config\n"
            f"current-context: {self.context}\n"
            "clusters:\n"
            f"- name: {self.context}\n  cluster:\n{cluster}"
            "contexts:\n"
            f"- name: {self.context}\n  context:\n    cluster: {self.context}\n    user: {self.context}\n"
            f"    namespace: {namespace}\n"
            "users:\n"
            f"- name: {self.context}\n  user:\n{user}"
            "preferences: {}\n"
        )

    def _ssl_context(self):
        if not self.tls:
            return None
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH, cafile=os.path.join(self.pki, "ca.crt"))
        ctx.load_cert_chain(os.path.join(self.pki, "server.crt"), os.path.join(self.pki, "server.key"))
        ctx.verify_mode = ssl.CERT_REQUIRED  # mTLS: clients must present a cert signed by our CA
        return ctx

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
        await web.TCPSite(api_runner, "127.0.0.1", self.port, ssl_context=self._ssl_context()).start()
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
            loop = asyncio.new_event_loop()
            self.loop = loop
            asyncio.set_event_loop(loop)
            loop.run_until_complete(self._amain())
            loop.run_forever()
            # stop() ran shutdown(): close transports and the loop from the loop's own thread
            try:
                loop.run_until_complete(loop.shutdown_asyncgens())
            finally:
                loop.close()

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
            # every task still pending (container output pumps, log followers, watches) is
            # cancelled and awaited here, so nothing is destroyed pending when the loop closes
            me = asyncio.current_task()
            rest = [t for t in asyncio.all_tasks() if t is not me and not t.done()]
            for t in rest:
                t.cancel()
            if rest:  # bounded: a handler that swallows one cancellation must not hang stop()
                await asyncio.wait(rest, timeout=2.0)
            # catch-all: any subprocess transport of this loop still open (a process whose
            # handle was dropped without close) is closed now, while the loop can still run
            # its callbacks, not later by the GC on a closed loop
            import gc
            from asyncio.base_subprocess import BaseSubprocessTransport

            loop = asyncio.get_running_loop()
            for o in gc.get_objects():
                # type(), not isinstance(): the latter reads __class__, which some proxy objects
                # in the heap (torch's deprecated reduce_op) answer with a warning
                if issubclass(type(o), BaseSubprocessTransport) and o._loop is loop and not o.is_closing():
                    o.close()
            await asyncio.sleep(0)  # let subprocess transports deliver their connection_lost

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
