"""The CLI against an API server that answers garbage: random bytes, impossible
Content-Length / chunk sizes, a WebSocket upgrade followed by a frame claiming 2^63 bytes,
100 kB status lines and malformed JSON. Every command must end with an error (or an empty
result) promptly — no crash, abort, hang or unbounded allocation. Under scripts/sanitize.sh the
sanitized CLI runs this too."""

import os
import random
import socket
import subprocess
import threading
import time

from conftest import ROOT

BIN = os.environ.get("DEVSPACE_BIN") or os.path.join(ROOT, "bin", "devspace")


def _responses(rng):
    return [
        lambda: bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 4000))),
        lambda: b"HTTP/1.1 200 OK\r\nContent-Length: 99999999999\r\n\r\n{\"kind\":",
        lambda: b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nfffffffffffffff\r\nabc",
        lambda: b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n",
        lambda: b"HTTP/1.1 200 OK\r\nContent-Length: 5\r\n\r\n{\"a\"",
        lambda: (b"HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                 b"Sec-WebSocket-Protocol: v4.channel.k8s.io\r\n\r\n" + bytes([0x82, 0x7f]) + b"\x7f" + b"\xff" * 7 + b"x"),
        lambda: b"HTTP/1.1 " + b"9" * 5000 + b"\r\nX: " + b"y" * 100000 + b"\r\n\r\n",
        lambda: b"HTTP/1.1 500 Oops\r\nContent-Type: application/json\r\nContent-Length: 20\r\n\r\n{\"message\": [1,2,{]",
        lambda: b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: 24\r\n\r\n{\"items\": [{\"a\": 1e999}]",
    ]


def test_cli_survives_a_hostile_api_server(tmp_path):
    rng = random.Random(1234)
    responses = _responses(rng)
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(64)
    port = srv.getsockname()[1]
    stop = threading.Event()

    def serve():
        while not stop.is_set():
            try:
                c, _ = srv.accept()
            except OSError:
                return
            try:
                c.settimeout(2)
                c.recv(65536)
                c.sendall(rng.choice(responses)())
            except OSError:
                pass
            finally:
                try:
                    c.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass
                c.close()

    threading.Thread(target=serve, daemon=True).start()
    kc = tmp_path / "kubeconfig"
    kc.write_text(f"""apiVersion: v1
kind: Config
clusters:
- name: c
  cluster: {{server: "http://127.0.0.1:{port}"}}
contexts:
- name: x
  context: {{cluster: c, user: u, namespace: default}}
current-context: x
users:
- name: u
  user: {{token: t}}
""")
    proj = tmp_path / "p"
    (proj / ".devspace").mkdir(parents=True)
    (proj / ".devspace" / "config.yaml").write_text(
        "version: v1alpha2\ncluster:\n  kubeContext: x\n  namespace: default\n"
        "dev:\n  selectors:\n  - name: default\n    labelSelector:\n      app: x\n")
    env = dict(os.environ, KUBECONFIG=str(kc), HOME=str(tmp_path), DEVSPACE_NONINTERACTIVE="1")
    try:
        for args in (["status", "deployments"], ["analyze", "--wait=false"], ["enter", "--", "ls"], ["logs"],
                     ["purge"], ["list", "spaces"]) * 4:
            t0 = time.time()
            p = subprocess.run([BIN] + args, cwd=proj, env=env, capture_output=True, text=True, timeout=60)
            assert p.returncode in (0, 1), (args, p.returncode, p.stderr[-2000:])
            assert time.time() - t0 < 20, (args, p.stdout[-500:], p.stderr[-500:])
    finally:
        stop.set()
        srv.close()
