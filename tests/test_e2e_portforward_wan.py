"""Port-forward of a request held across an app restart, with the cluster behind a slow link (40 ms
RTT, devspace_amd/localkube/netem.py), as a laptop reaches a remote MI355X node.

By default, on a remote cluster, connections go through the sync's in-container helper
(`devspace-helper forward`): a connection the restarting app refuses is held *in the pod* and
made once when the app listens, so every request reaches the app exactly once and within ms of
it listening. Through the kubelet's port-forward (DEVSPACE_PORTFORWARD_VIA=kubelet) every held
request is retried one stream at a time and reaches the app exactly once, as through kubectl
port-forward (/root/reference/pkg/devspace/kubectl/client.go:356-380); each retry costs a round
trip. With DEVSPACE_PORTFORWARD_HEDGE=1 (kubelet path) a held GET (repeatable, RFC 9110 §9.2.2) goes out on a new
stream pair of the pod's tunnel every third of a round trip while earlier attempts are in flight;
the first answer wins, and the app may see the GET more than once. A POST still goes out once.
An API server without the tunnel (before Kubernetes 1.30) gets a WebSocket per connection.
"""
import json
import os
import time
import urllib.request

import pytest
import yaml

from conftest import DevspaceEnv
from test_e2e_cli import running, wait_for
from test_e2e_services import _refused, _restart_project, _stop


@pytest.mark.parametrize("via,hedge", [("auto", False), ("kubelet", False), ("kubelet", True)],
                         ids=["default-helper", "kubelet", "kubelet-hedge-opt-in"])
def test_held_requests_across_a_restart_on_a_remote_cluster(tmp_path, via, hedge):
    from devspace_amd.localkube import LocalCluster
    from devspace_amd.localkube.netem import ShapedLink, point_kubeconfig

    cluster = LocalCluster(str(tmp_path / "state"), gpus=0, tls=True).start()
    link = None
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        lk.env.pop("DEVSPACE_PORTFORWARD_HEDGE", None)
        lk.env.pop("DEVSPACE_PORTFORWARD_VIA", None)
        if hedge:
            lk.env["DEVSPACE_PORTFORWARD_HEDGE"] = "1"
        if via != "auto":
            lk.env["DEVSPACE_PORTFORWARD_VIA"] = via
        link = ShapedLink(("127.0.0.1", cluster.port), rtt_ms=40, mbit=100).start()
        point_kubeconfig(lk.kubeconfig, cluster.server, link.url("https"))
        proj, remote, local = _restart_project(lk, "qs-wan-hold", "pf-wan")
        hits = tmp_path / "hits.log"
        values = os.path.join(proj, "chart", "values.yaml")
        v = yaml.safe_load(open(values))
        v["components"][0]["containers"][0]["env"] += [{"name": "HITS_FILE", "value": str(hits)},
                                                        {"name": "START_DELAY_MS", "value": "600"}]
        open(values, "w").write(yaml.safe_dump(v))
        index = os.path.join(proj, "index.js")
        # every request is logged; the app listens 0.6 s after it starts (a slow restart: the held
        # requests below certainly meet a refusing pod and are retried)
        last = "}).listen(port, () => console.log('Example app listening on port ' + port + '!'));"
        src = open(index).read()
        assert last in src
        src = src.replace(
            "http.createServer((req, res) => {",
            "const srv = http.createServer((req, res) => {\n  require('fs').appendFileSync(process.env.HITS_FILE, "
            "req.method + ' ' + req.url + '\\n');", 1).replace(
            last, "});\nsetTimeout(() => srv.listen(port, () => console.log('Example app listening on port ' + port + "
                  "'!')), Number(process.env.START_DELAY_MS || 0));")
        open(index, "w").write(src)
        dev = lk.popen(["dev", "--terminal=false"], proj)
        try:
            wait_for(lambda: (lambda b: b.startswith("Hello") if b else False)(_fetch(local)), timeout=90,
                     what="forwarded server")
            root = json.loads(running(lk.pods("pf-wan"))[0]["metadata"]["annotations"]["devspace.sh/local-roots"])
            pod_index = os.path.join(list(root.values())[0], "app", "index.js")
            pf_log = os.path.join(proj, ".devspace", "logs", "portforwarding.log")
            if via == "auto":  # the link to the helper comes up once the tunnel's round trip is known
                wait_for(lambda: os.path.exists(pf_log) and "through the in-container helper" in open(pf_log).read(),
                         timeout=30, what="helper link")
            t_link = time.monotonic()
            for i in range(4):
                with open(index, "a") as f:
                    f.write(f"// edit {i}\n")
                wait_for(lambda: f"// edit {i}" in open(pod_index).read(), timeout=30, what="synced edit")
                wait_for(lambda: _refused(remote), timeout=10, what="old server stopped")
                method = "GET" if i % 2 == 0 else "POST"
                req = urllib.request.Request(f"http://127.0.0.1:{local}/held-{i}",
                                             data=b"x" if method == "POST" else None, method=method)
                body = urllib.request.urlopen(req, timeout=15).read().decode()
                assert body.startswith("Hello"), body
                wait_for(lambda: not _refused(remote), timeout=30, what="new server")
        finally:
            _stop(dev)
        lines = hits.read_text().splitlines()
        for i in (1, 3):
            assert lines.count(f"POST /held-{i}") == 1, lines
        spans = [json.loads(l) for l in open(os.path.join(proj, ".devspace", "logs", "trace.jsonl"))
                 if '"portforward.stream"' in l]
        hedged = [s for s in spans if s.get("hedged") == "1"]
        log = open(pf_log).read() if os.path.exists(pf_log) else ""
        if via == "auto":
            # after the link is up every stream goes through the helper: no refused attempt, each
            # held request (GET and POST) delivered once
            late = [s for s in spans if s["start_us"] / 1e6 >= t_link]
            assert late and all(s.get("via") == "helper" and s["outcome"] == "reply" for s in late), late
            for i in (0, 2):
                assert lines.count(f"GET /held-{i}") == 1, lines
            assert not hedged, hedged
            return
        assert all(s.get("via") == "tunnel" for s in spans), spans
        if hedge:
            for i in (0, 2):
                assert 1 <= lines.count(f"GET /held-{i}") <= 8, lines
            assert any(s["outcome"] == "reply" for s in hedged), spans
            assert "may reach the app more than once" in log, log
        else:
            # each held GET reached the app exactly once, after at least one refused attempt
            for i in (0, 2):
                assert lines.count(f"GET /held-{i}") == 1, lines
            assert not hedged, hedged
            assert any(s["outcome"] == "refused" for s in spans), spans
            assert "more than once" not in log, log
    finally:
        if link is not None:
            link.stop()
        cluster.stop()


def _fetch(port):
    try:
        return urllib.request.urlopen(f"http://127.0.0.1:{port}/", timeout=5).read().decode()
    except Exception:
        return None


def test_an_api_server_without_the_tunnel_gets_a_websocket_per_connection(tmp_path):
    """Kubernetes before 1.30 refuses the SPDY-over-WebSocket upgrade (its stream negotiation does
    not know the subprotocol): the forward falls back to one portforward.k8s.io WebSocket per
    connection, says so in its log, and serves every connection."""
    from devspace_amd.localkube import LocalCluster

    cluster = LocalCluster(str(tmp_path / "state"), gpus=0, tls=True, portforward_tunnel=False).start()
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        proj, remote, local = _restart_project(lk, "qs-no-tunnel", "pf-old")
        dev = lk.popen(["dev", "--terminal=false"], proj)
        try:
            wait_for(lambda: (lambda b: b.startswith("Hello") if b else False)(_fetch(local)), timeout=90,
                     what="forwarded server")
            for _ in range(5):
                assert (_fetch(local) or "").startswith("Hello")
        finally:
            _stop(dev)
        assert cluster.api.portforward_tunnels == 0
        spans = [json.loads(l) for l in open(os.path.join(proj, ".devspace", "logs", "trace.jsonl"))
                 if '"portforward.stream"' in l]
        assert spans and all(s.get("via") == "websocket" for s in spans), spans
        log = open(os.path.join(proj, ".devspace", "logs", "portforwarding.log")).read()
        assert "no multiplexed port-forward" in log, log
    finally:
        cluster.stop()


BIG_ROUTES = r"""
const crypto = require('crypto');
const BIG = Buffer.alloc(48 << 20);
for (let i = 0; i < BIG.length; i += 4) BIG.writeUInt32LE(Math.imul(i, 2654435761 | 0) >>> 0, i);
let bigSent = 0;  // bytes of /big the app got rid of: written while the socket accepted them
const srv = http.createServer((req, res) => {
  if (req.url === '/big') {
    res.writeHead(200, {'Content-Length': BIG.length});
    bigSent = 0;
    const more = () => {
      while (bigSent < BIG.length) {
        const c = BIG.subarray(bigSent, bigSent + 65536);
        bigSent += c.length;
        if (!res.write(c)) return res.once('drain', more);  // backpressure: wait for the socket
      }
      res.end();
    };
    more();
    return;
  }
  if (req.url === '/progress') {
    res.end(String(bigSent));
    return;
  }
  if (req.url === '/upload') {
    const h = crypto.createHash('sha256');
    let n = 0;
    req.on('data', (c) => { n += c.length; h.update(c); });
    req.on('end', () => res.end(n + ' ' + h.digest('hex')));
    return;
  }
"""


@pytest.mark.parametrize("via", ["helper", "kubelet"])
def test_large_transfers_are_flow_controlled(tmp_path, via):
    """A 48 MiB download to a local reader that reads slowly neither piles up in `devspace dev`'s
    memory nor holds up the pod's other connections (a second request goes through meanwhile),
    and the bytes of a 48 MiB download and a 32 MiB upload arrive intact.
    * Through the in-container helper every connection has a window, 4 MiB unacknowledged per
      direction (src/sync/fwd_proto.h): the app itself is held back.
    * Through the kubelet's tunnel the client sends SPDY window updates, but kubelets
      (spdystream) do not enforce windows: past 4 MiB in memory the connection's data waits in a
      nameless temp file (kube::SpdyMailbox) instead of stalling the tunnel's reader."""
    import hashlib
    import socket

    import psutil

    from devspace_amd.localkube import LocalCluster

    cluster = LocalCluster(str(tmp_path / "state"), gpus=0, tls=True).start()
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        lk.env["DEVSPACE_PORTFORWARD_VIA"] = via
        proj, remote, local = _restart_project(lk, "qs-pf-big", "pf-big")
        index = os.path.join(proj, "index.js")
        src = open(index).read()
        assert "http.createServer((req, res) => {" in src
        open(index, "w").write(src.replace("http.createServer((req, res) => {", BIG_ROUTES, 1)
                               .replace("}).listen(port,", "});\nsrv.listen(port,", 1))
        dev = lk.popen(["dev", "--terminal=false"], proj)
        try:
            wait_for(lambda: (lambda b: b.startswith("Hello") if b else False)(_fetch(local)), timeout=90,
                     what="forwarded server")
            pf_log = os.path.join(proj, ".devspace", "logs", "portforwarding.log")
            if via == "helper":
                wait_for(lambda: os.path.exists(pf_log) and "through the in-container helper" in open(pf_log).read(),
                         timeout=30, what="helper link")
            expected = bytearray(48 << 20)
            mv = memoryview(expected).cast("I")
            for i in range(len(mv)):
                mv[i] = (i * 4 * 2654435761) & 0xFFFFFFFF
            proc = psutil.Process(dev.pid)
            rss0 = proc.memory_info().rss
            s = socket.create_connection(("127.0.0.1", local), timeout=30)
            s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 16)
            s.sendall(b"GET /big HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
            got = bytearray()
            peak = rss0
            t_end = time.monotonic() + 2.0
            while time.monotonic() < t_end:  # a slow reader: 64 KiB every 20 ms
                got += s.recv(1 << 16)
                time.sleep(0.02)
                peak = max(peak, proc.memory_info().rss)
            # how far ahead of the reader the app got: what the forward holds in between (another
            # connection through the same forward, not held back by the first one's window)
            app_ahead = (int(urllib.request.urlopen(f"http://127.0.0.1:{local}/progress", timeout=10).read())
                         - len(got)) / 2 ** 20
            while True:
                b = s.recv(1 << 20)
                if not b:
                    break
                got += b
            s.close()
            head, _, body = bytes(got).partition(b"\r\n\r\n")
            assert head.startswith(b"HTTP/1.1 200"), head[:200]
            assert len(body) == len(expected) and hashlib.sha256(body).digest() == hashlib.sha256(expected).digest()
            growth = (peak - rss0) / 2 ** 20
            print(f"while the reader lagged ({via}): the app was {app_ahead:.1f} MiB ahead, "
                  f"devspace dev RSS grew {growth:.1f} MiB")
            if via == "helper":
                assert app_ahead < 24, app_ahead
            if "/build/" not in os.environ.get("DEVSPACE_BIN", ""):  # sanitizer builds' RSS is their own
                assert growth < 24, growth
            payload = os.urandom(32 << 20)
            req = urllib.request.Request(f"http://127.0.0.1:{local}/upload", data=payload, method="POST")
            reply = urllib.request.urlopen(req, timeout=60).read().decode()
            assert reply == f"{len(payload)} {hashlib.sha256(payload).hexdigest()}", reply
        finally:
            _stop(dev)
        spans = [json.loads(l) for l in open(os.path.join(proj, ".devspace", "logs", "trace.jsonl"))
                 if '"portforward.stream"' in l]
        assert any(s.get("via") == ("helper" if via == "helper" else "tunnel") for s in spans), spans
    finally:
        cluster.stop()
