"""The shaped WAN link of the local cluster (devspace_amd/localkube/netem.py): it must add the
configured round-trip latency and cap the rate, both ways, and pass a half-close through, or
the WAN numbers built on it mean nothing."""

import socket
import threading
import time

from devspace_amd.localkube.netem import ShapedLink


def _echo_server():
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(8)

    def serve():
        while True:
            try:
                c, _ = srv.accept()
            except OSError:
                return

            def one(c=c):
                while True:
                    d = c.recv(1 << 16)
                    if not d:
                        c.shutdown(socket.SHUT_WR)
                        c.close()
                        return
                    c.sendall(d)

            threading.Thread(target=one, daemon=True).start()

    threading.Thread(target=serve, daemon=True).start()
    return srv


def test_round_trip_latency_is_added():
    srv = _echo_server()
    link = ShapedLink(srv.getsockname(), rtt_ms=40, mbit=0).start()
    try:
        c = socket.create_connection(("127.0.0.1", link.port))
        c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        rtts = []
        for _ in range(5):
            t0 = time.perf_counter()
            c.sendall(b"ping")
            assert c.recv(16) == b"ping"
            rtts.append((time.perf_counter() - t0) * 1000)
        rtts.sort()
        assert 38 <= rtts[2] < 60, rtts
        c.shutdown(socket.SHUT_WR)  # the half-close reaches the server, its close comes back
        assert c.recv(16) == b""
        c.close()
    finally:
        link.stop()
        srv.close()


def test_rate_is_capped_each_way():
    srv = _echo_server()
    link = ShapedLink(srv.getsockname(), rtt_ms=2, mbit=80).start()  # 10 MB/s
    try:
        c = socket.create_connection(("127.0.0.1", link.port))
        payload = b"x" * (4 << 20)
        got = bytearray()
        t0 = time.perf_counter()
        threading.Thread(target=lambda: (c.sendall(payload), c.shutdown(socket.SHUT_WR)), daemon=True).start()
        while True:
            d = c.recv(1 << 16)
            if not d:
                break
            got += d
        dt = time.perf_counter() - t0
        assert bytes(got) == payload
        mbps = len(payload) / dt / 1e6
        assert 6.0 < mbps < 11.0, mbps  # 10 MB/s each way (the echo's two directions overlap)
        c.close()
    finally:
        link.stop()
        srv.close()
