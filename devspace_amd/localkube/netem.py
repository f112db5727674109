"""A WAN link in front of the local cluster's API server: latency and bandwidth, both ways.

Every other number of the bench runs over loopback, where a protocol's round trips cost
microseconds. A developer's laptop talks to a cloud cluster over tens of milliseconds of RTT
and a few hundred Mbit/s at best, and there the number of round trips per edit and per
connection decides the dev loop. `ShapedLink` is a TCP proxy (TLS passes through untouched)
that delays every chunk by half the RTT in each direction and serialises it at the link rate,
so a kubeconfig pointed at it sees the cluster "far away": exec (sync), port-forward, logs and
every API request pay the same link costs they would on a real one.

    link = ShapedLink(("127.0.0.1", api_port), rtt_ms=30, mbit=100).start()
    point_kubeconfig(kubeconfig_path, cluster.server, link.url("https"))
"""

from __future__ import annotations

import collections
import socket
import threading
import time


class _Pipe:
    """One direction of one connection: a reader thread stamps each chunk with its delivery
    time (one-way delay after it left the link's serialiser), a writer thread sends it then."""

    def __init__(self, src, dst, delay_s, bytes_per_s, on_done):
        self.src, self.dst = src, dst
        self.delay_s, self.bps = delay_s, bytes_per_s
        self.q = collections.deque()
        self.cv = threading.Condition()
        self.link_free = 0.0
        self.on_done = on_done
        self.moved = 0
        threading.Thread(target=self._read, daemon=True).start()
        threading.Thread(target=self._write, daemon=True).start()

    def _read(self):
        while True:
            try:
                data = self.src.recv(1 << 16)
            except OSError:
                data = b""
            now = time.monotonic()
            with self.cv:
                if data:
                    ser = len(data) / self.bps if self.bps else 0.0
                    self.link_free = max(now, self.link_free) + ser
                    self.q.append((self.link_free + self.delay_s, data))
                else:
                    self.q.append((max(now, self.link_free) + self.delay_s, None))  # EOF after the data
                self.cv.notify()
            if not data:
                return

    def _write(self):
        while True:
            with self.cv:
                while not self.q:
                    self.cv.wait()
                due, data = self.q.popleft()
            wait = due - time.monotonic()
            if wait > 0:
                time.sleep(wait)
            if data is None:
                try:
                    self.dst.shutdown(socket.SHUT_WR)
                except OSError:
                    pass
                self.on_done()
                return
            try:
                self.dst.sendall(data)
                self.moved += len(data)
            except OSError:
                try:
                    self.src.shutdown(socket.SHUT_RD)
                except OSError:
                    pass
                self.on_done()
                return


class ShapedLink:
    """TCP proxy 127.0.0.1:<port> -> target with `rtt_ms` round-trip latency and `mbit` Mbit/s
    per direction (0 = unlimited)."""

    def __init__(self, target, rtt_ms: float = 30.0, mbit: float = 100.0):
        self.target = target
        self.delay_s = rtt_ms / 2000.0
        self.bps = mbit * 1e6 / 8.0 if mbit else 0.0
        self.sock = socket.socket()
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(128)
        self.port = self.sock.getsockname()[1]
        self.connections = 0
        self.bytes_up = self.bytes_down = 0
        self._stop = False
        self._lock = threading.Lock()

    def url(self, scheme="https"):
        return f"{scheme}://127.0.0.1:{self.port}"

    def start(self):
        threading.Thread(target=self._accept, daemon=True).start()
        return self

    def _accept(self):
        while not self._stop:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            try:
                s = socket.create_connection(self.target)
            except OSError:
                c.close()
                continue
            for x in (c, s):
                x.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            with self._lock:
                self.connections += 1
            self._pair(c, s)

    def _pair(self, c, s):
        left = [2]
        pipes = []

        def done():
            with self._lock:
                left[0] -= 1
                last = left[0] == 0
            if last:
                self.bytes_up += pipes[0].moved
                self.bytes_down += pipes[1].moved
                for x in (c, s):
                    try:
                        x.close()
                    except OSError:
                        pass

        pipes.append(_Pipe(c, s, self.delay_s, self.bps, done))  # client -> cluster
        pipes.append(_Pipe(s, c, self.delay_s, self.bps, done))  # cluster -> client

    def stop(self):
        self._stop = True
        try:
            self.sock.close()
        except OSError:
            pass


def point_kubeconfig(path: str, server: str, new_server: str) -> None:
    """Rewrites the kubeconfig's `server:` (the cluster's own URL) to the shaped link's."""
    with open(path) as f:
        text = f.read()
    assert f"server: {server}" in text, (server, text)
    with open(path, "w") as f:
        f.write(text.replace(f"server: {server}", f"server: {new_server}"))
