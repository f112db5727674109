"""The server side of Kubernetes' multiplexed port-forward (KEP-4006, Kubernetes >= 1.30): a
WebSocket with subprotocol "SPDY/3.1+portforward.k8s.io" whose binary messages carry a SPDY/3.1
byte stream. The client opens a pair of streams per forwarded connection (headers streamtype
error|data, port, requestid); when both arrived the kubelet dials the pod's port, copies bytes
on the data stream and reports a failed dial on the error stream. The client side is
src/kube/spdy.cc; this is what the local cluster serves so that path is exercised end to end.
"""

from __future__ import annotations

import asyncio
import struct
import zlib

PROTOCOL = "SPDY/3.1+portforward.k8s.io"

_NAMES = ["options", "head", "post", "put", "delete", "trace", "accept", "accept-charset", "accept-encoding",
          "accept-language", "accept-ranges", "age", "allow", "authorization", "cache-control", "connection",
          "content-base", "content-encoding", "content-language", "content-length", "content-location",
          "content-md5", "content-range", "content-type", "date", "etag", "expect", "expires", "from", "host",
          "if-match", "if-modified-since", "if-none-match", "if-range", "if-unmodified-since", "last-modified",
          "location", "max-forwards", "pragma", "proxy-authenticate", "proxy-authorization", "range", "referer",
          "retry-after", "server", "te", "trailer", "transfer-encoding", "upgrade", "user-agent", "vary", "via",
          "warning", "www-authenticate", "method", "get", "status", "200 OK", "version", "HTTP/1.1", "url",
          "public", "set-cookie", "keep-alive", "origin"]
# SPDY/3 header-compression dictionary (1423 bytes, zlib dictionary id 0xe3c6a7c2)
DICTIONARY = b"".join(struct.pack(">I", len(n)) + n.encode() for n in _NAMES) + (
    b"100101201202205206300302303304305306307402405406407408409410411412413414415416417502504505"
    b"203 Non-Authoritative Information204 No Content301 Moved Permanently400 Bad Request401 Unauthorized"
    b"403 Forbidden404 Not Found500 Internal Server Error501 Not Implemented503 Service Unavailable"
    b"Jan Feb Mar Apr May Jun Jul Aug Sept Oct Nov Dec 00:00:00 Mon, Tue, Wed, Thu, Fri, Sat, Sun, GMT"
    b"chunked,text/html,image/png,image/jpg,image/gif,application/xml,application/xhtml+xml,text/plain,"
    b"text/javascript,publicprivatemax-age=gzip,deflate,sdchcharset=utf-8charset=iso-8859-1,utf-,*,enq=0.")

SYN_STREAM, SYN_REPLY, RST_STREAM, SETTINGS, PING, GOAWAY, HEADERS, WINDOW_UPDATE = 1, 2, 3, 4, 6, 7, 8, 9
FLAG_FIN = 0x01


def control_frame(ftype: int, flags: int, body: bytes) -> bytes:
    return struct.pack(">HHI", 0x8003, ftype, (flags << 24) | len(body)) + body


def data_frame(sid: int, flags: int, data: bytes) -> bytes:
    return struct.pack(">II", sid & 0x7FFFFFFF, (flags << 24) | len(data)) + data


def parse_frames(buf: bytearray):
    """Yields (control, type_or_stream_id, flags, body) for every complete frame at the front of
    `buf`, removing them."""
    while len(buf) >= 8:
        w0, w1 = struct.unpack_from(">II", buf, 0)
        length = w1 & 0xFFFFFF
        if len(buf) < 8 + length:
            return
        body = bytes(buf[8:8 + length])
        del buf[:8 + length]
        if w0 & 0x80000000:
            yield True, w0 & 0xFFFF, w1 >> 24, body
        else:
            yield False, w0 & 0x7FFFFFFF, w1 >> 24, body


def encode_headers(h: dict) -> bytes:
    out = struct.pack(">I", len(h))
    for k, v in h.items():
        kb, vb = k.encode(), v.encode()
        out += struct.pack(">I", len(kb)) + kb + struct.pack(">I", len(vb)) + vb
    return out


def decode_headers(raw: bytes) -> dict:
    (n,), off, out = struct.unpack_from(">I", raw, 0), 4, {}
    for _ in range(n):
        (kl,) = struct.unpack_from(">I", raw, off)
        k = raw[off + 4:off + 4 + kl].decode()
        off += 4 + kl
        (vl,) = struct.unpack_from(">I", raw, off)
        out[k.lower()] = raw[off + 4:off + 4 + vl].decode()
        off += 4 + vl
    return out


class _Pair:
    """The error + data streams of one forwarded connection."""

    def __init__(self, rid, port):
        self.rid = rid
        self.port = port
        self.error = self.data = None
        self.pending = bytearray()  # data that arrived before the pod connection
        self.client_eof = False
        self.writer = None
        self.task = None
        self.done = False


class Tunnel:
    """One client's tunnel. `dial(port)` opens the pod connection (asyncio streams) or raises;
    `refused(port, err)` is the kubelet's error text for a failed dial."""

    def __init__(self, ws, dial, refused):
        self.ws = ws
        self.dial = dial
        self.refused = refused
        self.inz = zlib.decompressobj(zdict=DICTIONARY)
        self.outz = zlib.compressobj(zdict=DICTIONARY)
        self.wlock = asyncio.Lock()
        self.pairs = {}  # request id -> _Pair
        self.streams = {}  # stream id -> (_Pair, "error" | "data")
        self.streams_opened = 0
        self.pings_answered = 0  # of the PING (even id: the server's) sent when the tunnel opens

    async def _send(self, frame: bytes):
        async with self.wlock:
            await self.ws.send_bytes(frame)

    async def _reply(self, sid: int):
        async with self.wlock:  # header blocks are compressed in wire order
            block = self.outz.compress(encode_headers({})) + self.outz.flush(zlib.Z_SYNC_FLUSH)
            await self.ws.send_bytes(control_frame(SYN_REPLY, 0, struct.pack(">I", sid) + block))

    async def _data(self, sid: int, data: bytes, fin=False):
        for off in range(0, max(len(data), 1), 65535):
            chunk = data[off:off + 65535]
            last = off + 65535 >= len(data)
            await self._send(data_frame(sid, FLAG_FIN if fin and last else 0, chunk))

    async def _forward(self, pair: _Pair):
        try:
            await self._pump(pair)
        finally:  # the pair's bookkeeping goes with it
            self.pairs.pop(pair.rid, None)
            self.streams.pop(pair.error, None)
            self.streams.pop(pair.data, None)

    async def _pump(self, pair: _Pair):
        try:
            reader, writer = await self.dial(pair.port)
        except (OSError, LookupError) as e:  # refused, or the pod is gone
            # the kubelet's wording; the client keys on "connection refused"
            await self._data(pair.error, self.refused(pair.port, e).encode(), fin=True)
            await self._data(pair.data, b"", fin=True)
            pair.done = True
            return
        pair.writer = writer
        if pair.pending:
            writer.write(bytes(pair.pending))
            pair.pending.clear()
        if pair.client_eof and writer.can_write_eof():
            writer.write_eof()
        try:
            while True:
                chunk = await reader.read(65536)
                if not chunk:
                    break
                await self._data(pair.data, chunk)
        except (ConnectionError, asyncio.CancelledError):
            pass
        pair.done = True
        try:
            await self._data(pair.data, b"", fin=True)
            await self._data(pair.error, b"", fin=True)
        except ConnectionError:
            pass
        writer.close()

    def _on_syn(self, sid: int, flags: int, headers: dict):
        rid, role = headers.get("requestid", ""), headers.get("streamtype", "")
        try:
            port = int(headers.get("port", "0"))
        except ValueError:
            port = 0
        pair = self.pairs.get(rid)
        if pair is None:
            pair = self.pairs[rid] = _Pair(rid, port)
        setattr(pair, role if role in ("error", "data") else "error", sid)
        self.streams[sid] = (pair, role)
        if role == "data" and flags & FLAG_FIN:
            pair.client_eof = True
        if pair.error is not None and pair.data is not None and pair.task is None:
            self.streams_opened += 1
            pair.task = asyncio.ensure_future(self._forward(pair))

    def _on_data(self, sid: int, flags: int, data: bytes):
        entry = self.streams.get(sid)
        if entry is None:
            return
        pair, role = entry
        if role != "data":
            return  # the client writes nothing on the error stream
        if pair.writer is not None:
            if data:
                pair.writer.write(data)
            if flags & FLAG_FIN and pair.writer.can_write_eof():
                pair.writer.write_eof()
        else:
            pair.pending += data
            if flags & FLAG_FIN:
                pair.client_eof = True

    def _on_rst(self, sid: int):
        entry = self.streams.pop(sid, None)
        if entry is None:
            return
        pair, _ = entry
        if pair.task is not None and not pair.done:
            pair.task.cancel()
        if pair.writer is not None:
            pair.writer.close()

    async def run(self):
        from aiohttp import WSMsgType

        buf = bytearray()
        try:
            # the server's own PING (even ids are the server's, spdystream's convention): the
            # client must answer it, and must not answer the answers to its own (odd) ones
            await self._send(control_frame(PING, 0, struct.pack(">I", 2)))
            async for msg in self.ws:
                if msg.type != WSMsgType.BINARY:
                    continue
                buf += msg.data
                for control, t, flags, body in parse_frames(buf):
                    if not control:
                        self._on_data(t, flags, body)
                    elif t == SYN_STREAM:
                        sid = struct.unpack_from(">I", body, 0)[0] & 0x7FFFFFFF
                        headers = decode_headers(self.inz.decompress(body[10:]))
                        await self._reply(sid)
                        self._on_syn(sid, flags, headers)
                    elif t == RST_STREAM:
                        self._on_rst(struct.unpack_from(">I", body, 0)[0] & 0x7FFFFFFF)
                    elif t == PING:
                        if struct.unpack_from(">I", body, 0)[0] % 2 == 0:
                            self.pings_answered += 1  # our own, come back
                        else:
                            await self._send(control_frame(PING, 0, body))
                    elif t in (SYN_REPLY, HEADERS):
                        self.inz.decompress(body[4:])  # keep the zlib stream in step
                    elif t == GOAWAY:
                        break
        except ConnectionError:
            pass
        for pair in self.pairs.values():
            if pair.task is not None and not pair.done:
                pair.task.cancel()
            if pair.writer is not None:
                pair.writer.close()
