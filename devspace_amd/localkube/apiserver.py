"""Kubernetes API server subset (REST + WebSocket exec/attach/port-forward + logs).

Enough of the API surface for every call the devspace CLI makes:
CRUD on any resource kind (core + named groups), label/field selectors, graceful pod
deletion with ownerReference cascade, pod logs (tail / follow / previous), exec and attach on
the v4.channel.k8s.io WebSocket protocol (with TTY + resize), and WebSocket port-forwarding.
"""

from __future__ import annotations

import asyncio
import fcntl
import json
import os
import pty
import copy
import struct
import termios
import time

import yaml
from aiohttp import WSMsgType, web

from . import spdy
from .kubelet import close_proc
from .store import CLUSTER_SCOPED, ApiError, labels_match, parse_selector

GROUP_KINDS = {
    "apps": {"deployments", "statefulsets", "replicasets", "daemonsets", "controllerrevisions"},
    "batch": {"jobs", "cronjobs"},
    "rbac.authorization.k8s.io": {"roles", "rolebindings", "clusterroles", "clusterrolebindings"},
    "autoscaling": {"horizontalpodautoscalers"},
    "networking.k8s.io": {"ingresses", "networkpolicies"},
    "extensions": {"deployments", "ingresses", "replicasets", "daemonsets"},
}


def _err(e: ApiError):
    return web.json_response(e.status(), status=e.code)


def _exit_status(code):
    if code == 0:
        return {"metadata": {}, "status": "Success"}
    return {"metadata": {}, "status": "Failure", "message": f"command terminated with non-zero exit code: {code}",
            "reason": "NonZeroExitCode", "details": {"causes": [{"reason": "ExitCode", "message": str(code)}]}}


class ApiServer:
    def __init__(self, store, kubelet, token_validator=None):
        self.store = store
        self.kubelet = kubelet
        # token_validator(token) -> bool: when set, requests need a valid bearer token (or a
        # verified client certificate on the TLS listener) — expired tokens get 401
        self.token_validator = token_validator
        self.auth_failures = 0
        self.portforward_tunnels = 0  # multiplexed port-forward tunnels served (SPDY over WebSocket)
        self.portforward_tunnel = True  # False: serve only the WebSocket-per-connection protocols
        self.open_tunnels = set()  # their WebSockets (close_tunnels(): an idle timeout, a restart)
        self.tunnel_pings_answered = 0  # the tunnels' server PINGs the clients echoed
        # Fault switch (API Priority and Fairness under load): the first `throttle_first` requests
        # of every (verb, resource) are answered `429 Too Many Requests` + `Retry-After`. The
        # counts start over with reset_throttle(), so every CLI command can be throttled afresh.
        self.throttle_first = 0
        self.retry_after = "1"
        self.throttled = {}  # (verb, resource) -> requests answered 429
        # Namespace-scoped users (RBAC as a Role + RoleBinding in one namespace grants it, e.g.
        # a DevSpace.cloud Space or a multi-tenant cluster): bearer token -> the namespace it may
        # use. Everything cluster-scoped (nodes, namespaces, cluster roles, PVs) and every other
        # namespace answers 403 Forbidden; discovery (/version, /api, /apis) stays open.
        self.scoped_tokens = {}
        self.forbidden = 0

    async def close_tunnels(self):
        """Closes every open port-forward tunnel, as an API server's idle timeout or restart does."""
        for ws in list(self.open_tunnels):
            await ws.close()

    def reset_throttle(self, first=None, retry_after=None):
        if first is not None:
            self.throttle_first = first
        if retry_after is not None:
            self.retry_after = str(retry_after)
        self.throttled = {}

    @staticmethod
    def _verb(request):
        """(k8s verb, resource[/subresource]) of a REST path, as APF and RBAC see it."""
        p = request.path
        segs = [x for x in p.split("/") if x]
        segs = segs[2:] if segs[:1] == ["api"] else segs[3:]  # /api/v1/... | /apis/g/v/...
        if len(segs) >= 3 and segs[0] == "namespaces":
            segs = segs[2:]
        resource = segs[0] if segs else ""
        named = len(segs) > 1
        if len(segs) > 2:
            resource += "/" + segs[2]
        m = request.method
        if request.headers.get("Upgrade", "").lower() == "websocket":
            verb = "connect"
        elif m == "GET":
            verb = "watch" if request.query.get("watch") in ("1", "true") else ("get" if named else "list")
        else:
            verb = {"POST": "create", "PUT": "update", "PATCH": "patch"}.get(m) or (
                "delete" if named else "deletecollection")
        return verb, resource

    @web.middleware
    async def _rbac(self, request, handler):
        h = request.headers.get("Authorization", "")
        ns_allowed = self.scoped_tokens.get(h[7:]) if h.startswith("Bearer ") else None
        if ns_allowed is None or not request.path.startswith(("/api/", "/apis/")):
            return await handler(request)
        segs = [x for x in request.path.split("/") if x]
        group = "" if segs[:1] == ["api"] else (segs[1] if len(segs) > 1 else "")
        rest = segs[2:] if segs[:1] == ["api"] else segs[3:]
        if len(rest) >= 3 and rest[0] == "namespaces" and rest[1] == ns_allowed:
            return await handler(request)
        if not rest:  # /api/v1, /apis/apps/v1: resource discovery
            return await handler(request)
        verb, resource = self._verb(request)
        self.forbidden += 1
        where = f'in the namespace "{rest[1]}"' if len(rest) >= 3 and rest[0] == "namespaces" else "at the cluster scope"
        msg = (f'{resource.split("/")[0]} is forbidden: User "system:serviceaccount:{ns_allowed}:developer" cannot '
               f'{verb} resource "{resource.split("/")[0]}" in API group "{group}" {where}')
        return web.json_response({"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
                                  "message": msg, "reason": "Forbidden", "code": 403}, status=403)

    @web.middleware
    async def _throttle(self, request, handler):
        if self.throttle_first > 0 and request.path.startswith(("/api/", "/apis/")):
            key = self._verb(request)
            n = self.throttled.get(key, 0)
            if n < self.throttle_first:
                self.throttled[key] = n + 1
                return web.json_response(
                    {"kind": "Status", "apiVersion": "v1", "status": "Failure", "code": 429,
                     "reason": "TooManyRequests", "message": "Too many requests, please try again later.",
                     "details": {"retryAfterSeconds": int(self.retry_after)}},
                    status=429, headers={"Retry-After": self.retry_after})
        return await handler(request)

    @web.middleware
    async def _auth(self, request, handler):
        if self.token_validator is not None:
            tr = request.transport
            peer_cert = tr.get_extra_info("peercert") if tr is not None else None
            h = request.headers.get("Authorization", "")
            if not peer_cert and not (h.startswith("Bearer ") and self.token_validator(h[7:])):
                self.auth_failures += 1
                return web.json_response({"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                          "message": "Unauthorized", "reason": "Unauthorized", "code": 401},
                                         status=401)
        return await handler(request)

    def app(self):
        app = web.Application(client_max_size=256 * 1024 * 1024, middlewares=[self._auth, self._rbac, self._throttle])
        app.router.add_get("/version", self.version)
        app.router.add_get("/api", self.api_versions)
        app.router.add_get("/apis", self.api_groups)
        app.router.add_get("/healthz", self.healthz)
        app.router.add_route("*", "/api/{version}/{tail:.*}", self.dispatch_core)
        app.router.add_route("*", "/apis/{group}/{version}/{tail:.*}", self.dispatch_group)
        return app

    async def healthz(self, request):
        return web.Response(text="ok")

    async def version(self, request):
        return web.json_response({"major": "1", "minor": "29", "gitVersion": "v1.29.0-devspace-local",
                                  "platform": "linux/amd64"})

    async def api_versions(self, request):
        return web.json_response({"kind": "APIVersions", "versions": ["v1"]})

    async def api_groups(self, request):
        groups = [{"name": g, "versions": [{"groupVersion": f"{g}/v1", "version": "v1"}]} for g in GROUP_KINDS]
        return web.json_response({"kind": "APIGroupList", "groups": groups})

    async def dispatch_core(self, request):
        return await self._dispatch(request, "", request.match_info["version"])

    async def dispatch_group(self, request):
        return await self._dispatch(request, request.match_info["group"], request.match_info["version"])

    async def _dispatch(self, request, group, version):
        segs = [s for s in request.match_info["tail"].split("/") if s]
        api_version = version if not group else f"{group}/{version}"
        ns = name = sub = None
        if len(segs) >= 2 and segs[0] == "namespaces" and len(segs) >= 3:
            ns, resource = segs[1], segs[2]
            name = segs[3] if len(segs) > 3 else None
            sub = segs[4] if len(segs) > 4 else None
        else:
            resource = segs[0] if segs else ""
            name = segs[1] if len(segs) > 1 else None
            sub = segs[2] if len(segs) > 2 else None
        if group == "extensions":
            group = "apps" if resource in GROUP_KINDS["apps"] else "networking.k8s.io"
        try:
            if sub in ("exec", "attach") and resource == "pods":
                return await self.exec_ws(request, ns, name, sub)
            if sub == "portforward" and resource == "pods":
                return await self.portforward_ws(request, ns, name)
            if sub == "log" and resource == "pods":
                return await self.logs(request, ns, name)
            m = request.method
            if name is None:
                if m == "GET":
                    if request.query.get("watch") in ("1", "true"):
                        return await self.watch(request, group, resource, ns)
                    return self.list(request, group, resource, ns, api_version)
                if m == "POST":
                    body = await request.json()
                    if resource == "namespaces":
                        ns = ""
                    obj = self.store.create(group, resource, ns or body.get("metadata", {}).get("namespace") or "default",
                                            body, api_version)
                    return web.json_response(obj, status=201)
                if m == "DELETE":
                    for o in self.store.list(group, resource, ns, request.query.get("labelSelector", "")):
                        self._delete(group, resource, o["metadata"].get("namespace"), o["metadata"]["name"])
                    return web.json_response({"kind": "Status", "status": "Success"})
            else:
                if sub == "status" and m in ("PUT", "PATCH"):
                    body = await request.json()
                    o = self.store.update_status(group, resource, ns, name, body.get("status", {}))
                    if o is None:
                        raise ApiError(404, "NotFound", f'{resource} "{name}" not found')
                    return web.json_response(o)
                if m == "GET":
                    return web.json_response(self.store.get(group, resource, ns, name))
                if m == "PUT":
                    body = await request.json()
                    return web.json_response(self.store.replace(group, resource, ns, name, body))
                if m == "PATCH":
                    ct = request.content_type
                    if ct == "application/apply-patch+yaml":
                        manager = request.query.get("fieldManager")
                        if not manager:
                            raise ApiError(400, "BadRequest", "PATCH apply-patch+yaml requires fieldManager")
                        body = yaml.safe_load(await request.text())
                        obj, created = self.store.apply(group, resource, ns or "default", name, body, manager,
                                                        request.query.get("force") in ("true", "1"), api_version)
                        return web.json_response(obj, status=201 if created else 200)
                    if ct in ("application/merge-patch+json", "application/strategic-merge-patch+json",
                              "application/json"):
                        body = await request.json()
                        return web.json_response(self.store.patch(
                            group, resource, ns, name, body, strategic=ct == "application/strategic-merge-patch+json"))
                    raise ApiError(415, "UnsupportedMediaType", f"the body of the request was in an unknown format: {ct}")
                if m == "DELETE":
                    o = self._delete(group, resource, ns, name)
                    return web.json_response(o)
            return web.json_response({"kind": "Status", "status": "Failure", "message": "method not allowed",
                                      "code": 405}, status=405)
        except ApiError as e:
            return _err(e)
        except (ValueError, json.JSONDecodeError) as e:
            return _err(ApiError(400, "BadRequest", str(e)))

    def _delete(self, group, resource, ns, name):
        if resource == "pods":
            return self.store.mark_deleting(group, resource, ns, name)
        if resource == "persistentvolumeclaims":  # pvc-protection: finalized by the kubelet
            return self.store.delete_or_finalize(group, resource, ns, name)
        obj = self.store.get(group, resource, ns, name)
        if resource == "namespaces":
            for (g, r, n, nm), _ in list(self.store.objs.items()):
                if n == name and r not in CLUSTER_SCOPED:
                    if r == "pods":
                        self.store.mark_deleting(g, r, n, nm)
                    else:
                        try:
                            self.store.delete(g, r, n, nm)
                        except ApiError:
                            pass
        # cascade to owned objects (pods of deployments/statefulsets)
        for key, o in self.store.owned_by(obj["metadata"]["uid"]):
            g, r, n, nm = key
            if r == "pods":
                self.store.mark_deleting(g, r, n, nm)
            else:
                try:
                    self.store.delete(g, r, n, nm)
                except ApiError:
                    pass
        return self.store.delete(group, resource, ns, name)

    def list(self, request, group, resource, ns, api_version):
        field = None
        fs = request.query.get("fieldSelector", "")
        if fs:
            conds = [c.split("=", 1) for c in fs.split(",") if "=" in c]

            def field(o, conds=conds):
                for k, v in conds:
                    cur = o
                    for part in k.split("."):
                        cur = cur.get(part, {}) if isinstance(cur, dict) else {}
                    if str(cur) != v:
                        return False
                return True

        with self.store.lock:
            items = self.store.list(group, resource, ns, request.query.get("labelSelector", ""), field)
            rv = str(self.store.last_rv)
        kind = (items[0]["kind"] if items else resource[:1].upper() + resource[1:-1]) + "List"
        return web.json_response({"kind": kind, "apiVersion": api_version, "metadata": {"resourceVersion": rv},
                                  "items": items})

    @staticmethod
    def _field_filter(request):
        fs = request.query.get("fieldSelector", "")
        conds = [c.split("=", 1) for c in fs.split(",") if "=" in c]

        def match(o):
            for k, v in conds:
                cur = o
                for part in k.split("."):
                    cur = cur.get(part, {}) if isinstance(cur, dict) else {}
                if str(cur) != v:
                    return False
            return True

        return match

    # ------------------------------------------------------------------ watch

    async def watch(self, request, group, resource, ns):
        """?watch=1: newline-delimited WatchEvents, resumable from resourceVersion (410 when
        the backlog no longer reaches back that far), ended after timeoutSeconds."""
        reqs = parse_selector(request.query.get("labelSelector", ""))
        field = self._field_filter(request)
        timeout = float(request.query.get("timeoutSeconds", "1800") or 1800)
        rv = request.query.get("resourceVersion", "")
        loop = asyncio.get_running_loop()
        q = asyncio.Queue()

        def in_scope(key):
            return key[0] == group and key[1] == resource and (
                not ns or resource in CLUSTER_SCOPED or key[2] == ns)

        def listener(ev, key, obj):
            if in_scope(key):
                loop.call_soon_threadsafe(q.put_nowait, (ev, key, copy.deepcopy(obj)))

        def matches(o):
            return labels_match((o.get("metadata") or {}).get("labels"), reqs) and field(o)

        with self.store.lock:
            self.store.listeners.append(listener)
            if rv in ("", "0"):
                backlog = [("ADDED", None, o) for o in self.store.list(group, resource, ns)]
            else:
                try:
                    backlog = self.store.events_since(int(rv))
                except ValueError:
                    backlog = None
                if backlog is not None:
                    backlog = [(e, k, o) for (e, k, o) in backlog if in_scope(k)]
            current = {(o["metadata"].get("namespace", ""), o["metadata"]["name"])
                       for o in self.store.list(group, resource, ns) if matches(o)}
        resp = web.StreamResponse(headers={"Content-Type": "application/json"})
        resp.enable_chunked_encoding()
        await resp.prepare(request)
        visible = set(current) if rv not in ("", "0") else set()

        async def send(ev, obj):
            await resp.write((json.dumps({"type": ev, "object": obj}) + "\n").encode())

        async def emit(ev, obj):
            k = (obj["metadata"].get("namespace", ""), obj["metadata"]["name"])
            if ev == "DELETED":
                if k in visible or matches(obj):
                    visible.discard(k)
                    await send("DELETED", obj)
                return
            if matches(obj):
                await send("MODIFIED" if k in visible and ev != "ADDED" else "ADDED", obj)
                visible.add(k)
            elif k in visible:  # no longer selected
                visible.discard(k)
                await send("DELETED", obj)

        try:
            if backlog is None:
                await send("ERROR", {"kind": "Status", "apiVersion": "v1", "status": "Failure", "reason": "Expired",
                                     "code": 410, "message": f"too old resource version: {rv}"})
                return resp
            for ev, _, obj in backlog:
                await emit(ev, obj)
            deadline = time.monotonic() + timeout
            while True:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                try:
                    ev, _, obj = await asyncio.wait_for(q.get(), min(left, 0.25))
                except asyncio.TimeoutError:
                    # aiohttp does not cancel handlers when the client goes away: notice it here
                    tr = request.transport
                    if tr is None or tr.is_closing():
                        break
                    continue
                if rv not in ("", "0") and int(obj["metadata"].get("resourceVersion", "0") or 0) <= int(rv):
                    continue  # already replayed from the backlog
                await emit(ev, obj)
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            with self.store.lock:
                if listener in self.store.listeners:
                    self.store.listeners.remove(listener)
        try:
            await resp.write_eof()
        except ConnectionResetError:
            pass
        return resp

    # ------------------------------------------------------------------ logs

    async def logs(self, request, ns, name):
        self.store.get("", "pods", ns, name)
        rt, c = self.kubelet.container(ns, name, request.query.get("container"))
        if c is None:
            raise ApiError(400, "BadRequest", f'container "{request.query.get("container")}" is not valid for pod {name}')
        tail = int(request.query.get("tailLines", "-1") or -1)
        follow = request.query.get("follow") in ("true", "1")
        q = c.subscribe() if follow else None
        data = b""
        if os.path.exists(c.log_path):
            with open(c.log_path, "rb") as f:
                data = f.read()
        seen = len(data)
        if tail >= 0:
            lines = data.splitlines(keepends=True)
            data = b"".join(lines[-tail:]) if tail else b""
        if not follow:
            return web.Response(body=data, content_type="text/plain")
        resp = web.StreamResponse(headers={"Content-Type": "text/plain"})
        await resp.prepare(request)
        await resp.write(data)
        try:
            # stream new output as the container writes it (chunks already in `data` skipped)
            while (ns, name) in self.kubelet.pods:
                try:
                    off, chunk = await asyncio.wait_for(q.get(), 0.5)
                except asyncio.TimeoutError:
                    tr = request.transport
                    if tr is None or tr.is_closing():  # follower went away
                        break
                    continue
                if off is None:
                    continue  # process ended; a restarted container keeps appending
                end = off + len(chunk)
                if end <= seen:
                    continue
                if off < seen:
                    chunk = chunk[seen - off:]
                seen = end
                await resp.write(chunk)
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            c.unsubscribe(q)
        try:
            await resp.write_eof()
        except ConnectionResetError:
            pass
        return resp

    # ------------------------------------------------------------------ exec / attach

    async def exec_ws(self, request, ns, name, kind):
        pod = self.store.get("", "pods", ns, name)
        rt, c = self.kubelet.container(ns, name, request.query.get("container"))
        if c is None or "running" not in (c.state or {}):
            raise ApiError(400, "BadRequest", f"container not found or not running in pod {name}")
        ws = web.WebSocketResponse(protocols=("v5.channel.k8s.io", "v4.channel.k8s.io", "channel.k8s.io"),
                                   max_msg_size=0)
        await ws.prepare(request)
        tty = request.query.get("tty") in ("true", "1")
        if kind == "attach":
            await self._attach(ws, c)
            return ws
        cmd = self.kubelet.map_argv(c, request.query.getall("command", []))
        env = self.kubelet._env(rt, c)
        cwd = self.kubelet.workdir(c)
        os.makedirs(cwd, exist_ok=True)
        master = None
        try:
            if tty:
                master, slave = pty.openpty()
                proc = await asyncio.create_subprocess_exec(*cmd, cwd=cwd, env=env, stdin=slave, stdout=slave,
                                                            stderr=slave, start_new_session=True)
                os.close(slave)
            else:
                proc = await asyncio.create_subprocess_exec(*cmd, cwd=cwd, env=env, stdin=asyncio.subprocess.PIPE,
                                                            stdout=asyncio.subprocess.PIPE,
                                                            stderr=asyncio.subprocess.PIPE, start_new_session=True)
        except (FileNotFoundError, PermissionError) as e:
            await ws.send_bytes(b"\x03" + json.dumps({"status": "Failure", "message": str(e), "reason": "InternalError"}).encode())
            await ws.close()
            return ws
        loop = asyncio.get_running_loop()
        c.exec_procs.add(proc)

        async def pump(reader, ch):
            while True:
                data = await reader.read(65536)
                if not data:
                    break
                await ws.send_bytes(bytes([ch]) + data)

        tasks = []
        if tty:
            q = asyncio.Queue()

            def on_readable():
                try:
                    data = os.read(master, 65536)
                except OSError:
                    data = b""
                if not data:
                    try:
                        loop.remove_reader(master)
                    except Exception:
                        pass
                q.put_nowait(data)

            loop.add_reader(master, on_readable)

            async def pump_pty():
                while True:
                    try:
                        data = await q.get()
                    except Exception:
                        break
                    if not data:
                        break
                    await ws.send_bytes(b"\x01" + data)

            tasks.append(asyncio.create_task(pump_pty()))
        else:
            tasks.append(asyncio.create_task(pump(proc.stdout, 1)))
            tasks.append(asyncio.create_task(pump(proc.stderr, 2)))

        async def read_ws():
            async for msg in ws:
                if msg.type != WSMsgType.BINARY or not msg.data:
                    continue
                ch, data = msg.data[0], msg.data[1:]
                if ch == 255 and ws.ws_protocol == "v5.channel.k8s.io":
                    # v5 CLOSE signal: half-close the named stream (only stdin is writable)
                    if data[:1] == b"\x00" and not tty and proc.stdin and not proc.stdin.is_closing():
                        proc.stdin.close()
                    continue
                if ch == 0:
                    if tty:
                        os.write(master, data)
                    elif proc.stdin and not proc.stdin.is_closing():
                        try:
                            proc.stdin.write(data)
                            await proc.stdin.drain()
                        except (ConnectionResetError, BrokenPipeError):
                            pass
                elif ch == 4 and tty:
                    try:
                        sz = json.loads(data.decode())
                        fcntl.ioctl(master, termios.TIOCSWINSZ, struct.pack("HHHH", sz["Height"], sz["Width"], 0, 0))
                    except Exception:
                        pass
            # client went away: stop the process
            if proc.returncode is None:
                try:
                    os.killpg(proc.pid, 9)
                except ProcessLookupError:
                    pass

        reader = asyncio.create_task(read_ws())
        try:
            code = await proc.wait()
            c.exec_procs.discard(proc)
            if tty:
                try:
                    await asyncio.sleep(0.05)
                    loop.remove_reader(master)
                except Exception:
                    pass
                try:
                    while True:
                        rest = os.read(master, 65536)
                        if not rest:
                            break
                        await ws.send_bytes(b"\x01" + rest)
                except OSError:
                    pass
                q.put_nowait(b"")
            await asyncio.gather(*tasks, return_exceptions=True)
            if not ws.closed:
                await ws.send_bytes(b"\x03" + json.dumps(_exit_status(code)).encode())
                await ws.close()
            reader.cancel()
            if master is not None:
                try:
                    os.close(master)
                except OSError:
                    pass
        finally:
            # also when the handler is cancelled (cluster shutdown): the subprocess transport is
            # closed while the loop still runs, never by the GC after the loop has closed
            c.exec_procs.discard(proc)
            reader.cancel()
            for t in tasks:
                t.cancel()
            close_proc(proc)
        return ws

    async def _attach(self, ws, c):
        # output produced after the attach, streamed as the pump reads it from the container
        q = c.subscribe()

        async def drain():
            async for _ in ws:
                pass

        reader = asyncio.create_task(drain())
        try:
            while not ws.closed and c.proc is not None:
                try:
                    off, chunk = await asyncio.wait_for(q.get(), 0.5)
                except asyncio.TimeoutError:
                    continue
                if off is None:
                    break  # the attached process exited
                await ws.send_bytes(b"\x01" + chunk)
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            c.unsubscribe(q)
        if not ws.closed:
            await ws.send_bytes(b"\x03" + json.dumps(_exit_status(0)).encode())
            await ws.close()
        reader.cancel()

    # ------------------------------------------------------------------ port-forward

    @staticmethod
    def _refused_text(name, port, e):
        # the kubelet's wording (CRI streaming server): clients key on "connection refused"
        if isinstance(e, LookupError):
            return f"error forwarding port {port} to pod {name}, uid : {e.args[0]}"
        why = "connect: connection refused" if isinstance(e, ConnectionRefusedError) or "111" in str(e) else str(e)
        return (f"error forwarding port {port} to pod {name}, uid : failed to connect to localhost:{port} inside "
                f"namespace: dial tcp4 127.0.0.1:{port}: {why}")

    async def portforward_ws(self, request, ns, name):
        uid = self.store.get("", "pods", ns, name)["metadata"].get("uid")
        served = ((spdy.PROTOCOL,) if self.portforward_tunnel else ()) + ("v4.channel.k8s.io", "portforward.k8s.io")
        offered = [p.strip() for p in request.headers.get("Sec-WebSocket-Protocol", "").split(",") if p.strip()]
        if offered and not set(offered) & set(served):
            # the API server's stream negotiation refuses the upgrade (wsstream handshake)
            raise web.HTTPBadRequest(text=f"requested protocol(s) are not supported: {offered}; "
                                          f"supports {list(served)}")
        ws = web.WebSocketResponse(protocols=served, max_msg_size=0)
        await ws.prepare(request)
        if ws.ws_protocol == spdy.PROTOCOL:
            # Kubernetes >= 1.30: one tunnel, a stream pair per forwarded connection
            self.portforward_tunnels += 1

            async def dial(port):
                # the tunnel outlives its pod (pods share the host network here, so a port of
                # the pod's replacement would answer): a stream of a deleted pod fails as the
                # kubelet's does once the pod's sandbox is gone
                cur = self.store.try_get("", "pods", ns, name)
                if cur is None or cur["metadata"].get("uid") != uid:
                    raise LookupError(f'failed to find sandbox "{uid}" in store: not found')
                return await asyncio.open_connection("127.0.0.1", port)

            tunnel = spdy.Tunnel(ws, dial, lambda port, e: self._refused_text(name, port, e))
            self.open_tunnels.add(ws)
            try:
                await tunnel.run()
            finally:
                self.open_tunnels.discard(ws)
                self.tunnel_pings_answered += tunnel.pings_answered
            return ws
        port = int(request.query.get("ports", "0").split(",")[0])
        hdr = struct.pack("<H", port)
        await ws.send_bytes(b"\x00" + hdr)
        await ws.send_bytes(b"\x01" + hdr)
        try:
            reader, writer = await asyncio.open_connection("127.0.0.1", port)
        except OSError as e:
            await ws.send_bytes(b"\x01" + self._refused_text(name, port, e).encode())
            await ws.close()
            return ws

        async def up():
            try:
                while True:
                    data = await reader.read(65536)
                    if not data:
                        break
                    await ws.send_bytes(b"\x00" + data)
            except (ConnectionError, asyncio.CancelledError):  # either side went away
                pass
            await ws.close()

        t = asyncio.create_task(up())
        try:
            async for msg in ws:
                if msg.type == WSMsgType.BINARY and msg.data and msg.data[0] == 0:
                    writer.write(msg.data[1:])
                    await writer.drain()
        except ConnectionError:  # the pod's server closed the connection (e.g. a restart)
            pass
        writer.close()
        t.cancel()
        return ws
