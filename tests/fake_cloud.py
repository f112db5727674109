"""Fake DevSpace-cloud GraphQL provider for CLI tests (the real service is offline).

Answers the queries/mutations issued by src/cloud/cloud.cc (reference cloud/get.go,
create.go, delete.go, registry.go) from an in-memory model. Spaces point at a given Kubernetes
API server (the local cluster), so `devspace create space` + `devspace deploy` work end to end.
"""

import asyncio
import base64
import json
import threading

from aiohttp import web


def make_token(account="tester"):
    def b64(d):
        return base64.urlsafe_b64encode(json.dumps(d).encode()).decode().rstrip("=")

    return f"{b64({'alg': 'none'})}.{b64({'sub': account})}.sig"


class FakeCloud:
    def __init__(self, kube_server, registry="registry.fake.cloud"):
        self.kube_server = kube_server
        self.registry = registry
        self.spaces = {}
        self.projects = {}
        self.clusters = {1: "public-mi355x"}
        self.next_id = 100
        self.requests = []
        self.port = None
        self._loop = None
        self._thread = None
        self._ready = threading.Event()

    # ---------------------------------------------------------------- model

    def _space_json(self, s):
        return {
            "id": s["id"],
            "name": s["name"],
            "created_at": "2026-01-01T00:00:00Z",
            "kubeContextBykubeContextId": {
                "namespace": s["namespace"],
                "service_account_token": "fake-sa-token",
                "clusterByclusterId": {"ca_cert": "", "server": self.kube_server},
                "kubeContextDomainsBykubeContextId": [{"url": s["name"] + ".fake.cloud"}],
            },
        }

    def _handle(self, query, variables):
        q = " ".join(query.split())
        if "manager_createProject" in q:
            pid = self.next_id
            self.next_id += 1
            self.projects[pid] = variables["projectName"]
            return {"manager_createProject": {"ProjectID": pid}}
        if "manager_createSpace" in q:
            sid = self.next_id
            self.next_id += 1
            name = variables["spaceName"]
            self.spaces[sid] = {"id": sid, "name": name, "namespace": "space-" + name.lower()}
            return {"manager_createSpace": {"SpaceID": sid}}
        if "manager_deleteSpace" in q:
            self.spaces.pop(variables["spaceID"], None)
            return {"manager_deleteSpace": True}
        if "space_by_pk" in q:
            s = self.spaces.get(variables["ID"])
            return {"space_by_pk": self._space_json(s) if s else None}
        if "space(where" in q:
            return {"space": [self._space_json(s) for s in self.spaces.values() if s["name"] == variables["name"]]}
        if "space {" in q or "space{" in q:
            return {"space": [self._space_json(s) for s in self.spaces.values()]}
        if "project" in q:
            return {"project": [{"id": k, "name": v} for k, v in self.projects.items()]}
        if "cluster" in q:
            return {"cluster": [{"id": k, "name": v} for k, v in self.clusters.items()]}
        if "image_registry" in q:
            return {"image_registry": [{"url": self.registry}]}
        raise ValueError("unsupported query: " + q)

    # ---------------------------------------------------------------- server

    async def _graphql(self, request):
        body = await request.json()
        self.requests.append((request.headers.get("Authorization", ""), body.get("query", "")))
        if not request.headers.get("Authorization", "").startswith("Bearer ") or \
                request.headers["Authorization"] == "Bearer ":
            return web.json_response({"errors": [{"message": "not authenticated"}]})
        try:
            return web.json_response({"data": self._handle(body["query"], body.get("variables") or {})})
        except Exception as e:  # noqa: BLE001
            return web.json_response({"errors": [{"message": str(e)}]})

    def start(self):
        def run():
            self._loop = asyncio.new_event_loop()
            app = web.Application()
            app.router.add_post("/graphql", self._graphql)
            runner = web.AppRunner(app, access_log=None)
            self._loop.run_until_complete(runner.setup())
            site = web.TCPSite(runner, "127.0.0.1", 0)
            self._loop.run_until_complete(site.start())
            self.port = site._server.sockets[0].getsockname()[1]
            self._runner = runner
            self._ready.set()
            self._loop.run_forever()

        self._thread = threading.Thread(target=run, daemon=True)
        self._thread.start()
        self._ready.wait(10)
        return self

    def stop(self):
        if self._loop:
            fut = asyncio.run_coroutine_threadsafe(self._runner.cleanup(), self._loop)
            fut.result(10)
            self._loop.call_soon_threadsafe(self._loop.stop)
            self._thread.join(5)

    @property
    def url(self):
        return f"http://127.0.0.1:{self.port}"
