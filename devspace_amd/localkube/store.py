"""In-memory Kubernetes object store used by the local cluster's API server."""

from __future__ import annotations

import copy
import datetime
import itertools
import json
import os
import re
import threading
import time
import uuid

CLUSTER_SCOPED = {"namespaces", "nodes", "persistentvolumes", "clusterroles", "clusterrolebindings", "storageclasses",
                  "customresourcedefinitions", "priorityclasses"}

KIND_OF = {
    "pods": "Pod", "services": "Service", "secrets": "Secret", "configmaps": "ConfigMap", "events": "Event",
    "namespaces": "Namespace", "nodes": "Node", "serviceaccounts": "ServiceAccount",
    "persistentvolumeclaims": "PersistentVolumeClaim", "persistentvolumes": "PersistentVolume",
    "endpoints": "Endpoints", "deployments": "Deployment", "statefulsets": "StatefulSet",
    "replicasets": "ReplicaSet", "daemonsets": "DaemonSet", "jobs": "Job",
    "horizontalpodautoscalers": "HorizontalPodAutoscaler", "roles": "Role", "rolebindings": "RoleBinding",
    "clusterroles": "ClusterRole", "clusterrolebindings": "ClusterRoleBinding", "ingresses": "Ingress",
}


def now_rfc3339():
    return datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


class ApiError(Exception):
    def __init__(self, code, reason, message):
        super().__init__(message)
        self.code = code
        self.reason = reason
        self.message = message

    def status(self):
        return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure", "message": self.message,
                "reason": self.reason, "code": self.code}


def parse_selector(sel: str):
    """Equality/inequality/set-based label selectors: a=b, a==b, a!=b, a in (x,y), a notin (x), a, !a."""
    reqs = []
    if not sel:
        return reqs
    parts = re.findall(r"[^,(]+(?:\([^)]*\))?", sel)
    for p in parts:
        p = p.strip()
        if not p:
            continue
        m = re.match(r"^([^\s!=]+)\s+(in|notin)\s+\(([^)]*)\)$", p)
        if m:
            reqs.append((m.group(1), m.group(2), {v.strip() for v in m.group(3).split(",")}))
        elif "!=" in p:
            k, v = p.split("!=", 1)
            reqs.append((k.strip(), "!=", v.strip()))
        elif "==" in p:
            k, v = p.split("==", 1)
            reqs.append((k.strip(), "=", v.strip()))
        elif "=" in p:
            k, v = p.split("=", 1)
            reqs.append((k.strip(), "=", v.strip()))
        elif p.startswith("!"):
            reqs.append((p[1:].strip(), "!exists", None))
        else:
            reqs.append((p, "exists", None))
    return reqs


def labels_match(labels, reqs):
    labels = labels or {}
    for k, op, v in reqs:
        if op == "=" and labels.get(k) != v:
            return False
        if op == "!=" and labels.get(k) == v:
            return False
        if op == "in" and labels.get(k) not in v:
            return False
        if op == "notin" and labels.get(k) in v:
            return False
        if op == "exists" and k not in labels:
            return False
        if op == "!exists" and k in labels:
            return False
    return True


def merge_patch(target, patch):
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


class _Tracer:
    """LOCALKUBE_TRACE=<file>: one JSON line per object event with a ms wall-clock timestamp
    (where a cluster-side wait goes: pod created -> started -> ready -> workload ready)."""

    def __init__(self, path):
        self.f = open(path, "a", buffering=1)

    def __call__(self, ev, key, obj):
        if key[1] in ("events", "secrets", "configmaps", "serviceaccounts"):
            return
        st = obj.get("status") or {}
        rec = {"t_ms": round(time.time() * 1000.0, 2), "ev": ev, "res": key[1], "name": key[3],
               "phase": st.get("phase"), "ready": st.get("readyReplicas")}
        self.f.write(json.dumps(rec) + "\n")


class Store:
    def __init__(self):
        self.lock = threading.RLock()
        self.objs = {}  # (group, resource, ns, name) -> obj
        self.rv = itertools.count(1)
        self.listeners = []  # callables(event, key, obj)
        # callables(key) run on changes a controller must act on (creates, spec replaces,
        # deletes) but not on status writes, so a controller's own status updates never
        # re-trigger it
        self.wakers = []
        trace = os.environ.get("LOCALKUBE_TRACE")
        if trace:
            self.listeners.append(_Tracer(trace))

    def _key(self, group, resource, ns, name):
        return (group, resource, "" if resource in CLUSTER_SCOPED else (ns or "default"), name)

    def _wake(self, key):
        if key[1] == "events":
            return
        for fn in list(self.wakers):
            try:
                fn(key)
            except Exception:  # pragma: no cover
                pass

    def _notify(self, ev, key, obj):
        for fn in list(self.listeners):
            try:
                fn(ev, key, obj)
            except Exception:  # pragma: no cover - listener bugs must not break the API
                pass

    def get(self, group, resource, ns, name):
        with self.lock:
            o = self.objs.get(self._key(group, resource, ns, name))
            if o is None:
                raise ApiError(404, "NotFound", f'{resource} "{name}" not found')
            return copy.deepcopy(o)

    def try_get(self, group, resource, ns, name):
        try:
            return self.get(group, resource, ns, name)
        except ApiError:
            return None

    def list(self, group, resource, ns=None, selector="", field=None):
        reqs = parse_selector(selector)
        with self.lock:
            out = []
            for (g, r, n, _), o in self.objs.items():
                if g != group or r != resource:
                    continue
                if ns and resource not in CLUSTER_SCOPED and n != ns:
                    continue
                if not labels_match(o.get("metadata", {}).get("labels"), reqs):
                    continue
                if field and not field(o):
                    continue
                out.append(copy.deepcopy(o))
            out.sort(key=lambda o: o["metadata"].get("creationTimestamp", ""))
            return out

    def create(self, group, resource, ns, obj, api_version=None):
        with self.lock:
            md = obj.setdefault("metadata", {})
            if not md.get("name") and md.get("generateName"):
                md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
            name = md.get("name")
            if not name:
                raise ApiError(422, "Invalid", "metadata.name: Required value")
            key = self._key(group, resource, ns, name)
            if key in self.objs:
                raise ApiError(409, "AlreadyExists", f'{resource} "{name}" already exists')
            if resource not in CLUSTER_SCOPED:
                md["namespace"] = key[2]
                if resource != "namespaces" and not self.objs.get(("", "namespaces", "", key[2])) and key[2] != "default":
                    raise ApiError(404, "NotFound", f'namespaces "{key[2]}" not found')
            md["uid"] = str(uuid.uuid4())
            md["resourceVersion"] = str(next(self.rv))
            md["creationTimestamp"] = now_rfc3339()
            md.setdefault("generation", 1)
            obj.setdefault("kind", KIND_OF.get(resource, resource[:-1].capitalize()))
            if api_version:
                obj.setdefault("apiVersion", api_version)
            self.objs[key] = obj
            self._notify("ADDED", key, obj)
            self._wake(key)
            return copy.deepcopy(obj)

    def replace(self, group, resource, ns, name, obj):
        with self.lock:
            key = self._key(group, resource, ns, name)
            old = self.objs.get(key)
            if old is None:
                raise ApiError(404, "NotFound", f'{resource} "{name}" not found')
            md = obj.setdefault("metadata", {})
            rv = md.get("resourceVersion")
            if rv and rv != old["metadata"]["resourceVersion"]:
                raise ApiError(409, "Conflict", f"Operation cannot be fulfilled on {resource} \"{name}\": the object has been modified")
            for k in ("uid", "creationTimestamp", "namespace", "name"):
                if k in old["metadata"]:
                    md[k] = old["metadata"][k]
            if "status" not in obj and "status" in old:
                obj["status"] = old["status"]
            if obj.get("spec") != old.get("spec"):
                md["generation"] = old["metadata"].get("generation", 1) + 1
            else:
                md["generation"] = old["metadata"].get("generation", 1)
            if old["metadata"].get("deletionTimestamp"):
                md["deletionTimestamp"] = old["metadata"]["deletionTimestamp"]
            md["resourceVersion"] = str(next(self.rv))
            obj.setdefault("kind", old.get("kind"))
            obj.setdefault("apiVersion", old.get("apiVersion"))
            self.objs[key] = obj
            self._notify("MODIFIED", key, obj)
            self._wake(key)
            return copy.deepcopy(obj)

    def update_status(self, group, resource, ns, name, status):
        with self.lock:
            key = self._key(group, resource, ns, name)
            o = self.objs.get(key)
            if o is None:
                return None
            o["status"] = status
            o["metadata"]["resourceVersion"] = str(next(self.rv))
            self._notify("MODIFIED", key, o)
            return copy.deepcopy(o)

    def mutate(self, group, resource, ns, name, fn):
        with self.lock:
            key = self._key(group, resource, ns, name)
            o = self.objs.get(key)
            if o is None:
                return None
            fn(o)
            o["metadata"]["resourceVersion"] = str(next(self.rv))
            self._notify("MODIFIED", key, o)
            return copy.deepcopy(o)

    def patch(self, group, resource, ns, name, patch):
        with self.lock:
            key = self._key(group, resource, ns, name)
            old = self.objs.get(key)
            if old is None:
                raise ApiError(404, "NotFound", f'{resource} "{name}" not found')
            new = merge_patch(old, patch)
            new["metadata"]["resourceVersion"] = old["metadata"]["resourceVersion"]
            return self.replace(group, resource, ns, name, new)

    def delete(self, group, resource, ns, name):
        with self.lock:
            key = self._key(group, resource, ns, name)
            o = self.objs.pop(key, None)
            if o is None:
                raise ApiError(404, "NotFound", f'{resource} "{name}" not found')
            self._notify("DELETED", key, o)
            self._wake(key)
            return o

    def mark_deleting(self, group, resource, ns, name):
        """Graceful deletion (pods): set deletionTimestamp, the kubelet finishes it."""
        with self.lock:
            key = self._key(group, resource, ns, name)
            o = self.objs.get(key)
            if o is None:
                raise ApiError(404, "NotFound", f'{resource} "{name}" not found')
            o["metadata"].setdefault("deletionTimestamp", now_rfc3339())
            o["metadata"]["resourceVersion"] = str(next(self.rv))
            self._notify("MODIFIED", key, o)
            self._wake(key)
            return copy.deepcopy(o)

    def owned_by(self, uid):
        with self.lock:
            return [
                (k, copy.deepcopy(o))
                for k, o in self.objs.items()
                if any(r.get("uid") == uid for r in o.get("metadata", {}).get("ownerReferences", []) or [])
            ]
