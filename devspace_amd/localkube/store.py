"""In-memory Kubernetes object store used by the local cluster's API server."""

from __future__ import annotations

import collections
import copy
import datetime
import itertools
import json
import random
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


def strategic_merge(target, patch):
    """Strategic-merge-patch subset: like a JSON merge patch, but lists of named objects
    (containers, env, volumes, ports with names) merge element-wise by `name`."""
    if isinstance(patch, list) and isinstance(target, list) and patch and \
            all(isinstance(x, dict) and "name" in x for x in patch + target):
        out = [copy.deepcopy(x) for x in target]
        idx = {x["name"]: i for i, x in enumerate(out)}
        for x in patch:
            if x.get("$patch") == "delete":
                if x["name"] in idx:
                    out[idx[x["name"]]] = None
                continue
            if x["name"] in idx:
                out[idx[x["name"]]] = strategic_merge(out[idx[x["name"]]], x)
            else:
                out.append(copy.deepcopy(x))
        return [x for x in out if x is not None]
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = strategic_merge(out.get(k), v)
    return out


# ---------------------------------------------------------------- server-side apply

_SSA_SKIP = {("apiVersion",), ("kind",), ("metadata", "name"), ("metadata", "namespace")}


def field_paths(obj, prefix=()):
    """Leaf field paths of an applied configuration (lists are atomic leaves)."""
    out = set()
    if isinstance(obj, dict) and obj:
        for k, v in obj.items():
            out |= field_paths(v, prefix + (k,))
    elif prefix and prefix not in _SSA_SKIP:
        out.add(prefix)
    return out


def to_fields_v1(paths):
    root = {}
    for p in sorted(paths):
        cur = root
        for part in p:
            cur = cur.setdefault("f:" + part, {})
    return root


def from_fields_v1(fv, prefix=()):
    out = set()
    for k, v in (fv or {}).items():
        if not k.startswith("f:"):
            continue
        p = prefix + (k[2:],)
        if v:
            out |= from_fields_v1(v, p)
        else:
            out.add(p)
    return out


def _get_path(obj, path):
    cur = obj
    for part in path:
        if not isinstance(cur, dict) or part not in cur:
            return None, False
        cur = cur[part]
    return cur, True


def _del_path(obj, path):
    cur = obj
    for part in path[:-1]:
        if not isinstance(cur, dict) or part not in cur:
            return
        cur = cur[part]
    if isinstance(cur, dict):
        cur.pop(path[-1], None)


def _deep_merge(target, patch):
    if not isinstance(patch, dict) or not isinstance(target, dict):
        return copy.deepcopy(patch)
    out = dict(target)
    for k, v in patch.items():
        out[k] = _deep_merge(out.get(k), v)
    return out


# ---------------------------------------------------------------- immutable fields

_STS_MUTABLE = {"replicas", "template", "updateStrategy", "persistentVolumeClaimRetentionPolicy", "minReadySeconds",
                "ordinals", "revisionHistoryLimit"}


def validate_update(resource, name, old, new):
    """422 for changes a real API server refuses (the fields that made round-1's PUT-replace
    apply delete PVCs on real clusters)."""
    os_, ns_ = old.get("spec") or {}, new.get("spec") or {}

    def invalid(msg):
        kind = KIND_OF.get(resource, resource)
        raise ApiError(422, "Invalid", f'{kind} "{name}" is invalid: {msg}')

    if resource == "persistentvolumeclaims":
        strip = lambda sp: {k: v for k, v in sp.items() if k not in ("resources", "volumeAttributesClassName")}
        if strip(os_) != strip(ns_):
            invalid("spec: Forbidden: spec is immutable after creation except resources.requests and "
                    "volumeAttributesClassName for bound claims")
    elif resource == "services":
        oip, nip = os_.get("clusterIP"), ns_.get("clusterIP")
        if oip and nip and nip != oip:
            invalid(f'spec.clusterIP: Invalid value: "{nip}": field is immutable')
        if oip and not nip and os_.get("type", "ClusterIP") == ns_.get("type", "ClusterIP"):
            invalid('spec.clusterIP: Invalid value: "": field is immutable')
    elif resource in ("deployments", "replicasets", "daemonsets", "statefulsets"):
        if "selector" in os_ and ns_.get("selector") != os_.get("selector"):
            invalid(f"spec.selector: Invalid value: {json.dumps(ns_.get('selector'))}: field is immutable")
        if resource == "statefulsets":
            a = {k: v for k, v in os_.items() if k not in _STS_MUTABLE}
            b = {k: v for k, v in ns_.items() if k not in _STS_MUTABLE}
            if a != b:
                invalid("spec: Forbidden: updates to statefulset spec for fields other than 'replicas', 'ordinals', "
                        "'template', 'updateStrategy', 'persistentVolumeClaimRetentionPolicy' and 'minReadySeconds' "
                        "are forbidden")
    elif resource == "jobs":
        for f in ("selector", "template"):
            if f in os_ and ns_.get(f) != os_.get(f):
                invalid(f"spec.{f}: Invalid value: field is immutable")


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
        self.last_rv = 0
        self.listeners = []  # callables(event, key, obj)
        # watch backlog: (rv, event, key, obj) for ?watch=1&resourceVersion=N resumption
        self.history = collections.deque(maxlen=50000)
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

    def next_rv(self):
        self.last_rv = next(self.rv)
        return str(self.last_rv)

    def events_since(self, rv):
        """Events after resourceVersion rv, or None if rv predates the backlog (410 Gone)."""
        with self.lock:
            if len(self.history) == self.history.maxlen and rv < self.history[0][0] - 1:
                return None
            return [(e, k, copy.deepcopy(o)) for (r, e, k, o) in self.history if r > rv]

    def _notify(self, ev, key, obj):
        try:
            self.history.append((int(obj["metadata"]["resourceVersion"]), ev, key, copy.deepcopy(obj)))
        except (KeyError, TypeError, ValueError):
            pass
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
            md["resourceVersion"] = self.next_rv()
            md["creationTimestamp"] = now_rfc3339()
            md.setdefault("generation", 1)
            if resource == "persistentvolumeclaims":
                fins = md.setdefault("finalizers", [])
                if "kubernetes.io/pvc-protection" not in fins:
                    fins.append("kubernetes.io/pvc-protection")
            if resource == "services":
                spec = obj.setdefault("spec", {})
                if not spec.get("clusterIP"):
                    spec["clusterIP"] = f"10.96.{random.randint(0, 255)}.{random.randint(1, 254)}"
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
            if "finalizers" not in md and old["metadata"].get("finalizers"):
                md["finalizers"] = old["metadata"]["finalizers"]
            if "managedFields" not in md and old["metadata"].get("managedFields"):
                md["managedFields"] = old["metadata"]["managedFields"]
            validate_update(resource, name, old, obj)
            if "status" not in obj and "status" in old:
                obj["status"] = old["status"]
            if obj.get("spec") != old.get("spec"):
                md["generation"] = old["metadata"].get("generation", 1) + 1
            else:
                md["generation"] = old["metadata"].get("generation", 1)
            if old["metadata"].get("deletionTimestamp"):
                md["deletionTimestamp"] = old["metadata"]["deletionTimestamp"]
            md["resourceVersion"] = self.next_rv()
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
            o["metadata"]["resourceVersion"] = self.next_rv()
            self._notify("MODIFIED", key, o)
            return copy.deepcopy(o)

    def mutate(self, group, resource, ns, name, fn):
        with self.lock:
            key = self._key(group, resource, ns, name)
            o = self.objs.get(key)
            if o is None:
                return None
            fn(o)
            o["metadata"]["resourceVersion"] = self.next_rv()
            self._notify("MODIFIED", key, o)
            return copy.deepcopy(o)

    def patch(self, group, resource, ns, name, patch, strategic=False):
        with self.lock:
            key = self._key(group, resource, ns, name)
            old = self.objs.get(key)
            if old is None:
                raise ApiError(404, "NotFound", f'{resource} "{name}" not found')
            new = (strategic_merge if strategic else merge_patch)(old, patch)
            new["metadata"]["resourceVersion"] = old["metadata"]["resourceVersion"]
            return self.replace(group, resource, ns, name, new)

    def apply(self, group, resource, ns, name, cfg, manager, force, api_version=None):
        """Server-side apply: `manager` owns exactly the fields of its last applied
        configuration; fields it stops applying are removed unless another manager owns them;
        fields owned by other appliers conflict (409) unless force. Returns (obj, created)."""
        if not isinstance(cfg, dict):
            raise ApiError(400, "BadRequest", "apply patch must be an object")
        cfg = copy.deepcopy(cfg)
        cfg.pop("status", None)
        md = cfg.setdefault("metadata", {})
        if md.get("name") and md["name"] != name:
            raise ApiError(400, "BadRequest", "the name of the object does not match the name on the URL")
        md["name"] = name
        for k in ("resourceVersion", "uid", "managedFields", "creationTimestamp"):
            md.pop(k, None)
        paths = field_paths(cfg)
        entry = {"manager": manager, "operation": "Apply", "apiVersion": cfg.get("apiVersion") or api_version,
                 "time": now_rfc3339(), "fieldsType": "FieldsV1", "fieldsV1": to_fields_v1(paths)}
        with self.lock:
            key = self._key(group, resource, ns, name)
            old = self.objs.get(key)
            if old is None:
                md["managedFields"] = [entry]
                return self.create(group, resource, ns, cfg, api_version), True
            managed = copy.deepcopy(old["metadata"].get("managedFields") or [])
            mine = next((m for m in managed if m["manager"] == manager and m.get("operation") == "Apply"), None)
            prev = from_fields_v1(mine["fieldsV1"]) if mine else set()
            others = [m for m in managed if m is not mine]
            conflicts = []
            for m in others:
                if m.get("operation") != "Apply":
                    continue
                theirs = from_fields_v1(m.get("fieldsV1"))
                for p in paths & theirs:
                    if _get_path(old, p)[0] != _get_path(cfg, p)[0]:
                        conflicts.append(f'conflict with "{m["manager"]}": .{".".join(p)}')
            if conflicts and not force:
                raise ApiError(409, "Conflict", "Apply failed with %d conflicts: %s" % (len(conflicts),
                                                                                    "; ".join(conflicts)))
            base = copy.deepcopy(old)
            base.pop("status", None)
            new = _deep_merge(base, cfg)
            owned_by_others = set()
            for m in others:
                owned_by_others |= from_fields_v1(m.get("fieldsV1"))
            for p in prev - paths:
                if p not in owned_by_others:
                    _del_path(new, p)
            new_managed = []
            for m in others:
                if force and m.get("operation") == "Apply":
                    m = dict(m, fieldsV1=to_fields_v1(from_fields_v1(m.get("fieldsV1")) - paths))
                new_managed.append(m)
            new_managed.append(entry)
            new["metadata"]["managedFields"] = new_managed
            new["metadata"]["resourceVersion"] = old["metadata"]["resourceVersion"]
            if "status" in old:
                new["status"] = old["status"]
            return self.replace(group, resource, ns, name, new), False

    def delete(self, group, resource, ns, name):
        with self.lock:
            key = self._key(group, resource, ns, name)
            o = self.objs.pop(key, None)
            if o is None:
                raise ApiError(404, "NotFound", f'{resource} "{name}" not found')
            o["metadata"]["resourceVersion"] = self.next_rv()
            self._notify("DELETED", key, o)
            self._wake(key)
            return o

    def delete_or_finalize(self, group, resource, ns, name):
        """DELETE of an object carrying finalizers only sets deletionTimestamp (the owning
        controller removes it later, e.g. pvc-protection once no pod uses the claim)."""
        with self.lock:
            o = self.objs.get(self._key(group, resource, ns, name))
            if o is None:
                raise ApiError(404, "NotFound", f'{resource} "{name}" not found')
            if o["metadata"].get("finalizers"):
                return self.mark_deleting(group, resource, ns, name)
            return self.delete(group, resource, ns, name)

    def mark_deleting(self, group, resource, ns, name):
        """Graceful deletion (pods): set deletionTimestamp, the kubelet finishes it."""
        with self.lock:
            key = self._key(group, resource, ns, name)
            o = self.objs.get(key)
            if o is None:
                raise ApiError(404, "NotFound", f'{resource} "{name}" not found')
            o["metadata"].setdefault("deletionTimestamp", now_rfc3339())
            o["metadata"]["resourceVersion"] = self.next_rv()
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
