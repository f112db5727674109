"""Process kubelet + workload controllers for the local cluster.

Pods are host processes: each container gets a rootfs directory (copied from the local image
store), runs with its working directory mapped under that root, logs to a file, and is
restarted per restartPolicy with CrashLoopBackOff semantics. `amd.com/gpu` requests are
scheduled against the node's GPUs and exposed via HIP_VISIBLE_DEVICES (one process per GPU
inside the pod is the workload's business — see devspace_amd.runner).
"""

from __future__ import annotations

import asyncio
import hashlib
import json
import os
import shutil
import signal
import sys
import time

from .store import ApiError, now_rfc3339

LOCAL_ROOTS_ANNOTATION = "devspace.sh/local-roots"
GPU_ANNOTATION = "devspace.sh/gpus"
GPU_RESOURCE = "amd.com/gpu"

# Images that stand for "the host runtime" (the local cluster runs workloads on the host's
# python/node/rocm stack instead of pulling layers).
HOST_IMAGES = ("rocm/pytorch", "rocm/dev", "python", "node", "ubuntu", "debian", "busybox", "alpine",
               "devspace-local/runtime", "gcr.io/kaniko-project/executor")

def close_proc(proc):
    """Close an asyncio subprocess's transport (its pipes) from the running loop. Left to the
    GC, the transport closes after the loop did and raises 'Event loop is closed'."""
    t = getattr(proc, "_transport", None) if proc is not None else None
    if t is not None and not t.is_closing():
        t.close()


HOST_ONLY_ENV = {"RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                 "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT", "KUBECONFIG",
                 "DOCKER_HOST", "DOCKER_CERT_PATH", "DOCKER_TLS_VERIFY", "HIP_VISIBLE_DEVICES",
                 "CUDA_VISIBLE_DEVICES", "DEVSPACE_NONINTERACTIVE",
                 # a container sees its image's Python path, not the developer's checkout: a pod
                 # imports devspace_amd only when its project vendors it (rocm-pytorch kit)
                 "PYTHONPATH"}
HOST_ONLY_ENV_PREFIXES = ("TORCHELASTIC_", "TORCH_ELASTIC_", "PET_")

# Binaries of tool images that exist on the host under another name / as an emulation.
RUNTIME_ALIASES = {
    "/busybox/sleep": ("sleep",),
    "/busybox/sh": ("sh",),
    "/kaniko/executor": (sys.executable, "-m", "devspace_amd.localkube.kaniko"),
}


# AMD GPU device plugin: compute partitions per GPU by mode (MI355X: 8 XCDs, one per CPX partition)
PARTITIONS = {"spx": 1, "dpx": 2, "qpx": 4, "cpx": 8}


def _gpu_request(container, resource=GPU_RESOURCE):
    res = container.get("resources") or {}
    for part in ("limits", "requests"):
        v = (res.get(part) or {}).get(resource)
        if v is not None:
            try:
                return int(str(v))
            except ValueError:
                return 0
    return 0


def template_hash(template):
    return hashlib.sha256(json.dumps(template, sort_keys=True).encode()).hexdigest()[:10]


class Container:
    def __init__(self, name, spec, root):
        self.name = name
        self.spec = spec
        self.root = root
        self.proc = None
        self.exec_procs = set()  # `kubectl exec` processes: killed with the container (cgroup)
        self.restarts = 0
        self.state = {"waiting": {"reason": "ContainerCreating"}}
        self.last_state = {}
        self.next_start = 0.0
        self.log_path = root + ".log"
        self.started_at = None
        self.image_config = {}
        self.fatal = None  # waiting reason that will not recover (ErrImagePull, ...)
        self.fatal_at = 0.0
        self.pulling = False  # slow-pull mode: its `Pulling` event was sent
        self.pull_started_now = False
        # Output streaming (like a CRI log pipe): the pump appends to the log file and pushes
        # (offset, chunk) to attach/follow subscribers as soon as the process writes it;
        # (None, None) marks the end of this process' output.
        self.subscribers = set()
        self.log_size = os.path.getsize(self.log_path) if os.path.exists(self.log_path) else 0
        self.pump = None

    def subscribe(self):
        q = asyncio.Queue()
        self.subscribers.add(q)
        return q

    def unsubscribe(self, q):
        self.subscribers.discard(q)

    async def pump_output(self, stream):
        with open(self.log_path, "ab", buffering=0) as logf:
            while True:
                chunk = await stream.read(65536)
                if not chunk:
                    break
                logf.write(chunk)
                off = self.log_size
                self.log_size += len(chunk)
                for q in list(self.subscribers):
                    q.put_nowait((off, chunk))
        for q in list(self.subscribers):
            q.put_nowait((None, None))


class PodRuntime:
    def __init__(self, ns, name, uid, base):
        self.ns, self.name, self.uid = ns, name, uid
        self.dir = os.path.join(base, f"{ns}_{name}_{uid[:8]}")
        self.containers = {}
        self.gpus = []
        self.deleting = False


class Kubelet:
    def __init__(self, store, images, state_dir, node_name="devspace-local", gpus=0, extra_env=None):
        self.store = store
        self.images = images
        self.state_dir = state_dir
        self.node_name = node_name
        self.physical_gpus = gpus
        self.gpus_total = gpus  # schedulable devices: GPUs, or compute partitions of them
        self.gpus_free = list(range(gpus))
        self.partition, self.memory_partition, self.gpu_resource = "spx", "nps1", GPU_RESOURCE
        self.unhealthy = 0
        self.pods = {}  # (ns, name) -> PodRuntime
        self.extra_env = extra_env or {}
        self.pods_dir = os.path.join(state_dir, "pods")
        os.makedirs(self.pods_dir, exist_ok=True)
        self._stop = False
        self._event_names = {}  # (ns, uid, reason, message, type) -> Event name, for aggregation
        self._exited_procs = []
        # Slow-pull mode: an image this node has not pulled yet takes `pull_seconds` to pull
        # (a first `rocm/pytorch` pull onto a fresh GPU node takes minutes): the container waits
        # in ContainerCreating after a `Pulling` event, then `Pulled` ("Successfully pulled ...").
        self.pull_seconds = 0.0
        self.pulled = set()
        self._pull_done = {}  # image -> monotonic time its pull completes
        # Flaky registry: pulls of images starting with a key fail with a transient error (an i/o
        # timeout) until the monotonic time given; the kubelet retries after its back-off, as a
        # real one does.
        self.pull_flaky = {}

    # ------------------------------------------------------------ node

    def set_gpu_topology(self, partition="spx", memory_partition="nps1", strategy="single", unhealthy=0):
        """What the AMD GPU device plugin and node labeller would show for this node: each GPU in
        `partition` mode is 1 (SPX), 2 (DPX), 4 (QPX) or 8 (CPX) schedulable devices, advertised as
        amd.com/gpu ("single" strategy) or amd.com/<partition>_<nps> ("mixed"); `unhealthy` devices
        stay in capacity but leave allocatable (the plugin's health check). Call before start()."""
        partition, memory_partition = partition.lower(), memory_partition.lower()
        if partition not in PARTITIONS:
            raise ValueError(f"unknown compute partition mode {partition!r}")
        self.partition, self.memory_partition = partition, memory_partition
        self.gpu_resource = GPU_RESOURCE if strategy == "single" else f"amd.com/{partition}_{memory_partition}"
        self.gpus_total = self.physical_gpus * PARTITIONS[partition]
        self.unhealthy = max(0, min(unhealthy, self.gpus_total))
        self.gpus_free = list(range(self.gpus_total - self.unhealthy))  # the last ones failed

    def add_gpus(self, n):
        """A GPU node pool scaled up (a cluster autoscaler's new node, folded into this one): n more
        physical GPUs in the current partition mode, advertised at once."""
        old_total = self.gpus_total
        self.physical_gpus += n
        self.gpus_total = self.physical_gpus * PARTITIONS[self.partition]
        self.gpus_free.extend(range(old_total, self.gpus_total))
        res = self.gpu_resource

        def grow(o):
            for part in ("capacity", "allocatable"):
                o["status"][part][res] = str(self.gpus_total - (self.unhealthy if part == "allocatable" else 0))

        self.store.mutate("", "nodes", "", self.node_name, grow)

    def register_node(self):
        res = self.gpu_resource
        node = {
            "apiVersion": "v1",
            "kind": "Node",
            "metadata": {
                "name": self.node_name,
                "labels": {
                    "kubernetes.io/hostname": self.node_name,
                    "beta.amd.com/gpu.family.AI": "1" if self.gpus_total else "0",
                    "amd.com/gpu.product-name": "AMD_Instinct_MI355X" if self.gpus_total else "",
                    "amd.com/gpu.device-id": "75a3" if self.gpus_total else "",
                    **({"amd.com/gpu.vram": "288G",
                        "amd.com/gpu.compute-partitioning-mode": self.partition,
                        "amd.com/gpu.memory-partitioning-mode": self.memory_partition} if self.gpus_total else {}),
                },
            },
            "status": {
                "capacity": {"cpu": str(os.cpu_count() or 1), "memory": "64Gi", res: str(self.gpus_total)},
                "allocatable": {"cpu": str(os.cpu_count() or 1), "memory": "64Gi",
                                res: str(self.gpus_total - self.unhealthy)},
                "conditions": [{"type": "Ready", "status": "True"}],
                "nodeInfo": {"kubeletVersion": "v1.29.0-devspace-local", "osImage": "local processes"},
            },
        }
        try:
            self.store.create("", "nodes", "", node, "v1")
        except ApiError:
            pass

    # ------------------------------------------------------------ events

    def _trace(self, what, **kw):
        """Kubelet-side timings into LOCALKUBE_TRACE (same file as the store's object events)."""
        path = os.environ.get("LOCALKUBE_TRACE")
        if path:
            rec = {"t_ms": round(time.time() * 1000.0, 2), "ev": what, "res": "kubelet", "name": kw.pop("pod", ""),
                   "phase": None, "ready": None}
            rec.update({k: round(v, 2) if isinstance(v, float) else v for k, v in kw.items()})
            with open(path, "a") as f:
                f.write(json.dumps(rec) + "\n")

    def event(self, obj, reason, message, etype="Normal"):
        md = obj["metadata"]
        ns = md.get("namespace", "default")
        # Repeats of one event (same object, reason, message, type) bump count/lastTimestamp of
        # the existing Event, as client-go's EventCorrelator does, instead of adding objects.
        key = (ns, md.get("uid") or md["name"], reason, message, etype)
        seen = self._event_names.get(key)
        if seen is not None:
            def bump(ev):
                ev["count"] = int(ev.get("count") or 1) + 1
                ev["lastTimestamp"] = now_rfc3339()

            if self.store.mutate("", "events", ns, seen, bump) is not None:
                return
        name = f"{md['name']}.{int(time.time() * 1e6):x}"
        self._event_names[key] = name
        ev = {
            "apiVersion": "v1",
            "kind": "Event",
            "metadata": {"name": name, "namespace": ns},
            "involvedObject": {"kind": obj.get("kind", "Pod"), "name": md["name"], "namespace": ns,
                               "uid": md.get("uid"), "apiVersion": obj.get("apiVersion", "v1")},
            "reason": reason,
            "message": message,
            "type": etype,
            "count": 1,
            "firstTimestamp": now_rfc3339(),
            "lastTimestamp": now_rfc3339(),
            "source": {"component": "kubelet", "host": self.node_name},
        }
        try:
            self.store.create("", "events", ns, ev, "v1")
        except ApiError:
            pass

    # ------------------------------------------------------------ controllers

    def reconcile_workloads(self):
        for group, resource in (("apps", "deployments"), ("apps", "statefulsets"), ("apps", "replicasets"),
                                ("apps", "daemonsets")):
            for obj in self.store.list(group, resource):
                self._reconcile_one(group, resource, obj)

    def _reconcile_one(self, group, resource, obj):
        md = obj["metadata"]
        ns = md["namespace"]
        spec = obj.get("spec", {})
        template = spec.get("template", {})
        replicas = 1 if resource == "daemonsets" else int(spec.get("replicas", 1) if spec.get("replicas") is not None else 1)
        h = template_hash(template)
        owned = [o for (k, o) in self.store.owned_by(md["uid"]) if k[1] == "pods"]
        current = [p for p in owned if p["metadata"].get("labels", {}).get("pod-template-hash") == h
                   and not p["metadata"].get("deletionTimestamp")]
        stale = [p for p in owned if p["metadata"].get("labels", {}).get("pod-template-hash") != h]
        for p in stale:  # Recreate strategy: the local cluster has no surge capacity worth modelling
            if not p["metadata"].get("deletionTimestamp"):
                self.store.mark_deleting("", "pods", ns, p["metadata"]["name"])
        for p in current[replicas:]:
            self.store.mark_deleting("", "pods", ns, p["metadata"]["name"])
        current = current[:replicas]
        names = {p["metadata"]["name"] for p in current}
        for i in range(len(current), replicas):
            if resource == "statefulsets":
                name = f"{md['name']}-{i}"
                while name in names:
                    i += 1
                    name = f"{md['name']}-{i}"
                if self.store.try_get("", "pods", ns, name):
                    continue  # old ordinal still terminating
            else:
                name = f"{md['name']}-{h[:8]}-{os.urandom(3).hex()[:5]}"
            names.add(name)
            pmd = dict(template.get("metadata") or {})
            labels = dict(pmd.get("labels") or {})
            labels["pod-template-hash"] = h
            pod = {
                "apiVersion": "v1",
                "kind": "Pod",
                "metadata": {
                    "name": name,
                    "namespace": ns,
                    "labels": labels,
                    "annotations": dict(pmd.get("annotations") or {}),
                    "ownerReferences": [{"apiVersion": obj.get("apiVersion", "apps/v1"), "kind": obj.get("kind"),
                                         "name": md["name"], "uid": md["uid"], "controller": True}],
                },
                "spec": json.loads(json.dumps(template.get("spec") or {})),
                "status": {"phase": "Pending"},
            }
            try:
                self.store.create("", "pods", ns, pod, "v1")
                self.event(obj, "SuccessfulCreate", f"Created pod: {name}")
            except ApiError:
                pass
        ready = 0
        for p in current:
            st = p.get("status", {})
            if st.get("phase") == "Running" and all(c.get("ready") for c in st.get("containerStatuses", []) or [{}]):
                ready += 1
        status = {"observedGeneration": md.get("generation", 1), "replicas": len(current),
                  "readyReplicas": ready, "availableReplicas": ready, "updatedReplicas": len(current),
                  "currentReplicas": len(current)}
        if obj.get("status") != status:
            self.store.update_status(group, resource, ns, md["name"], status)

    def reconcile_jobs(self):
        """Job controller (batch/v1): one pod at a time from the template; a succeeded pod
        completes the Job (condition Complete), failed pods are replaced until
        spec.backoffLimit (default 6) is exceeded (condition Failed). Helm hooks wait on this."""
        for job in self.store.list("batch", "jobs"):
            md, spec = job["metadata"], job.get("spec", {})
            st = job.get("status") or {}
            if md.get("deletionTimestamp") or any(c.get("status") == "True" and c.get("type") in ("Complete", "Failed")
                                                  for c in st.get("conditions", [])):
                continue
            ns = md["namespace"]
            pods = [o for (k, o) in self.store.owned_by(md["uid"]) if k[1] == "pods"]
            succeeded = sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Succeeded")
            failed = sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Failed")
            active = [p for p in pods if (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")
                      and not p["metadata"].get("deletionTimestamp")]
            now = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
            status = {"active": len(active), "succeeded": succeeded, "failed": failed,
                      "startTime": st.get("startTime") or now}
            if succeeded >= int(spec.get("completions") or 1):
                status["conditions"] = [{"type": "Complete", "status": "True", "lastTransitionTime": now}]
                status["completionTime"] = now
                status["active"] = 0
                self.event(job, "Completed", "Job completed")
            elif failed > int(spec.get("backoffLimit", 6)):
                status["conditions"] = [{"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded",
                                         "message": "Job has reached the specified backoff limit",
                                         "lastTransitionTime": now}]
                status["active"] = 0
                self.event(job, "BackoffLimitExceeded", "Job has reached the specified backoff limit", "Warning")
            elif not active:
                template = spec.get("template") or {}
                pmd = dict(template.get("metadata") or {})
                labels = dict(pmd.get("labels") or {})
                labels.setdefault("job-name", md["name"])
                labels.setdefault("controller-uid", md["uid"])
                name = f"{md['name']}-{os.urandom(3).hex()[:5]}"
                pspec = json.loads(json.dumps(template.get("spec") or {}))
                pspec.setdefault("restartPolicy", "Never")
                pod = {"apiVersion": "v1", "kind": "Pod",
                       "metadata": {"name": name, "namespace": ns, "labels": labels,
                                    "annotations": dict(pmd.get("annotations") or {}),
                                    "ownerReferences": [{"apiVersion": "batch/v1", "kind": "Job", "name": md["name"],
                                                         "uid": md["uid"], "controller": True}]},
                       "spec": pspec, "status": {"phase": "Pending"}}
                try:
                    self.store.create("", "pods", ns, pod, "v1")
                    self.event(job, "SuccessfulCreate", f"Created pod: {name}")
                    status["active"] = 1
                except ApiError:
                    pass
            if {k: v for k, v in st.items()} != status:
                self.store.update_status("batch", "jobs", ns, md["name"], status)

    def reconcile_pvcs(self):
        """PV binder + pvc-protection: bind new claims to a local volume (the binder writes
        spec.volumeName, as on a real cluster), release a deleted claim once no pod uses it."""
        for pvc in self.store.list("", "persistentvolumeclaims"):
            md = pvc["metadata"]
            ns, name = md["namespace"], md["name"]
            if md.get("deletionTimestamp"):
                in_use = any(
                    v.get("persistentVolumeClaim", {}).get("claimName") == name
                    for p in self.store.list("", "pods", ns)
                    for v in (p.get("spec") or {}).get("volumes") or [])
                if not in_use:
                    try:
                        self.store.delete("", "persistentvolumeclaims", ns, name)
                    except ApiError:
                        pass
                continue
            if not (pvc.get("spec") or {}).get("volumeName"):
                vol = "pvc-" + md["uid"]

                def bind(o, vol=vol):
                    o.setdefault("spec", {})["volumeName"] = vol
                    o.setdefault("metadata", {}).setdefault("annotations", {})[
                        "pv.kubernetes.io/bind-completed"] = "yes"

                self.store.mutate("", "persistentvolumeclaims", ns, name, bind)
            if (pvc.get("status") or {}).get("phase") != "Bound":
                self.store.update_status("", "persistentvolumeclaims", ns, name,
                                         {"phase": "Bound", "accessModes": (pvc.get("spec") or {}).get("accessModes"),
                                          "capacity": ((pvc.get("spec") or {}).get("resources") or {}).get("requests")})

    # ------------------------------------------------------------ pods

    async def reconcile_pods(self):
        """Returns True when a pod status was written (workload status needs a refresh)."""
        seen = set()
        changed = False
        for pod in self.store.list("", "pods"):
            md = pod["metadata"]
            key = (md["namespace"], md["name"])
            seen.add(key)
            rt = self.pods.get(key)
            if md.get("deletionTimestamp"):
                await self._delete_pod(key, pod)
                continue
            if rt is None:
                rt = self._admit(pod)
                if rt is None:
                    continue
            changed |= await self._sync_containers(rt, pod)
        for key in list(self.pods):
            if key not in seen:  # removed from the store without graceful deletion
                await self._kill_pod(self.pods.pop(key), 0)
        return changed

    def _admit(self, pod):
        md = pod["metadata"]
        containers = pod.get("spec", {}).get("containers", []) or []
        want = sum(_gpu_request(c, self.gpu_resource) for c in containers)
        if want > len(self.gpus_free):
            st = pod.get("status") or {}
            if not any(c.get("reason") == "Unschedulable" for c in st.get("conditions") or []):
                msg = f"0/1 nodes are available: 1 Insufficient {self.gpu_resource}."
                self.store.update_status("", "pods", md["namespace"], md["name"], {
                    "phase": "Pending", "conditions": [{"type": "PodScheduled", "status": "False",
                                                        "reason": "Unschedulable", "message": msg}]})
                self.event(pod, "FailedScheduling", msg, "Warning")
            return None
        rt = PodRuntime(md["namespace"], md["name"], md["uid"], self.pods_dir)
        rt.gpus = [self.gpus_free.pop(0) for _ in range(want)]
        os.makedirs(rt.dir, exist_ok=True)
        roots = {}
        for c in containers:
            root = os.path.join(rt.dir, c["name"])
            os.makedirs(root, exist_ok=True)
            rt.containers[c["name"]] = Container(c["name"], c, root)
            roots[c["name"]] = root

        def annotate(o):
            o["metadata"].setdefault("annotations", {})[LOCAL_ROOTS_ANNOTATION] = json.dumps(roots)
            if rt.gpus:
                o["metadata"]["annotations"][GPU_ANNOTATION] = ",".join(map(str, rt.gpus))
            o["spec"]["nodeName"] = self.node_name

        self.store.mutate("", "pods", md["namespace"], md["name"], annotate)
        self.event(pod, "Scheduled", f"Successfully assigned {md['namespace']}/{md['name']} to {self.node_name}")
        self.pods[(md["namespace"], md["name"])] = rt
        return rt

    def _pulled(self, pod, c):
        """Slow-pull mode: False while the container's image is still being pulled (the first
        call emits the `Pulling` event), True once it is on the node."""
        image = c.spec.get("image", "")
        if self.pull_seconds <= 0 or image in self.pulled or self.images.resolve(image) is None:
            return True  # an image that does not exist fails in _prepare_rootfs (ErrImagePull)
        now = time.monotonic()
        done = self._pull_done.get(image)
        if done is None:
            done = self._pull_done[image] = now + self.pull_seconds
        if not c.pulling:
            c.pulling = True
            c.pull_started_now = True
            self.event(pod, "Pulling", f'Pulling image "{image}"')
        if now < done:
            return False
        self.pulled.add(image)
        self.event(pod, "Pulled", f'Successfully pulled image "{image}" in {self.pull_seconds:.3f}s')
        return True

    def _prepare_rootfs(self, rt, c, pod):
        image = c.spec.get("image", "")
        if any(image.startswith(k) and time.monotonic() < t for k, t in self.pull_flaky.items()):
            return "ErrImagePull", (f'Failed to pull image "{image}": rpc error: code = Unknown desc = failed to '
                                    f'resolve reference "{image}": dial tcp 10.96.0.53:443: i/o timeout')
        img = self.images.resolve(image)
        if img is None:
            if not image or not any(image.split("@")[0].split(":")[0].endswith(h) or image.startswith(h)
                                    for h in HOST_IMAGES):
                return "ErrImagePull", f'Failed to pull image "{image}": not found in the local registry'
            img = {"config": {}, "rootfs": None}
        else:
            self.event(pod, "Pulled", f'Container image "{image}" present in local registry')
        c.image_config = img.get("config") or {}
        if img.get("rootfs") and os.path.isdir(img["rootfs"]):
            shutil.copytree(img["rootfs"], c.root, symlinks=True, dirs_exist_ok=True)
        for vm in c.spec.get("volumeMounts") or []:
            self._mount(rt, pod, c, vm)
        return None, None

    def _mount(self, rt, pod, c, vm):
        vols = {v["name"]: v for v in pod.get("spec", {}).get("volumes") or []}
        v = vols.get(vm.get("name"), {})
        target = os.path.join(c.root, vm.get("mountPath", "/").lstrip("/"))
        if v.get("persistentVolumeClaim"):
            src = os.path.join(self.state_dir, "volumes", rt.ns, v["persistentVolumeClaim"]["claimName"],
                               (vm.get("subPath") or "").lstrip("/"))
        else:
            src = os.path.join(rt.dir, "volumes", vm.get("name", "v"), (vm.get("subPath") or "").lstrip("/"))
        os.makedirs(src, exist_ok=True)
        if os.path.islink(target) or os.path.exists(target):
            return
        os.makedirs(os.path.dirname(target), exist_ok=True)
        os.symlink(src, target)

    def _argv(self, c):
        spec, cfg = c.spec, c.image_config
        cmd, args = spec.get("command"), spec.get("args")
        if cmd:
            argv = list(cmd) + list(args or [])
        elif args:
            argv = list(cfg.get("Entrypoint") or []) + list(args)
        else:
            argv = list(cfg.get("Entrypoint") or []) + list(cfg.get("Cmd") or [])
        return self.map_argv(c, argv)

    def map_argv(self, c, argv):
        """Container paths -> host paths under the container root, plus runtime aliases for the
        well-known tool images (busybox shell utils, the kaniko executor)."""
        argv = [str(a) for a in argv]
        if argv and argv[0] in RUNTIME_ALIASES:
            argv = list(RUNTIME_ALIASES[argv[0]]) + argv[1:]
        out = []
        for a in argv:
            a = str(a)
            if a.startswith("/") and len(a) > 1 and not a.startswith(c.root + "/") and a != sys.executable:
                first = a.lstrip("/").split("/", 1)[0]
                if first and os.path.exists(os.path.join(c.root, first)):
                    a = os.path.join(c.root, a.lstrip("/"))
            out.append(a)
        return out

    def _env(self, rt, c):
        # Containers do not inherit the launcher's process-group / client configuration (a pod
        # started from a torchrun'd process must not join that rendezvous).
        env = {k: v for k, v in os.environ.items()
               if k not in HOST_ONLY_ENV and not k.startswith(HOST_ONLY_ENV_PREFIXES)}
        env.update(self.extra_env)
        for kv in c.image_config.get("Env") or []:
            if "=" in kv:
                k, v = kv.split("=", 1)
                env[k] = v
        for e in c.spec.get("env") or []:
            if "value" in e:
                env[e["name"]] = str(e["value"])
        if self._argv(c)[:3] == [sys.executable, "-m", "devspace_amd.localkube.kaniko"]:
            # the kaniko emulation is part of this cluster, not of the image
            env["PYTHONPATH"] = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["HOSTNAME"] = rt.name
        env["DEVSPACE_CONTAINER_ROOT"] = c.root
        env["DEVSPACE_LOCAL_IMAGES"] = self.images.root  # used by the kaniko emulation
        # Node GPU index i is the i-th device this node process may use (the device plugin's
        # view): map through the host's own HIP_VISIBLE_DEVICES when it restricts devices.
        host_vis = [v.strip() for v in os.environ.get("HIP_VISIBLE_DEVICES", "").split(",") if v.strip()]
        if rt.gpus:
            # A node configured with more GPUs than the host has (a bench rehearsal of N ranks on a
            # smaller box) maps its extra indices onto the real devices instead of naming devices
            # this process may not use.
            real = self._real_gpus()
            parts = PARTITIONS.get(self.partition, 1)  # a partition runs on its GPU (g // parts)
            phys = [g // parts for g in rt.gpus]
            ids = [host_vis[g] if g < len(host_vis) else str(g) for g in ((g % real if real else g) for g in phys)]
            env["HIP_VISIBLE_DEVICES"] = ",".join(dict.fromkeys(ids))
        elif self.gpus_total:
            env["HIP_VISIBLE_DEVICES"] = "-1"  # no amd.com/gpu request: no GPU access
        elif host_vis:
            env["HIP_VISIBLE_DEVICES"] = ",".join(host_vis)
        return env

    def _real_gpus(self):
        if not hasattr(self, "_real_gpu_count"):
            from .cluster import detect_gpus  # noqa: WPS433 - cluster imports this module

            self._real_gpu_count = detect_gpus()
        return self._real_gpu_count

    def workdir(self, c):
        wd = c.spec.get("workingDir") or c.image_config.get("WorkingDir") or "/"
        return os.path.join(c.root, wd.lstrip("/"))

    async def _start(self, rt, c, pod):
        argv = self._argv(c)
        if not argv:
            c.state = {"waiting": {"reason": "CreateContainerConfigError", "message": "no command specified"}}
            c.fatal = "CreateContainerConfigError"
            return
        cwd = self.workdir(c)
        os.makedirs(cwd, exist_ok=True)
        try:
            c.proc = await asyncio.create_subprocess_exec(*argv, cwd=cwd, env=self._env(rt, c),
                                                          stdout=asyncio.subprocess.PIPE,
                                                          stderr=asyncio.subprocess.STDOUT,
                                                          stdin=asyncio.subprocess.DEVNULL, start_new_session=True)
        except (FileNotFoundError, PermissionError) as e:
            c.state = {"waiting": {"reason": "RunContainerError", "message": str(e)}}
            c.next_start = time.time() + min(30.0, 0.5 * (2 ** c.restarts))
            c.restarts += 1
            self.event(pod, "Failed", f"Error: {e}", "Warning")
            return
        c.pump = asyncio.create_task(c.pump_output(c.proc.stdout))
        c.started_at = now_rfc3339()
        c.state = {"running": {"startedAt": c.started_at}}
        self.event(pod, "Started", f"Started container {c.name}")

    async def _sync_containers(self, rt, pod):
        changed = False
        for name, c in rt.containers.items():
            if c.fatal:
                if getattr(c, "retry_at", None) and time.monotonic() >= c.retry_at:
                    c.fatal, c.retry_at = None, None  # a transient pull error: try again after the back-off
                    continue
                if c.fatal == "ErrImagePull" and time.monotonic() - c.fatal_at >= 1.0:
                    # the kubelet's image back-off, as on a real node: ErrImagePull -> ImagePullBackOff
                    image = c.spec.get("image", "")
                    c.fatal = "ImagePullBackOff"
                    c.state = {"waiting": {"reason": "ImagePullBackOff",
                                           "message": f'Back-off pulling image "{image}"'}}
                    self.event(pod, "BackOff", f'Back-off pulling image "{image}"', "Warning")
                    changed = True
                continue
            if c.proc is None and c.started_at is None and c.restarts == 0 and not c.next_start:
                if not self._pulled(pod, c):
                    changed |= c.pull_started_now
                    c.pull_started_now = False
                    continue
                t0 = time.perf_counter()
                reason, msg = self._prepare_rootfs(rt, c, pod)
                if reason:
                    c.state = {"waiting": {"reason": reason, "message": msg}}
                    c.fatal = reason
                    c.fatal_at = time.monotonic()
                    if "i/o timeout" in msg:
                        c.retry_at = c.fatal_at + 2.0
                    self.event(pod, "Failed", msg, "Warning")
                    changed = True
                    continue
                t1 = time.perf_counter()
                await self._start(rt, c, pod)
                self._trace("container_start", pod=rt.name, container=name, rootfs_ms=(t1 - t0) * 1e3,
                            exec_ms=(time.perf_counter() - t1) * 1e3)
                changed = True
            elif c.proc is not None and c.proc.returncode is not None:
                code = c.proc.returncode
                c.last_state = {"terminated": {"exitCode": code, "reason": "Completed" if code == 0 else "Error",
                                               "startedAt": c.started_at, "finishedAt": now_rfc3339()}}
                # its pipes may outlive it (grandchildren keep them open): closed at shutdown
                self._exited_procs = [p for p in self._exited_procs
                                      if getattr(p, "_transport", None) and not p._transport.is_closing()]
                self._exited_procs.append(c.proc)
                c.proc = None
                policy = pod.get("spec", {}).get("restartPolicy", "Always")
                if policy == "Never" or (policy == "OnFailure" and code == 0):
                    c.state = dict(c.last_state)
                else:
                    c.restarts += 1
                    delay = min(30.0, 0.5 * (2 ** (c.restarts - 1)))
                    c.next_start = time.time() + delay
                    c.state = {"waiting": {"reason": "CrashLoopBackOff",
                                           "message": f"back-off {delay:.1f}s restarting failed container={name}"}}
                    self.event(pod, "BackOff", f"Back-off restarting failed container {name}", "Warning")
                changed = True
            elif c.proc is None and c.next_start and time.time() >= c.next_start:
                c.next_start = 0.0
                await self._start(rt, c, pod)
                changed = True
        if changed or not (pod.get("status") or {}).get("containerStatuses"):
            self._write_status(rt, pod)
            return True
        return False

    def _write_status(self, rt, pod):
        statuses = []
        all_running = True
        any_fatal = None
        for c in rt.containers.values():
            running = "running" in c.state
            all_running &= running
            if c.fatal:
                any_fatal = c.fatal
            statuses.append({"name": c.name, "ready": running, "restartCount": c.restarts,
                             "image": c.spec.get("image", ""), "imageID": "", "containerID": f"local://{c.name}",
                             "state": c.state, "lastState": c.last_state, "started": running})
        phase = "Running" if all_running else "Pending"
        if not all_running and any("terminated" in s["state"] for s in statuses) and all(
                "terminated" in s["state"] for s in statuses):
            phase = "Succeeded" if all(s["state"]["terminated"]["exitCode"] == 0 for s in statuses) else "Failed"
        status = {
            "phase": phase,
            "hostIP": "127.0.0.1",
            "podIP": "127.0.0.1",
            "startTime": pod["metadata"].get("creationTimestamp"),
            "conditions": [{"type": "PodScheduled", "status": "True"},
                           {"type": "Ready", "status": "True" if all_running else "False"},
                           {"type": "ContainersReady", "status": "True" if all_running else "False"}],
            "containerStatuses": statuses,
        }
        self.store.update_status("", "pods", rt.ns, rt.name, status)

    async def _kill_pod(self, rt, grace):
        # exec'd processes die with the container, as in a real container cgroup: they must
        # not outlive the pod and watch its filesystem being removed
        for c in rt.containers.values():
            for ep in list(c.exec_procs):
                if ep.returncode is None:
                    try:
                        os.killpg(ep.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
        procs = [c.proc for c in rt.containers.values() if c.proc and c.proc.returncode is None]
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        deadline = time.time() + grace
        for p in procs:
            try:
                await asyncio.wait_for(p.wait(), timeout=max(0.05, deadline - time.time()))
            except asyncio.TimeoutError:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                await p.wait()
        for c in rt.containers.values():  # drain the log pumps so no pipe outlives the pod
            if getattr(c, "pump", None) is not None and not c.pump.done():
                try:
                    await asyncio.wait_for(asyncio.shield(c.pump), timeout=0.5)
                except (asyncio.TimeoutError, asyncio.CancelledError):
                    c.pump.cancel()
            close_proc(c.proc)
        self.gpus_free.extend(rt.gpus)
        self.gpus_free.sort()
        rt.gpus = []
        shutil.rmtree(rt.dir, ignore_errors=True)
        for c in rt.containers.values():
            try:
                os.unlink(c.log_path)
            except OSError:
                pass

    async def _delete_pod(self, key, pod):
        rt = self.pods.pop(key, None)
        if rt is not None:
            grace = min(5, int(pod.get("spec", {}).get("terminationGracePeriodSeconds", 5) or 0))
            await self._kill_pod(rt, grace)
        try:
            self.store.delete("", "pods", key[0], key[1])
        except ApiError:
            pass

    # ------------------------------------------------------------ helpers for the API server

    def container(self, ns, pod, name):
        rt = self.pods.get((ns, pod))
        if rt is None:
            return None, None
        if not name:
            name = next(iter(rt.containers), None)
        return rt, rt.containers.get(name)

    async def run(self):
        """Reconcile loop: runs on every create/replace/delete in the store (no polling delay
        between `helm install` and the pod starting) and at least every 50 ms (process exits,
        restart back-offs). Workload status is refreshed after the pods in the same pass, so a
        Deployment reports ready replicas as soon as its pod runs."""
        self.register_node()
        loop = asyncio.get_running_loop()
        wake = asyncio.Event()

        def waker(_key):
            loop.call_soon_threadsafe(wake.set)

        self.store.wakers.append(waker)
        try:
            while not self._stop:
                wake.clear()
                try:
                    self.reconcile_workloads()
                    self.reconcile_jobs()
                    self.reconcile_pvcs()
                    if await self.reconcile_pods():
                        self.reconcile_workloads()
                        self.reconcile_jobs()
                except Exception as e:  # keep the node alive; surface in the log
                    print(f"[localkube] reconcile error: {e!r}", flush=True)
                try:
                    await asyncio.wait_for(wake.wait(), 0.05)
                except asyncio.TimeoutError:
                    pass
        finally:
            self.store.wakers.remove(waker)

    async def shutdown(self):
        self._stop = True
        for key in list(self.pods):
            await self._kill_pod(self.pods.pop(key), 1)
        for proc in self._exited_procs:
            close_proc(proc)
        self._exited_procs.clear()
