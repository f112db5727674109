"""Docker Engine API subset over a unix socket + local image store / registry.

Serves what the devspace builder needs (reference: builder/docker/docker.go): /_ping,
/version, /info, /auth, /build (tar context + Dockerfile), /images/{name}/push,
/images/{name}/tag, /images/{name}/json. Images are directories (rootfs + config.json); a
Dockerfile is interpreted instruction by instruction (FROM/WORKDIR/COPY/ADD/ENV/ARG/EXPOSE/
CMD/ENTRYPOINT/LABEL/USER). RUN is recorded, and executed only when the store's `run_steps` is
on: then its command runs on the host runtime (the pods' runtime here) in the image's working
directory, and the resulting filesystem is kept as that layer's snapshot, restored instead of
running the step again when a later build hits the same cache key.

Layer cache keys as the classic builder computes them: each instruction's key chains the
previous one with the instruction text (after ARG/ENV substitution), and a COPY/ADD also with
the content (paths, modes, bytes; not mtimes) of what it copies. A key the daemon built before
is "Using cache"; the image's RootFS.Layers lists the keys of its filesystem layers (COPY, ADD,
RUN). So a Dockerfile that copies train.py before a slow RUN rebuilds that RUN on every edit
of train.py, and one that copies it after does not, which a test can see without executing RUN.
"""

from __future__ import annotations

import glob
import gzip
import hashlib
import io
import json
import os
import re
import shlex
import shutil
import tarfile
import tempfile

from aiohttp import web


def normalize(ref: str):
    """'docker.io/library/node:8' -> ('node', '8'); digests dropped."""
    ref = ref.split("@")[0]
    name, tag = ref, "latest"
    last = ref.rsplit("/", 1)[-1]
    if ":" in last:
        name, tag = ref.rsplit(":", 1)
    for p in ("docker.io/library/", "docker.io/", "index.docker.io/library/", "library/"):
        if name.startswith(p):
            name = name[len(p):]
    return name, tag


class ImageStore:
    MAX_SNAPSHOTS = 16  # RUN layers whose filesystem is kept (oldest dropped first)

    def __init__(self, root):
        self.root = root
        self.run_steps = False  # execute RUN (on the host runtime) instead of only recording it
        os.makedirs(os.path.join(root, "images"), exist_ok=True)
        os.makedirs(os.path.join(root, "registry"), exist_ok=True)

    def snapshot_dir(self, key):
        return os.path.join(self.root, "layers", key)

    def keep_snapshot(self, key, rootfs):
        d = self.snapshot_dir(key)
        if os.path.exists(d):
            shutil.rmtree(d)
        shutil.copytree(rootfs, d, symlinks=True)
        base = os.path.join(self.root, "layers")
        snaps = sorted((os.path.getmtime(os.path.join(base, n)), n) for n in os.listdir(base))
        for _, n in snaps[:max(0, len(snaps) - self.MAX_SNAPSHOTS)]:
            shutil.rmtree(os.path.join(base, n), ignore_errors=True)

    def _dir(self, kind, ref):
        name, tag = normalize(ref)
        return os.path.join(self.root, kind, name.replace("/", "__"), tag)

    def local(self, ref):
        d = self._dir("images", ref)
        return d if os.path.exists(os.path.join(d, "config.json")) else None

    def resolve(self, ref):
        """Registry first (what a node would pull), then the daemon's local images."""
        for kind in ("registry", "images"):
            d = self._dir(kind, ref)
            if os.path.exists(os.path.join(d, "config.json")):
                with open(os.path.join(d, "config.json")) as f:
                    cfg = json.load(f)
                return {"config": cfg, "rootfs": os.path.join(d, "rootfs"), "dir": d}
        return None

    def save(self, ref, rootfs_src, config):
        d = self._dir("images", ref)
        if os.path.exists(d):
            shutil.rmtree(d)
        os.makedirs(d)
        shutil.copytree(rootfs_src, os.path.join(d, "rootfs"), symlinks=True)
        with open(os.path.join(d, "config.json"), "w") as f:
            json.dump(config, f)
        return d

    def push(self, ref):
        src = self.local(ref)
        if not src:
            return False
        dst = self._dir("registry", ref)
        if os.path.exists(dst):
            shutil.rmtree(dst)
        shutil.copytree(src, dst, symlinks=True)
        return True

    # -- layer cache (keys only: the local builder keeps no per-layer filesystem) -----------
    def _layers_path(self):
        return os.path.join(self.root, "layers.json")

    def layers_seen(self):
        try:
            with open(self._layers_path()) as f:
                return json.load(f)
        except (OSError, ValueError):
            return {}

    def remember_layers(self, keys):
        seen = self.layers_seen()
        seen.update(keys)
        with open(self._layers_path() + ".tmp", "w") as f:
            json.dump(seen, f)
        os.replace(self._layers_path() + ".tmp", self._layers_path())

    def tag(self, src_ref, dst_ref):
        src = self.local(src_ref)
        if not src:
            return False
        dst = self._dir("images", dst_ref)
        if os.path.exists(dst):
            shutil.rmtree(dst)
        shutil.copytree(src, dst, symlinks=True)
        return True


def _parse_dockerfile(text):
    lines, cur = [], ""
    for raw in text.splitlines():
        s = raw.rstrip()
        if not cur and (not s.strip() or s.strip().startswith("#")):
            continue
        if s.endswith("\\"):
            cur += s[:-1] + " "
            continue
        cur += s
        lines.append(cur.strip())
        cur = ""
    if cur.strip():
        lines.append(cur.strip())
    out = []
    for l in lines:
        parts = l.split(None, 1)
        out.append((parts[0].upper(), parts[1] if len(parts) > 1 else ""))
    return out


def _exec_form(arg):
    arg = arg.strip()
    if arg.startswith("["):
        try:
            return json.loads(arg)
        except ValueError:
            pass
    return ["/bin/sh", "-c", arg]


def _content_hash(paths, base):
    """What a COPY/ADD copies, as the classic builder checksums it: relative paths, modes, symlink
    targets and file bytes; mtimes and ownership do not count."""
    h = hashlib.sha256()

    def add(p):
        st = os.lstat(p)
        h.update(os.path.relpath(p, base).encode() + b"\0" + str(st.st_mode).encode() + b"\0")
        if os.path.islink(p):
            h.update(b"L" + os.readlink(p).encode())
        elif os.path.isfile(p):
            with open(p, "rb") as f:
                for chunk in iter(lambda: f.read(1 << 20), b""):
                    h.update(chunk)

    for top in paths:
        if os.path.isdir(top) and not os.path.islink(top):
            for d, dirs, files in os.walk(top):
                dirs.sort()
                add(d)
                for name in sorted(files) + [x for x in dirs if os.path.islink(os.path.join(d, x))]:
                    add(os.path.join(d, name))
        else:
            add(top)
    return h.hexdigest()


def _run_step(argv, rootfs, config, work, log, timeout=900):
    """A RUN on the host runtime: in the image's working directory, with its ENV over the host's
    (the pods run on the host's tools too) and a HOME of the build's own."""
    import subprocess

    cwd = os.path.join(rootfs, config["WorkingDir"].lstrip("/"))
    os.makedirs(cwd, exist_ok=True)
    env = dict(os.environ)
    for kv in config["Env"]:
        k, _, v = kv.partition("=")
        env[k] = v
    env["HOME"] = os.path.join(work, "home")
    os.makedirs(env["HOME"], exist_ok=True)
    log(" ---> Running in the local runtime")
    p = subprocess.run(argv, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    for line in (p.stdout + p.stderr).splitlines():
        log(line)
    if p.returncode != 0:
        raise RuntimeError(f"The command '{' '.join(argv)}' returned a non-zero code: {p.returncode}")


def build_image(store, context_dir, dockerfile, tag, buildargs=None, target=None, log=print):
    with open(os.path.join(context_dir, dockerfile)) as f:
        instrs = _parse_dockerfile(f.read())
    args = dict(buildargs or {})
    stages = {}
    work = tempfile.mkdtemp(prefix="lk-build-")
    rootfs = os.path.join(work, "rootfs")
    os.makedirs(rootfs)
    config = {"Env": [], "Cmd": None, "Entrypoint": None, "WorkingDir": "/", "ExposedPorts": {}, "Labels": {}}
    stage_name = None
    total = len(instrs)
    key = hashlib.sha256(b"scratch").hexdigest()  # the chained cache key of the current step
    layers, history, new_keys = [], [], {}
    seen = store.layers_seen()

    def subst(s):
        env = dict(args)
        for kv in config["Env"]:
            k, _, v = kv.partition("=")
            env[k] = v
        return re.sub(r"\$\{?([A-Za-z_][A-Za-z0-9_]*)\}?", lambda m: env.get(m.group(1), m.group(0)), s)

    for i, (op, arg) in enumerate(instrs, 1):
        log(f"Step {i}/{total} : {op} {arg}")
        copied = None  # COPY/ADD: the content hash of its sources
        if op == "FROM":
            if stage_name and target and stage_name == target:
                break
            parts = arg.split()
            base = subst(parts[0])
            stage_name = parts[2] if len(parts) >= 3 and parts[1].lower() == "as" else None
            shutil.rmtree(rootfs)
            os.makedirs(rootfs)
            config = {"Env": [], "Cmd": None, "Entrypoint": None, "WorkingDir": "/", "ExposedPorts": {}, "Labels": {}}
            if base in stages:
                shutil.copytree(stages[base]["rootfs"], rootfs, dirs_exist_ok=True, symlinks=True)
                config = json.loads(json.dumps(stages[base]["config"]))
                key, layers = stages[base]["key"], list(stages[base]["layers"])
            else:
                img = store.resolve(base)
                if img:
                    shutil.copytree(img["rootfs"], rootfs, dirs_exist_ok=True, symlinks=True)
                    config.update({k: v for k, v in img["config"].items() if k not in ("RootFS", "History")})
                    layers = list((img["config"].get("RootFS") or {}).get("Layers") or [])
                    key = hashlib.sha256(("FROM " + base + "|" + ",".join(layers)).encode()).hexdigest()
                else:
                    log(f" ---> using host runtime for base image {base}")
                    layers = []
                    key = hashlib.sha256(("FROM " + base).encode()).hexdigest()
            history = []
        elif op == "WORKDIR":
            wd = subst(arg)
            config["WorkingDir"] = wd if wd.startswith("/") else os.path.join(config["WorkingDir"], wd)
            os.makedirs(os.path.join(rootfs, config["WorkingDir"].lstrip("/")), exist_ok=True)
        elif op in ("COPY", "ADD"):
            toks = [t for t in shlex.split(subst(arg)) if not t.startswith("--chown") and not t.startswith("--chmod")]
            from_stage = None
            if toks and toks[0].startswith("--from="):
                from_stage = toks.pop(0).split("=", 1)[1]
            if toks and toks[0].startswith("["):
                toks = json.loads(" ".join(toks))
            srcs, dst = toks[:-1], toks[-1]
            base_src = stages[from_stage]["rootfs"] if from_stage in stages else context_dir
            dst_abs = dst if dst.startswith("/") else os.path.join(config["WorkingDir"], dst)
            dst_path = os.path.join(rootfs, dst_abs.lstrip("/"))
            expanded = []
            for s in srcs:
                pat = os.path.join(base_src, s.lstrip("/") if from_stage else s)
                if any(ch in s for ch in "*?["):
                    hits = sorted(glob.glob(pat))
                    if not hits:
                        raise RuntimeError(f"COPY failed: no source files were specified ({s})")
                    expanded.extend(hits)
                    if len(hits) > 1 and not dst.endswith("/"):
                        dst = dst + "/"
                else:
                    expanded.append(pat)
            missing = [os.path.relpath(sp, base_src) for sp in expanded if not os.path.lexists(os.path.normpath(sp))]
            if missing:
                raise RuntimeError(f"COPY failed: stat {missing[0]}: file does not exist")
            copied = _content_hash([os.path.normpath(sp) for sp in expanded], base_src)
            for sp in expanded:
                s = os.path.relpath(sp, base_src)
                sp = os.path.normpath(sp)
                if os.path.isdir(sp):
                    shutil.copytree(sp, dst_path, dirs_exist_ok=True, symlinks=True)
                elif os.path.exists(sp):
                    if dst.endswith("/") or len(srcs) > 1 or os.path.isdir(dst_path):
                        os.makedirs(dst_path, exist_ok=True)
                        shutil.copy2(sp, os.path.join(dst_path, os.path.basename(sp)))
                    else:
                        os.makedirs(os.path.dirname(dst_path), exist_ok=True)
                        shutil.copy2(sp, dst_path)
                else:
                    raise RuntimeError(f"COPY failed: stat {s}: file does not exist")
        elif op == "ENV":
            a = subst(arg)
            if "=" in a.split()[0]:
                for kv in shlex.split(a):
                    k, _, v = kv.partition("=")
                    config["Env"] = [e for e in config["Env"] if not e.startswith(k + "=")] + [f"{k}={v}"]
            else:
                k, _, v = a.partition(" ")
                config["Env"] = [e for e in config["Env"] if not e.startswith(k + "=")] + [f"{k}={v.strip()}"]
        elif op == "ARG":
            k, _, v = arg.partition("=")
            args.setdefault(k.strip(), v.strip())
        elif op == "EXPOSE":
            for p in arg.split():
                config["ExposedPorts"][p if "/" in p else p + "/tcp"] = {}
        elif op == "CMD":
            config["Cmd"] = _exec_form(subst(arg))
        elif op == "ENTRYPOINT":
            config["Entrypoint"] = _exec_form(subst(arg))
        elif op == "LABEL":
            for kv in shlex.split(arg):
                k, _, v = kv.partition("=")
                config["Labels"][k] = v
        elif op == "RUN" and not store.run_steps:
            log(" ---> RUN recorded, not executed by the local builder (no network on this host)")
        if op != "FROM":
            text = f"{op} {subst(arg)}" + (f" content={copied}" if copied else "")
            key = hashlib.sha256((key + "|" + text).encode()).hexdigest()
            fs_layer = op in ("COPY", "ADD", "RUN")
            if op == "RUN" and store.run_steps:
                snap = store.snapshot_dir(key)
                if key in seen and os.path.isdir(snap):
                    # the layer this step made before: its filesystem instead of running it again
                    shutil.rmtree(rootfs)
                    shutil.copytree(snap, rootfs, symlinks=True)
                    os.utime(snap)  # most recently used
                else:
                    _run_step(_exec_form(subst(arg)), rootfs, config, work, log)
                    store.keep_snapshot(key, rootfs)
                    seen.pop(key, None)  # ran: not "Using cache"
            if key in seen:
                log(" ---> Using cache")
            log(f" ---> {key[:12]}")
            if fs_layer:
                layers.append("sha256:" + key)
            history.append({"created_by": f"{op} {arg}", "empty_layer": not fs_layer, "key": key,
                            "cached": key in seen})
            new_keys[key] = f"{op} {arg}"
        if stage_name:
            stages[stage_name] = {"rootfs": rootfs + "-" + stage_name, "config": json.loads(json.dumps(config)),
                                  "key": key, "layers": list(layers)}
            if os.path.exists(stages[stage_name]["rootfs"]):
                shutil.rmtree(stages[stage_name]["rootfs"])
            shutil.copytree(rootfs, stages[stage_name]["rootfs"], symlinks=True)
    config["RootFS"] = {"Type": "layers", "Layers": layers}
    config["History"] = history
    store.save(tag, rootfs, config)
    store.remember_layers(new_keys)
    shutil.rmtree(work, ignore_errors=True)
    return "sha256:" + hashlib.sha256(json.dumps(config, sort_keys=True).encode() + tag.encode()).hexdigest()


def make_app(store: ImageStore):
    app = web.Application(client_max_size=1024 ** 3)

    async def ping(request):
        return web.Response(text="OK")

    async def version(request):
        return web.json_response({"Version": "24.0.0-devspace-local", "ApiVersion": "1.43", "Os": "linux",
                                  "Arch": "amd64"})

    async def info(request):
        return web.json_response({"Name": "devspace-local", "ServerVersion": "24.0.0-devspace-local",
                                  "IndexServerAddress": "https://index.docker.io/v1/"})

    async def auth(request):
        return web.json_response({"Status": "Login Succeeded", "IdentityToken": ""})

    async def build(request):
        q = request.query
        tag = q.get("t", "")
        dockerfile = q.get("dockerfile", "Dockerfile")
        buildargs = json.loads(q.get("buildargs", "{}") or "{}")
        target = q.get("target") or None
        # the context streams in (chunked or sized) to a temp file, as dockerd spools it: a
        # multi-GB context never sits in memory on either side
        ctx = tempfile.mkdtemp(prefix="lk-ctx-")
        spool = tempfile.NamedTemporaryFile(prefix="lk-ctx-", suffix=".tar", delete=False)
        try:
            async for chunk in request.content.iter_chunked(1 << 20):
                spool.write(chunk)
        finally:
            spool.close()
        resp = web.StreamResponse(headers={"Content-Type": "application/json"})
        await resp.prepare(request)

        async def emit(obj):
            await resp.write((json.dumps(obj) + "\r\n").encode())

        try:
            with tarfile.open(spool.name, "r:*") as tf:  # plain or gzip
                tf.extractall(ctx, filter="fully_trusted") if hasattr(tarfile, "data_filter") else tf.extractall(ctx)
            logs = []
            image_id = build_image(store, ctx, dockerfile, tag, buildargs, target, log=logs.append)
            for l in logs:
                await emit({"stream": l + "\n"})
            await emit({"aux": {"ID": image_id}})
            await emit({"stream": f"Successfully built {image_id[7:19]}\n"})
            await emit({"stream": f"Successfully tagged {tag}\n"})
        except Exception as e:
            await emit({"errorDetail": {"message": str(e)}, "error": str(e)})
        finally:
            shutil.rmtree(ctx, ignore_errors=True)
            os.unlink(spool.name)
        await resp.write_eof()
        return resp

    async def push(request):
        name = request.match_info["name"]
        tag = request.query.get("tag", "latest")
        ref = f"{name}:{tag}"
        resp = web.StreamResponse(headers={"Content-Type": "application/json"})
        await resp.prepare(request)
        if store.push(ref):
            await resp.write(json.dumps({"status": f"The push refers to repository [{name}]"}).encode() + b"\r\n")
            await resp.write(json.dumps({"status": "Pushed", "id": tag}).encode() + b"\r\n")
            await resp.write(json.dumps({"status": f"{tag}: digest: sha256:{hashlib.sha256(ref.encode()).hexdigest()} size: 1"}).encode() + b"\r\n")
        else:
            msg = f"An image does not exist locally with the tag: {name}"
            await resp.write(json.dumps({"errorDetail": {"message": msg}, "error": msg}).encode() + b"\r\n")
        await resp.write_eof()
        return resp

    async def tag_image(request):
        name = request.match_info["name"]
        repo, tag = request.query.get("repo"), request.query.get("tag", "latest")
        if not store.tag(name, f"{repo}:{tag}"):
            return web.json_response({"message": f"No such image: {name}"}, status=404)
        return web.Response(status=201)

    async def inspect(request):
        name = request.match_info["name"]
        img = store.resolve(name)
        if not img:
            return web.json_response({"message": f"No such image: {name}"}, status=404)
        cfg = {k: v for k, v in img["config"].items() if k not in ("RootFS", "History")}
        return web.json_response({"Id": "sha256:" + hashlib.sha256(name.encode()).hexdigest(), "Config": cfg,
                                  "RootFS": img["config"].get("RootFS") or {"Type": "layers", "Layers": []},
                                  "RepoTags": [name]})

    async def history(request):
        name = request.match_info["name"]
        img = store.resolve(name)
        if not img:
            return web.json_response({"message": f"No such image: {name}"}, status=404)
        out = [{"Id": "sha256:" + h["key"], "CreatedBy": h["created_by"], "Size": 0,
                "Comment": "cached" if h.get("cached") else ""} for h in img["config"].get("History") or []]
        return web.json_response(list(reversed(out)))  # newest first, as dockerd answers

    for prefix in ("", "/v{ver}"):
        app.router.add_get(prefix + "/_ping", ping)  # add_get also registers HEAD
        app.router.add_get(prefix + "/version", version)
        app.router.add_get(prefix + "/info", info)
        app.router.add_post(prefix + "/auth", auth)
        app.router.add_post(prefix + "/build", build)
        app.router.add_post(prefix + "/images/{name:.+}/push", push)
        app.router.add_post(prefix + "/images/{name:.+}/tag", tag_image)
        app.router.add_get(prefix + "/images/{name:.+}/json", inspect)
        app.router.add_get(prefix + "/images/{name:.+}/history", history)
    return app
