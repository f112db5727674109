"""End-to-end CLI tests against the bundled local cluster (no GPU needed).

Mirrors the reference's manual/e2e flows (README quickstart: init -> deploy -> dev -> enter ->
logs -> analyze -> purge) with the real `devspace` binary talking REST/WebSocket/Docker-API to
devspace_amd.localkube.
"""

import os
import re
import signal
import time

import pytest

from conftest import ROOT


def wait_for(fn, timeout=30.0, interval=0.05, what="condition"):
    deadline = time.time() + timeout
    last = None
    while time.time() < deadline:
        last = fn()
        if last:
            return last
        time.sleep(interval)
    raise AssertionError(f"timed out waiting for {what} (last={last!r})")


def running(pods):
    return [p for p in pods if (p.get("status") or {}).get("phase") == "Running"
            and not p["metadata"].get("deletionTimestamp")]


def container_root(lk, pod, container=None):
    import json

    c = container or pod["spec"]["containers"][0]["name"]
    return json.loads(pod["metadata"]["annotations"]["devspace.sh/local-roots"])[c]


def test_quickstart_deploy_logs_enter_analyze_purge(localkube):
    lk = localkube
    proj = lk.project("quickstart")
    out = lk.run(["deploy"], proj).stdout
    assert "Successfully deployed!" in out
    import json

    spans = [json.loads(l) for l in open(os.path.join(proj, ".devspace", "logs", "trace.jsonl"))]
    names = {s["span"] for s in spans}
    assert {"image.build", "image.push", "deploy", "deploy.helm_wait"} <= names, names
    assert all(s["dur_us"] >= 0 for s in spans)
    pods = wait_for(lambda: running(lk.pods("quickstart")), what="quickstart pod")
    assert pods[0]["spec"]["containers"][0]["image"].startswith("devspace-local/quickstart:")

    # (check=False: a pod that is briefly not Running between two polls is polled again)
    logs = wait_for(lambda: "listening" in lk.run(["logs"], proj, check=False).stdout
                    and lk.run(["logs"], proj, check=False).stdout, what="app log line")
    assert "Example app listening on port 3000!" in logs

    out = lk.run(["enter", "--", "cat", "package.json"], proj).stdout
    assert '"name": "quickstart"' in out

    out = lk.run(["analyze", "--wait=false"], proj).stdout
    assert "No problems found" in out

    out = lk.run(["status", "deployments"], proj).stdout
    assert "devspace-app" in out and "DEPLOYED" in out.upper()

    # second deploy without changes: image and chart are cached
    out = lk.run(["deploy"], proj).stdout
    assert "Successfully deployed!" in out
    assert "Building image" not in out

    lk.run(["purge"], proj)
    wait_for(lambda: not lk.pods("quickstart"), what="pods deleted")


def test_kubectl_deployment_and_image_rewrite(localkube):
    lk = localkube
    proj = lk.project("quickstart-kubectl")
    lk.run(["deploy"], proj)
    pods = wait_for(lambda: running(lk.pods("quickstart-kubectl")), what="pod")
    image = pods[0]["spec"]["containers"][0]["image"]
    assert re.match(r"devspace-local/quickstart-kubectl:\w+$", image), image
    svc = lk.cluster.store.try_get("", "services", "quickstart-kubectl", "quickstart")
    assert svc and svc["spec"]["ports"][0]["port"] == 80
    lk.run(["purge", "-d", "devspace-default"], proj)
    wait_for(lambda: not lk.pods("quickstart-kubectl"), what="pods deleted")


def test_dev_sync_both_directions_and_clean_exit(localkube):
    lk = localkube
    proj = lk.project("quickstart", "quickstart-dev")
    dev = lk.popen(["dev", "--terminal=false"], proj)
    try:
        pods = wait_for(lambda: running(lk.pods("quickstart")), timeout=60, what="dev pod")
        root = container_root(lk, pods[0])
        # dev mode overrides the entrypoint with sleep
        assert wait_for(lambda: os.path.exists(os.path.join(root, "app", "index.js")), what="initial upload")

        with open(os.path.join(proj, "index.js"), "a") as f:
            f.write("// local edit\n")
        wait_for(lambda: "// local edit" in open(os.path.join(root, "app", "index.js")).read(), what="upstream")

        os.makedirs(os.path.join(proj, "lib"), exist_ok=True)
        with open(os.path.join(proj, "lib", "util.js"), "w") as f:
            f.write("module.exports = 42;\n")
        wait_for(lambda: os.path.exists(os.path.join(root, "app", "lib", "util.js")), what="new dir upstream")

        lk.run(["enter", "--", "sh", "-c", "echo from-pod > from_pod.txt"], proj)
        wait_for(lambda: os.path.exists(os.path.join(proj, "from_pod.txt")), what="downstream")
        assert open(os.path.join(proj, "from_pod.txt")).read().strip() == "from-pod"

        # excluded paths (uploadExcludePaths: chart/) never reach the pod
        with open(os.path.join(proj, "chart", "extra.txt"), "w") as f:
            f.write("x")
        time.sleep(0.5)
        assert not os.path.exists(os.path.join(root, "app", "chart", "extra.txt"))
    finally:
        os.killpg(dev.pid, signal.SIGINT)
        try:
            out, _ = dev.communicate(timeout=30)
        except Exception:
            os.killpg(dev.pid, signal.SIGKILL)
            out, _ = dev.communicate()
    assert "Sync started" in out, out
    status = lk.run(["status", "sync"], proj).stdout
    row = [l for l in status.splitlines() if "/app" in l][0].split()
    assert row[0] == "Stopped" and int(row[-1]) >= 3, status
    lk.run(["purge"], proj)


def test_init_scripted_then_deploy(localkube):
    lk = localkube
    proj = os.path.join(lk.base, "init-node")
    os.makedirs(proj, exist_ok=True)
    with open(os.path.join(proj, "index.js"), "w") as f:
        f.write("require('http').createServer((q,s)=>s.end('hi')).listen(3010, ()=>console.log('up'));\n")
    with open(os.path.join(proj, "package.json"), "w") as f:
        f.write('{"name":"init-node","version":"1.0.0","scripts":{"start":"node index.js"}}\n')
    # language, namespace, port, registry, image name, pull secrets
    answers = "\ninit-ns\n3010\nlocal.registry\nlocal.registry/init-node\nno\n"
    out = lk.run(["init"], proj, input=answers).stdout
    assert "Project successfully initialized" in out
    cfg = open(os.path.join(proj, ".devspace", "config.yaml")).read()
    assert "image: local.registry/init-node" in cfg
    assert "namespace: init-ns" in cfg
    assert "chartPath: ./chart" in cfg
    values = open(os.path.join(proj, "chart", "values.yaml")).read()
    assert "containerPort: 3010" in values and "#image#" not in values
    assert open(os.path.join(proj, "Dockerfile")).read().startswith("FROM node")
    lk.run(["deploy"], proj)
    wait_for(lambda: running(lk.pods("init-ns")), what="init pod")
    lk.run(["purge"], proj)


def test_init_detects_rocm_pytorch_and_requests_gpus(localkube):
    lk = localkube
    proj = os.path.join(lk.base, "init-torch")
    os.makedirs(proj, exist_ok=True)
    with open(os.path.join(proj, "model.py"), "w") as f:
        f.write("import torch\nprint(torch.__version__)\n")
    # language (detected default), gpus, namespace, port, registry, image, pull secret
    answers = "\n2\ntorch-ns\n\nlocal.registry\nlocal.registry/torch\nno\n"
    out = lk.run(["init"], proj, input=answers).stdout
    assert "Project successfully initialized" in out
    assert "FROM rocm/pytorch" in open(os.path.join(proj, "Dockerfile")).read()
    # the workload kit (runner + fused gfx950 ops) is vendored from the package, byte for byte
    for rel in ("runner.py", "ops/fused.py", "ops/fused_ops.hip", "ops/build.py"):
        assert open(os.path.join(proj, "devspace_amd", rel), "rb").read() == \
            open(os.path.join(ROOT, "devspace_amd", rel), "rb").read(), rel
    assert open(os.path.join(proj, "train.py")).read() == open(os.path.join(ROOT, "examples", "rocm-pytorch",
                                                                            "train.py")).read()
    assert 'CMD ["python", "-m", "devspace_amd.runner"' in open(os.path.join(proj, "Dockerfile")).read()
    values = open(os.path.join(proj, "chart", "values.yaml")).read()
    assert re.search(r"gpu: 2\b", values)
    cfg = open(os.path.join(proj, ".devspace", "config.yaml")).read()
    assert "overrideImages" not in cfg  # the training runner keeps running in dev mode

    # The cluster advertises 0 GPUs: the pod stays Pending. With helm wait the deploy times out
    # and the analyze report (install.go analyzeError) explains the scheduling failure.
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = cfg.replace("chartPath: ./chart", "chartPath: ./chart\n    timeout: 3")
    open(cfg_path, "w").write(cfg)
    p = lk.run(["deploy"], proj, check=False, timeout=120)
    assert p.returncode != 0
    assert "amd.com/gpu" in p.stdout + p.stderr, p.stdout + p.stderr
    assert "no node advertises amd.com/gpu" in p.stdout + p.stderr  # pre-deploy capacity check
    # without waiting the release stays and the pending pod can be inspected
    open(cfg_path, "w").write(cfg.replace("timeout: 3", "wait: false"))
    lk.run(["deploy", "-d"], proj, timeout=120)
    pods = wait_for(lambda: lk.pods("torch-ns"), what="gpu pod object")
    c = pods[0]["spec"]["containers"][0]
    assert str(c["resources"]["limits"]["amd.com/gpu"]) == "2"
    env = {e["name"]: e.get("value") for e in c.get("env") or []}
    assert env.get("DEVSPACE_NPROC") == "2"
    assert any(v["name"] == "dshm" for v in pods[0]["spec"]["volumes"])
    report = lk.run(["analyze", "--wait=false", "-n", "torch-ns"], proj, check=False).stdout
    assert "amd.com/gpu" in report
    lk.run(["purge"], proj)


def test_init_8_gpus_sizes_pod_and_analyze_flags_undersized(localkube):
    """`devspace init` of a rocm-pytorch project for 8 GPUs: CPU and memory sized
    per GPU with requests = limits, memory >= memory-backed shm + a host budget per rank, the
    amd.com/gpu NoSchedule toleration, ML sync excludes and a pinned base image tag. Then the
    round-2 sizing (2 CPUs / 4 Gi for 8 GPUs with 128 Gi shm) is flagged by `analyze`."""
    import yaml

    lk = localkube
    proj = os.path.join(lk.base, "init-torch8")
    os.makedirs(proj, exist_ok=True)
    with open(os.path.join(proj, "train.py"), "w") as f:
        f.write("import torch\nprint(torch.__version__)\n")
    answers = "\n8\ntorch8-ns\n\nlocal.registry\nlocal.registry/torch8\nno\n"
    out = lk.run(["init"], proj, input=answers).stdout
    assert "Project successfully initialized" in out
    assert "Sizing the pod for 8 device(s)" in out, out
    values = yaml.safe_load(open(os.path.join(proj, "chart", "values.yaml")))
    comp = values["components"][0]
    res = comp["containers"][0]["resources"]
    assert res["limits"] == {"gpu": 8, "cpu": "96", "memory": "640Gi"}, res
    assert res["requests"] == {"cpu": "96", "memory": "640Gi"}, res
    assert comp["shmPerGPU"] == 16 and comp["hostMemoryPerGPU"] == 64
    df = open(os.path.join(proj, "Dockerfile")).read()
    assert re.search(r"^FROM rocm/pytorch:rocm[\w.]+_pytorch_release_[\d.]+$", df, re.M), df
    cfg = yaml.safe_load(open(os.path.join(proj, ".devspace", "config.yaml")))
    excludes = cfg["dev"]["sync"][0]["excludePaths"]
    for e in ("__pycache__/", "*.pyc", ".ipynb_checkpoints/", "checkpoints/", "*.pt", "*.safetensors", "wandb/", "data/"):
        assert e in excludes, excludes
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    raw = open(cfg_path).read().replace("chartPath: ./chart", "chartPath: ./chart\n    wait: false")
    open(cfg_path, "w").write(raw)
    lk.run(["deploy"], proj, timeout=120)
    pods = wait_for(lambda: lk.pods("torch8-ns"), what="gpu pod object")
    spec = pods[0]["spec"]
    c = spec["containers"][0]
    assert c["resources"]["limits"]["cpu"] == "96" and c["resources"]["requests"]["memory"] == "640Gi"
    assert {"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"} in spec["tolerations"]
    shm = [v for v in spec["volumes"] if v["name"] == "dshm"][0]["emptyDir"]["sizeLimit"]
    assert shm == "128Gi"
    report = lk.run(["analyze", "--wait=false", "-n", "torch8-ns"], proj, check=False).stdout
    assert "OOM" not in report and "CPU(s) for" not in report, report
    # the round-2 defaults: 2 CPUs and 4 Gi for 8 ranks sharing a 128 Gi memory-backed /dev/shm
    values["components"][0]["containers"][0]["resources"] = {"limits": {"gpu": 8, "cpu": "2", "memory": "4Gi"},
                                                            "requests": {"cpu": "2", "memory": "4Gi"}}
    open(os.path.join(proj, "chart", "values.yaml"), "w").write(yaml.safe_dump(values))
    lk.run(["deploy", "-d"], proj, timeout=120)
    wait_for(lambda: [p for p in lk.pods("torch8-ns")
                      if p["spec"]["containers"][0]["resources"]["limits"]["memory"] == "4Gi"], what="resized pod")
    report = lk.run(["analyze", "--wait=false", "-n", "torch8-ns"], proj, check=False).stdout
    assert "OOM-killed" in report and "2 CPU(s) for 8 GPU rank(s)" in report, report
    lk.run(["purge"], proj)


def test_init_rejects_invalid_image_name(localkube):
    lk = localkube
    proj = os.path.join(lk.base, "init-badimg")
    os.makedirs(proj, exist_ok=True)
    with open(os.path.join(proj, "index.js"), "w") as f:
        f.write("console.log(1)\n")
    answers = "\nbad-ns\n3000\nlocal.registry\nlocal.registry//Bad\nno\n"
    p = lk.run(["init"], proj, input=answers, check=False)
    assert p.returncode != 0
    assert "invalid image name" in p.stdout + p.stderr, p.stdout + p.stderr


def test_add_list_remove_config_commands(localkube):
    lk = localkube
    proj = lk.project("quickstart", "quickstart-cfg")
    lk.run(["add", "port", "9090:90", "--selector", "default"], proj)
    lk.run(["add", "sync", "--local", "./src", "--container", "/app/src", "--selector", "default",
            "--exclude", "node_modules/,*.log"], proj)
    lk.run(["add", "selector", "db", "--label-selector", "app=db"], proj)
    lk.run(["add", "deployment", "extra", "--manifests", "kube/*.yaml"], proj)
    lk.run(["add", "image", "worker", "--image", "devspace-local/worker", "--dockerfile", "worker/Dockerfile"],
           proj)
    ports = lk.run(["list", "ports"], proj).stdout
    assert "9090:90" in ports and "13000:3000" in ports
    sync = lk.run(["list", "sync"], proj).stdout
    assert "/app/src" in sync and "node_modules/" in sync
    sels = lk.run(["list", "selectors"], proj).stdout
    assert "app=db" in sels
    cfg = open(os.path.join(proj, ".devspace", "config.yaml")).read()
    assert "name: extra" in cfg and "devspace-local/worker" in cfg

    lk.run(["remove", "port", "9090"], proj)
    lk.run(["remove", "sync", "--container", "/app/src"], proj)
    lk.run(["remove", "selector", "db"], proj)
    lk.run(["remove", "deployment", "extra"], proj)
    lk.run(["remove", "image", "worker"], proj)
    cfg = open(os.path.join(proj, ".devspace", "config.yaml")).read()
    assert "9090" not in cfg and "/app/src" not in cfg and "name: extra" not in cfg and "worker" not in cfg
    assert "13000" in cfg  # untouched entries survive
    lk.run(["update", "config"], proj)


def test_errors_outside_project(localkube, tmp_path):
    p = localkube.run(["deploy"], str(tmp_path), check=False)
    assert p.returncode != 0
    assert "Couldn't find a DevSpace configuration" in (p.stdout + p.stderr)


def test_version_and_help(localkube, tmp_path):
    out = localkube.run(["--version"], str(tmp_path)).stdout
    assert "devspace version" in out
    out = localkube.run(["--help"], str(tmp_path)).stdout
    for cmd in ("init", "deploy", "dev", "enter", "logs", "analyze", "purge", "reset", "add", "list", "remove",
                "status", "use", "update", "create", "login", "install", "upgrade"):
        assert re.search(rf"^\s+{cmd}\s", out, re.M), cmd


@pytest.mark.parametrize("example", ["microservices"])
def test_multi_deployment_example(localkube, example):
    lk = localkube
    proj = lk.project(example)
    # php/apache is not installed on this host: don't wait for that pod to become ready
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = open(cfg_path).read().replace("chartPath: php/chart", "chartPath: php/chart\n    wait: false")
    open(cfg_path, "w").write(cfg)
    lk.run(["deploy"], proj, timeout=120)
    node = wait_for(lambda: running(lk.pods("microservices", "release=devspace-node")), what="node pod")
    assert node[0]["spec"]["containers"][0]["image"].startswith("devspace-local/ms-node:")
    php = wait_for(lambda: lk.pods("microservices", "release=devspace-php"), what="php pod")
    assert php[0]["spec"]["containers"][0]["image"].startswith("devspace-local/ms-php")
    lk.run(["purge"], proj)


def test_kaniko_in_cluster_build(localkube):
    lk = localkube
    proj = lk.project("kaniko")
    env_backup = lk.env.pop("DOCKER_HOST")
    try:
        out = lk.run(["deploy"], proj, timeout=180).stdout
    finally:
        lk.env["DOCKER_HOST"] = env_backup
    assert "with engine 'kaniko'" in out
    assert "Done building image" in out, out
    assert "Kaniko build pod started (gcr.io/kaniko-project/executor:debug-5ac29a97734170a0547fea33b348dc7c328e2f8a)" \
        in out, out  # the reference's executor by default
    pods = wait_for(lambda: running(lk.pods("kaniko", "app.kubernetes.io/component=default")), what="app pod")
    assert pods[0]["spec"]["containers"][0]["image"].startswith("devspace-local/kaniko-app:")
    # the build pod is deleted after the build
    wait_for(lambda: not lk.pods("kaniko", "devspace-build-id"), what="build pod cleanup")
    lk.run(["purge"], proj)


def test_kaniko_executor_image_is_configurable(localkube):
    """the executor is no longer pinned to the reference's 2019 build:
    images.*.build.kaniko.image (or DEVSPACE_KANIKO_IMAGE) names another one."""
    import yaml

    lk = localkube
    proj = lk.project("kaniko", "kaniko-newer")
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = yaml.safe_load(open(cfg_path))
    for img in cfg["images"].values():
        img["build"]["kaniko"]["image"] = "gcr.io/kaniko-project/executor:v1.23.2-debug"
    open(cfg_path, "w").write(yaml.safe_dump(cfg))
    env_backup = lk.env.pop("DOCKER_HOST")
    try:
        out = lk.run(["deploy"], proj, timeout=180).stdout
        assert "Kaniko build pod started (gcr.io/kaniko-project/executor:v1.23.2-debug)" in out, out
        assert "Done building image" in out, out
        # a non-debug executor has no /busybox to exec the build in: said up front
        for img in cfg["images"].values():
            img["build"]["kaniko"]["image"] = "gcr.io/kaniko-project/executor:v1.23.2"
        open(cfg_path, "w").write(yaml.safe_dump(cfg))
        p = lk.run(["deploy", "--force-build"], proj, timeout=180, check=False)
        assert "is not a debug build" in p.stdout + p.stderr, p.stdout + p.stderr
    finally:
        lk.env["DOCKER_HOST"] = env_backup
        lk.run(["purge"], proj, check=False)


def _make_chart_repo(base):
    """file:// helm repository with one chart (cache-0.3.1: a Deployment + Service)."""
    import io
    import tarfile

    repo = os.path.join(base, "chart-repo")
    os.makedirs(repo, exist_ok=True)
    files = {
        "cache/Chart.yaml": "apiVersion: v1\nname: cache\nversion: 0.3.1\nappVersion: 7.2.0\n",
        "cache/values.yaml": "image: devspace-local/cache-server\nport: 6379\n",
        "cache/README.md": "# cache\nSet `cache.port` to change the port.\n",
        "cache/templates/deployment.yaml": (
            "apiVersion: apps/v1\nkind: Deployment\nmetadata:\n  name: {{ .Release.Name }}-cache\n"
            "spec:\n  replicas: 1\n  selector:\n    matchLabels: {app: {{ .Release.Name }}-cache}\n"
            "  template:\n    metadata:\n      labels: {app: {{ .Release.Name }}-cache}\n    spec:\n"
            "      containers:\n      - name: cache\n        image: {{ .Values.image }}\n"
            "        args: [\"--port\", \"{{ .Values.port }}\"]\n"),
    }
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        for name, data in files.items():
            ti = tarfile.TarInfo(name)
            ti.size = len(data.encode())
            tf.addfile(ti, io.BytesIO(data.encode()))
    with open(os.path.join(repo, "cache-0.3.1.tgz"), "wb") as f:
        f.write(buf.getvalue())
    with open(os.path.join(repo, "index.yaml"), "w") as f:
        f.write("apiVersion: v1\nentries:\n  cache:\n  - name: cache\n    version: 0.3.1\n    appVersion: 7.2.0\n"
                "    description: in-memory cache\n    urls: [cache-0.3.1.tgz]\n")
    return repo


def test_add_list_remove_package_from_chart_repo(localkube):
    lk = localkube
    proj = lk.project("quickstart", "quickstart-pkg")
    repo = _make_chart_repo(lk.base)
    helm_home = os.path.join(lk.base, "helm-home")
    os.makedirs(helm_home, exist_ok=True)
    with open(os.path.join(helm_home, "repositories.yaml"), "w") as f:
        f.write(f"apiVersion: v1\nrepositories:\n- name: local\n  url: file://{repo}\n")
    lk.env["DEVSPACE_HELM_HOME"] = helm_home
    try:
        listing = lk.run(["add", "package"], proj).stdout
        assert "cache" in listing and "0.3.1" in listing
        out = lk.run(["add", "package", "cache"], proj, input="yes\n").stdout
        assert "Successfully added package cache" in out
        assert "Set `cache.port`" in out  # README shown
        chart = os.path.join(proj, "chart")
        assert os.path.exists(os.path.join(chart, "charts", "cache-0.3.1.tgz"))
        assert "name: cache" in open(os.path.join(chart, "requirements.yaml")).read()
        assert "\ncache:" in open(os.path.join(chart, "values.yaml")).read()
        assert "name: cache" in open(os.path.join(proj, ".devspace", "config.yaml")).read()
        assert "cache" in lk.run(["list", "packages"], proj).stdout
        p = lk.run(["add", "package", "cache", "--skip-question"], proj, check=False)
        assert p.returncode != 0 and "already added" in p.stdout + p.stderr

        cfg_path = os.path.join(proj, ".devspace", "config.yaml")
        cfg = open(cfg_path).read().replace("chartPath: ./chart", "chartPath: ./chart\n    wait: false")
        open(cfg_path, "w").write(cfg)
        lk.run(["deploy"], proj)
        dep = lk.cluster.store.try_get("apps", "deployments", "quickstart", "devspace-app-cache")
        assert dep is not None
        assert dep["spec"]["template"]["spec"]["containers"][0]["args"] == ["--port", "6379"]

        lk.run(["remove", "package", "cache"], proj)
        assert not os.path.exists(os.path.join(chart, "charts", "cache-0.3.1.tgz"))
        assert "cache" not in open(os.path.join(chart, "requirements.yaml")).read()
        lk.run(["purge"], proj)
    finally:
        lk.env.pop("DEVSPACE_HELM_HOME", None)


def test_minikube_example_builds_in_minikube_daemon(tmp_path):
    """examples/minikube: kube context `minikube` -> the image is built by minikube's Docker
    daemon (`minikube docker-env`, builder/docker/client.go) and not pushed (skipPush)."""
    from devspace_amd.localkube import LocalCluster

    from conftest import DevspaceEnv

    base = str(tmp_path)
    cluster = LocalCluster(os.path.join(base, "state"), gpus=0, context="minikube").start()
    try:
        lk = DevspaceEnv(cluster, base)
        shim = tmp_path / "shim"
        shim.mkdir()
        (shim / "minikube").write_text(
            "#!/bin/sh\n[ \"$1\" = docker-env ] || exit 1\n"
            f"echo DOCKER_HOST=unix://{cluster.docker_sock}\necho MINIKUBE_ACTIVE_DOCKERD=minikube\n")
        (shim / "minikube").chmod(0o755)
        lk.env.pop("DOCKER_HOST")  # only `minikube docker-env` knows where the daemon is
        lk.env["PATH"] = f"{shim}:{lk.env['PATH']}"
        proj = lk.project("minikube")
        out = lk.run(["deploy"], proj, timeout=120).stdout
        assert "Skip image push for devspace" in out, out
        pods = wait_for(lambda: running(lk.pods("devspace")), what="minikube example pod")
        assert pods[0]["spec"]["containers"][0]["image"].startswith("devspace:"), pods[0]["spec"]
        # never pushed: the registry side of the image store stays empty
        assert not cluster.images.resolve("registry.invalid/devspace")
        lk.run(["purge"], proj)
    finally:
        cluster.stop()


def test_analyze_reports_crash_loop_with_gpu_runtime_error(localkube):
    """A container that keeps failing with a HIP error: analyze reports the restarts, the last
    exit code, the crash log and the ROCm/HIP/RCCL error line (reference: analyze/pods.go
    getContainerProblem; the GPU line is the MI355X delta)."""
    lk = localkube
    proj = lk.project("quickstart-kubectl", "crashing-gpu-app")
    path = os.path.join(proj, "kube", "deployment.yaml")
    src = open(path).read().replace(
        "        ports:\n",
        "        command: [\"sh\", \"-c\", \"echo 'loading model'; echo 'RuntimeError: HIP error: "
        "hipErrorNoBinaryForGpu' >&2; exit 3\"]\n        ports:\n", 1)
    assert "hipErrorNoBinaryForGpu" in src
    open(path, "w").write(src)
    cfg = os.path.join(proj, ".devspace", "config.yaml")
    text = open(cfg).read().replace("namespace: quickstart-kubectl", "namespace: crashing-gpu-app")
    with open(cfg, "w") as f:
        f.write(text)
    lk.run(["deploy"], proj)

    def restarted():
        for p in lk.pods("crashing-gpu-app"):
            for c in (p.get("status") or {}).get("containerStatuses") or []:
                if c.get("restartCount", 0) >= 1 and c.get("lastState", {}).get("terminated"):
                    return True
        return False

    wait_for(restarted, timeout=60, what="a restarted container")
    out = lk.run(["analyze", "--wait=false"], proj, check=False).stdout
    assert "Restarts:" in out and "Last Exit:" in out and "Code: 3" in out, out
    assert "hipErrorNoBinaryForGpu" in out, out  # the crash log tail
    assert "failed with a ROCm/HIP/RCCL error: HIP error" in out, out
    assert "the pod requests no amd.com/gpu" in out, out  # the likely cause, named
    lk.run(["purge"], proj)


def test_create_pull_secret_from_docker_credentials(localkube):
    """images.*.createPullSecret (/root/reference/pkg/devspace/registry/init.go:24-84): with
    credentials for the image's registry in the Docker config, `devspace deploy` creates a
    kubernetes.io/dockerconfigjson secret `devspace-auth-<registry>` in the deployment's
    namespace, the chart's pods get it as an imagePullSecret, and a later deploy with new
    credentials updates the secret in place. Without credentials no secret is written.
    A secret created after the first deploy reaches the release: the redeploy decision includes
    the chart's computed values (the reference's looks at the chart and override files only,
    deploy/helm/deploy.go:64), so does an edit of helm.overrideValues."""
    import base64
    import json

    lk = localkube
    proj = lk.project("quickstart", "quickstart-pullsecret")
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = open(cfg_path).read().replace("namespace: quickstart", "namespace: qs-pull")
    cfg = cfg.replace("    image: devspace-local/quickstart", "    image: devspace-local/quickstart\n    createPullSecret: true")
    assert "createPullSecret: true" in cfg
    open(cfg_path, "w").write(cfg)
    dcfg = os.path.join(lk.base, "dockercfg-pull")
    os.makedirs(dcfg, exist_ok=True)

    def creds(user, pw):
        auth = base64.b64encode(f"{user}:{pw}".encode()).decode()
        with open(os.path.join(dcfg, "config.json"), "w") as f:
            json.dump({"auths": {"https://index.docker.io/v1/": {"auth": auth}}}, f)

    def secret_auth():
        secrets = [s for s in lk.cluster.store.list("", "secrets", "qs-pull")
                   if s["metadata"]["name"] == "devspace-auth-docker"]
        if not secrets:
            return None
        assert secrets[0]["type"] == "kubernetes.io/dockerconfigjson"
        doc = json.loads(base64.b64decode(secrets[0]["data"][".dockerconfigjson"]))
        (entry,) = doc["auths"].values()
        return base64.b64decode(entry["auth"]).decode()

    saved = dict(lk.env)
    try:
        lk.env["DOCKER_CONFIG"] = dcfg
        os.makedirs(os.path.join(dcfg, "empty"), exist_ok=True)
        with open(os.path.join(dcfg, "config.json"), "w") as f:
            json.dump({"auths": {}}, f)
        lk.run(["deploy"], proj)
        assert secret_auth() is None  # no credentials for Docker Hub: nothing to write

        creds("alice", "s3cret")
        out = lk.run(["deploy"], proj).stdout
        assert "Successfully deployed!" in out
        assert secret_auth() == "alice:s3cret"
        dep = lk.cluster.store.list("apps", "deployments", "qs-pull")[0]
        assert {"name": "devspace-auth-docker"} in dep["spec"]["template"]["spec"]["imagePullSecrets"]

        creds("alice", "rotated")
        out = lk.run(["deploy"], proj).stdout
        assert secret_auth() == "alice:rotated"
        assert "Skipping chart" in out  # same secret name, same values: the release stays

        # an edit of helm.overrideValues in the config reaches the release without a chart edit
        cfg = open(cfg_path).read().replace("chartPath: ./chart",
                                            "chartPath: ./chart\n    overrideValues:\n      pullSecrets:\n      - team-registry", 1)
        open(cfg_path, "w").write(cfg)
        out = lk.run(["deploy"], proj).stdout
        assert "Skipping chart" not in out, out
        dep = lk.cluster.store.list("apps", "deployments", "qs-pull")[0]
        names = [s["name"] for s in dep["spec"]["template"]["spec"]["imagePullSecrets"]]
        assert names == ["team-registry", "devspace-auth-docker"], names
    finally:
        lk.env.clear()
        lk.env.update(saved)
        lk.run(["purge"], proj, check=False)


def test_pull_secret_credentials_from_a_credential_helper(localkube):
    """Docker credential helpers (`credsStore` / `credHelpers` in the Docker config, the
    docker-credential-<name> protocol: the server URL on stdin of `get`, JSON with Username and
    Secret on stdout) feed createPullSecret the same way stored auths do
    (/root/reference/pkg/devspace/docker/auth.go via the Docker CLI config)."""
    import base64
    import json
    import stat

    lk = localkube
    proj = lk.project("quickstart", "quickstart-credhelper")
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    cfg = open(cfg_path).read().replace("namespace: quickstart", "namespace: qs-helper")
    cfg = cfg.replace("    image: devspace-local/quickstart", "    image: devspace-local/quickstart\n    createPullSecret: true")
    open(cfg_path, "w").write(cfg)
    dcfg = os.path.join(lk.base, "dockercfg-helper")
    bindir = os.path.join(lk.base, "credhelper-bin")
    os.makedirs(dcfg, exist_ok=True)
    os.makedirs(bindir, exist_ok=True)
    seen = os.path.join(lk.base, "credhelper-seen.txt")
    helper = os.path.join(bindir, "docker-credential-fake")
    with open(helper, "w") as f:
        f.write("#!/bin/sh\n"
                "[ \"$1\" = get ] || exit 1\n"
                f"cat > {seen}\n"
                "printf '{\"ServerURL\":\"https://index.docker.io/v1/\",\"Username\":\"carol\",\"Secret\":\"from-helper\"}'\n")
    os.chmod(helper, os.stat(helper).st_mode | stat.S_IEXEC)
    with open(os.path.join(dcfg, "config.json"), "w") as f:
        json.dump({"auths": {}, "credsStore": "fake"}, f)
    saved = dict(lk.env)
    try:
        lk.env["DOCKER_CONFIG"] = dcfg
        lk.env["PATH"] = bindir + os.pathsep + lk.env.get("PATH", "")
        lk.run(["deploy"], proj)
        assert "index.docker.io" in open(seen).read()
        (secret,) = [s for s in lk.cluster.store.list("", "secrets", "qs-helper")
                     if s["metadata"]["name"] == "devspace-auth-docker"]
        doc = json.loads(base64.b64decode(secret["data"][".dockerconfigjson"]))
        (entry,) = doc["auths"].values()
        assert base64.b64decode(entry["auth"]).decode() == "carol:from-helper"
    finally:
        lk.env.clear()
        lk.env.update(saved)
        lk.run(["purge"], proj, check=False)
