#!/usr/bin/env python3
"""Generates the reference pages under docs/reference/ from the built tool itself, so they
cannot drift from it:

  cli.md            every command's `--help` (walks `devspace <cmd> --help` recursively)
  configuration.md  every key of the strict .devspace/config.yaml schema (v1alpha2), taken from
                    the native module's schema (`_native.config_schema`), with the descriptions
                    kept below (a key without a description, or a description of a key the
                    schema does not have, is an error)
  environment.md    every DEVSPACE_* variable the CLI (src/) and the workload kit
                    (devspace_amd/) read, with the descriptions kept below (same rule)

    python scripts/gen_docs.py           write the pages
    python scripts/gen_docs.py --check   exit 1 if a page differs from what would be written
"""

import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "docs", "reference")
BIN = os.path.join(ROOT, "bin", "devspace")

# ------------------------------------------------------------------------ configuration keys

CONFIG = {
    "version": "Schema version of the file. `v1alpha2` is current; a `v1alpha1` file is upgraded on load "
               "(`devspace update config` rewrites it).",
    "cluster": "Which cluster and namespace to use. Empty: the current kubectl context.",
    "cluster.cloudProvider": "Cloud provider name (`devspace login`, `devspace create space`); kube context and "
                             "namespace then come from the space.",
    "cluster.kubeContext": "kubeconfig context to use instead of the current one.",
    "cluster.namespace": "Default namespace for deployments, sync, ports and terminal.",
    "cluster.apiServer": "API server URL, for a cluster given inline instead of through a kubeconfig context.",
    "cluster.caCert": "PEM CA certificate of an inline cluster.",
    "cluster.user": "Credentials of an inline cluster.",
    "cluster.user.clientCert": "PEM client certificate.",
    "cluster.user.clientKey": "PEM client key.",
    "cluster.user.token": "Bearer token.",
    "dev": "What `devspace dev` starts after building and deploying.",
    "dev.terminal": "The terminal `devspace dev` opens (and `devspace enter` uses by default).",
    "dev.terminal.disabled": "Do not open a terminal; `dev` then attaches to the container output.",
    "dev.terminal.selector": "Name of an entry of `dev.selectors` picking the pod.",
    "dev.terminal.labelSelector": "Label selector picking the pod (the newest running match).",
    "dev.terminal.namespace": "Namespace of the pod.",
    "dev.terminal.containerName": "Container to open the shell in (default: the first one).",
    "dev.terminal.command": "Command to run instead of the default shell (bash if present, else sh).",
    "dev.autoReload": "Paths, deployments and images whose change makes `dev` rebuild and redeploy instead of "
                      "syncing (e.g. Dockerfile, chart, package.json).",
    "dev.autoReload.paths": "Glob patterns (`**` supported) watched for a rebuild + redeploy.",
    "dev.autoReload.deployments": "Deployments whose chart or manifests trigger a redeploy when they change.",
    "dev.autoReload.images": "Images whose Dockerfile triggers a rebuild + redeploy when it changes.",
    "dev.overrideImages": "Entrypoint overrides applied to images built by `dev` (e.g. `sleep` so the container "
                          "idles until you start the app in the terminal).",
    "dev.overrideImages[]": "One override.",
    "dev.overrideImages[].name": "Key of the image in `images`.",
    "dev.overrideImages[].entrypoint": "Entrypoint (and arguments) written into the dev image.",
    "dev.selectors": "Named pod selections that `ports`, `sync` and `terminal` refer to by name.",
    "dev.selectors[]": "One selector.",
    "dev.selectors[].name": "Name the other sections use.",
    "dev.selectors[].namespace": "Namespace of the pods.",
    "dev.selectors[].labelSelector": "Labels the pod must carry; the newest running match is used.",
    "dev.selectors[].containerName": "Container inside the pod (default: the first one).",
    "dev.ports": "Port forwarding from localhost to pods.",
    "dev.ports[]": "One forwarded pod.",
    "dev.ports[].selector": "Name of an entry of `dev.selectors`.",
    "dev.ports[].namespace": "Namespace of the pod.",
    "dev.ports[].labelSelector": "Labels of the pod.",
    "dev.ports[].portMappings": "Local to remote port pairs.",
    "dev.ports[].portMappings[]": "One port pair.",
    "dev.ports[].portMappings[].localPort": "Port to listen on locally.",
    "dev.ports[].portMappings[].remotePort": "Port in the pod (default: the local port).",
    "dev.ports[].portMappings[].bindAddress": "Local address to listen on. Default: localhost on both 127.0.0.1 "
                                              "and ::1; IPv6 literals and host names are accepted.",
    "dev.sync": "Two-way file sync between local paths and containers.",
    "dev.sync[]": "One synced path.",
    "dev.sync[].selector": "Name of an entry of `dev.selectors`.",
    "dev.sync[].namespace": "Namespace of the pod.",
    "dev.sync[].labelSelector": "Labels of the pod.",
    "dev.sync[].containerName": "Container to sync into (default: the first one).",
    "dev.sync[].localSubPath": "Local directory, relative to the project (default: the project root).",
    "dev.sync[].containerPath": "Absolute path in the container.",
    "dev.sync[].excludePaths": "gitignore-style patterns excluded in both directions.",
    "dev.sync[].downloadExcludePaths": "Patterns never downloaded from the container (e.g. build output).",
    "dev.sync[].uploadExcludePaths": "Patterns never uploaded to the container (e.g. local node_modules/).",
    "dev.sync[].bandwidthLimits": "Transfer rate limits of this sync path.",
    "dev.sync[].bandwidthLimits.download": "Container to local, KB/s.",
    "dev.sync[].bandwidthLimits.upload": "Local to container, KB/s.",
    "deployments": "What `deploy` and `dev` deploy, in order (`purge` removes them in reverse order).",
    "deployments[]": "One deployment: a Helm chart or kubectl manifests.",
    "deployments[].name": "Release name (Helm) or label of the deployment.",
    "deployments[].namespace": "Namespace (default: `cluster.namespace`, else the context's).",
    "deployments[].helm": "Deploy a chart with the built-in Helm 3 engine (release stored as a Secret; no Tiller).",
    "deployments[].helm.chartPath": "Chart directory (e.g. `./chart`).",
    "deployments[].helm.wait": "Wait until the release's pods are ready (default true).",
    "deployments[].helm.timeout": "Readiness wait in seconds (default 40, 300 for charts requesting amd.com/gpu).",
    "deployments[].helm.maxHistory": "Release revisions kept (default 10, 0 keeps all), as `helm --history-max`.",
    "deployments[].helm.tillerNamespace": "Accepted for compatibility with Helm 2 configs; ignored (Helm 3 has no "
                                          "Tiller).",
    "deployments[].helm.overrides": "Extra values files merged over the chart's values.yaml, in order.",
    "deployments[].helm.overrideValues": "Inline values merged last.",
    "deployments[].kubectl": "Apply plain manifests (server-side apply through the built-in client).",
    "deployments[].kubectl.cmdPath": "Use this kubectl binary (`apply --force` / `delete`) instead of the built-in "
                                     "client.",
    "deployments[].kubectl.manifests": "Manifest files or globs (`.yaml`/`.yml`); `image:` values naming a "
                                       "configured image are rewritten to the built tag.",
    "images": "Images to build, by key.",
    "images.<name>": "One image.",
    "images.<name>.image": "Repository (e.g. `registry.example.com/team/app`).",
    "images.<name>.tag": "Tag to use instead of a random 7-character tag per build.",
    "images.<name>.createPullSecret": "Create a docker-registry pull secret for this registry in the namespace.",
    "images.<name>.insecure": "Registry served over plain HTTP or with an untrusted certificate.",
    "images.<name>.skipPush": "Build only (e.g. into minikube's Docker daemon); no push.",
    "images.<name>.build": "How the image is built.",
    "images.<name>.build.disabled": "Do not build; deploy the image as is.",
    "images.<name>.build.contextPath": "Build context directory (default: the project root); `.dockerignore` "
                                       "applies.",
    "images.<name>.build.dockerfilePath": "Dockerfile (default `./Dockerfile`).",
    "images.<name>.build.kaniko": "Build in the cluster with kaniko instead of a local Docker daemon.",
    "images.<name>.build.kaniko.cache": "Use kaniko's layer cache (default true).",
    "images.<name>.build.kaniko.namespace": "Namespace of the build pod.",
    "images.<name>.build.kaniko.pullSecret": "Secret with registry credentials for the build pod.",
    "images.<name>.build.kaniko.image": "Executor image of the build pod (default: the reference's pinned "
                                        "`gcr.io/kaniko-project/executor:debug-…`; a debug variant, the build runs "
                                        "by exec in its `/busybox`). `DEVSPACE_KANIKO_IMAGE` when unset.",
    "images.<name>.build.docker": "Docker daemon builds.",
    "images.<name>.build.docker.preferMinikube": "Build in minikube's Docker daemon when the context is minikube "
                                                 "(default true).",
    "images.<name>.build.options": "Docker build options.",
    "images.<name>.build.options.buildArgs": "`--build-arg` values.",
    "images.<name>.build.options.target": "Multi-stage target.",
    "images.<name>.build.options.network": "Network mode of the build's RUN steps.",
}

# ------------------------------------------------------------------------ environment

ENV = {
    # CLI (src/)
    "DEVSPACE_BUILD_PARALLEL": "`0` builds images one after another (default: independent images build "
                               "concurrently).",
    "DEVSPACE_FORCE_COLOR": "Colored console output even when stdout is not a terminal.",
    "DEVSPACE_GITHUB_API": "GitHub API endpoint for `devspace upgrade` release discovery (default "
                           "https://api.github.com).",
    "DEVSPACE_HELM_HOME": "Helm repository cache and repositories file (default `~/.devspace/helm`).",
    "DEVSPACE_HELM_MAX_HISTORY": "Release revisions kept for every Helm deployment (a deployment's "
                                 "`helm.maxHistory` wins).",
    "DEVSPACE_HELPER": "Path of the static in-container sync helper to upload (default: `devspace-helper` next to "
                       "the binary).",
    "DEVSPACE_INIT_NO_NODE_DISCOVERY": "`devspace init` does not read the cluster's nodes to size GPU pods (per-GPU "
                                       "defaults are used).",
    "DEVSPACE_INIT_GPUS": "Answers `devspace init`'s GPU-count question (same as `--gpus`).",
    "DEVSPACE_INIT_IMAGE": "Answers `devspace init`'s image question (same as `--image`); with it, no Docker Hub "
                           "account is needed.",
    "DEVSPACE_INIT_LANGUAGE": "Answers `devspace init`'s language question (same as `--language`).",
    "DEVSPACE_INIT_NAMESPACE": "Answers `devspace init`'s namespace question (same as `--namespace`).",
    "DEVSPACE_INIT_PORT": "Answers `devspace init`'s port question (same as `--port`).",
    "DEVSPACE_INIT_PULL_SECRET": "Answers `devspace init`'s pull-secret question, `yes` or `no` (same as "
                                 "`--pullSecret`).",
    "DEVSPACE_INIT_REGISTRY": "Answers `devspace init`'s registry question (same as `--registry`).",
    "DEVSPACE_NONINTERACTIVE": "Never prompt and never read stdin, whatever it is (an open pipe included): every "
                               "question takes its flag, its `DEVSPACE_INIT_*` variable or its default, or the "
                               "command fails naming what to set (CI); also skips the update check.",
    "DEVSPACE_SCAN_MAX_MS": "Longest interval of the stat-scan file watcher (default 1000).",
    "DEVSPACE_SCAN_MIN_MS": "Shortest interval of the stat-scan file watcher (default 20); the interval otherwise "
                            "follows the scan's cost (at most 5 % of a core).",
    "DEVSPACE_WATCHER": "`scan`: watch sync paths with the portable stat-scan watcher instead of the platform's "
                        "event backend (inotify on Linux). The portable build always scans.",
    "DEVSPACE_KANIKO_IMAGE": "The kaniko executor image for in-cluster builds when the config sets none "
                             "(`images.*.build.kaniko.image`); default the reference's pinned debug build. It must be "
                             "a debug variant (the build runs by exec in its `/busybox` shell).",
    "DEVSPACE_PARENT_PID": "When `devspace`'s parent process has this pid, `devspace` ends (SIGTERM) when that "
                           "parent dies, however it dies: test harnesses and scripts set it so no CLI outlives "
                           "them (`tests/conftest.py`, `bench.py`).",
    "DEVSPACE_PORTFORWARD_VIA": "How forwarded connections reach the pod: `auto` (default) through the sync's "
                                "in-container helper on a remote cluster (tunnel round trip of 5 ms or more; a "
                                "connection the restarting app refuses is held in the pod and made once when it "
                                "listens), else the kubelet's port-forward; `helper` whenever the helper is in the "
                                "container; `kubelet` never through the helper.",
    "DEVSPACE_PORTFORWARD_SPILL_MB": "Disk (MiB, default 1024) a port-forwarded connection through the kubelet's "
                                     "tunnel may use for data its local reader has not taken yet, past 4 MiB in memory "
                                     "(a nameless temp file in $TMPDIR). Kubelets do not enforce SPDY windows, so without "
                                     "it one slow reader holds up the pod's other connections. `0`: no spill.",
    "DEVSPACE_PORTFORWARD_HEDGE": "`1`: a held GET/HEAD/OPTIONS on a remote cluster (tunnel round trip of 5 ms or "
                                  "more) is hedged: a new attempt every third of a round trip while earlier ones are "
                                  "in flight; the app may see the request up to about four times. Default: one "
                                  "stream at a time, each request delivered once.",
    "DEVSPACE_PORTFORWARD_HOLD_MS": "How long a local connection is held while the pod refuses it (its app "
                                    "restarting) before it is dropped; default 3000, 0 drops at once as kubectl "
                                    "does.",
    "DEVSPACE_PORTFORWARD_PREOPEN": "`0`: a held connection does not open its next attempt's stream while the "
                                    "current attempt is in flight.",
    "DEVSPACE_PORTFORWARD_SPARES": "Pre-dialed API-server connections kept for new port-forward streams (0-8, "
                                   "default 2).",
    "DEVSPACE_REFERENCE_TIMING": "`1` reproduces the original DevSpace's waits (1 s pod-discovery sleeps, 5 s "
                                 "rollout polls, no kept-alive connections, no TLS session reuse); used for the "
                                 "benchmark's reference column.",
    "DEVSPACE_PULL_TIMEOUT": "Seconds a rollout wait may last in all while a pod of the release is still pulling "
                             "its image (default 1800); past the chart's timeout the wait goes on only for "
                             "pulls, and a first install whose pull outlasts this is kept, not purged.",
    "DEVSPACE_PORTFORWARD_TUNNEL": "`0`: no multiplexed port-forward tunnel (`SPDY/3.1+portforward.k8s.io`); every "
                                   "forwarded connection gets a WebSocket of its own, as against an API server "
                                   "older than Kubernetes 1.30.",
    "DEVSPACE_PULL_ERROR_GRACE_S": "Seconds an `ErrImagePull`/`ImagePullBackOff` the kubelet may yet get past "
                                   "(a registry timeout, a 5xx) may last before the rollout wait fails (default 30); "
                                   "a missing image, an invalid name or a denied pull fail at once.",
    "DEVSPACE_UNSCHEDULABLE_GRACE_S": "Seconds a pod may stay `Unschedulable` before the rollout wait fails (default "
                                      "10); while the cluster autoscaler reports `TriggeredScaleUp` for the pod the "
                                      "wait runs to the chart's timeout.",
    "DEVSPACE_RELEASE_REPO": "GitHub `owner/repo` whose releases `devspace upgrade` installs.",
    "DEVSPACE_RELEASE_URL": "Plain HTTP(S) release mirror for `devspace upgrade` (`<url>/latest`, "
                            "`<url>/devspace-linux-amd64` and its `.sha256`).",
    "DEVSPACE_ROCM_IMAGE": "Base image `devspace init` writes for rocm-pytorch projects; must carry a concrete tag.",
    "DEVSPACE_SKIP_UPDATE_CHECK": "No daily check for a newer release.",
    "DEVSPACE_STUCK_AFTER_S": "Seconds without the runner's loop coming round (or 50 step periods) after which an "
                              "edit restarts a group stuck in a step (default 60, 0 = never; `--stuck-after`).",
    "DEVSPACE_SYNC_MODE": "Sync protocol: `helper` (default when `devspace-helper` ships next to the binary: "
                          "inotify in the pod, streamed archives; falls back to `fast` where it cannot run), `fast` "
                          "(POSIX tools only, event-driven) or `compat` (the original protocol and timing).",
    "DEVSPACE_SYNC_STOP_WARN_MS": "A sync stop that takes longer than this logs which of its loops are still running and "
    "the step it waits on, to `sync.log` and stderr, every period (default 20000).",
    "DEVSPACE_SYNC_WARN_FILE_MB": "Size above which a synced file is logged as large (default 1024).",
    "DEVSPACE_TRACE": "`0` disables the phase spans written to `.devspace/logs/trace.jsonl`.",
    "DEVSPACE_VAR_<NAME>": "Value of config variable `${NAME}`; no question is asked for it.",
    # workload kit (devspace_amd/), read inside GPU pods
    "DEVSPACE_DIST_BACKEND": "Process-group backend of the runner's ranks (default `nccl`, i.e. RCCL, on GPUs and "
                             "`gloo` on CPUs); `gloo` lets several ranks share one GPU for a rehearsal.",
    "DEVSPACE_GEMM_TUNING": "GEMM kernel selection of the runner: `off` (default), `shipped` (pre-tuned "
                            "gfx950 table) or `online` (tune unseen shapes, persist them).",
    "DEVSPACE_GEMM_TUNING_FILE": "Where `online` GEMM tuning persists its table.",
    "DEVSPACE_GEMM_TUNING_MS": "Time budget per shape of `online` GEMM tuning (default 30).",
    "DEVSPACE_GROUP_TIMEOUT_S": "Seconds a collective of the runner's ranks may wait for every rank (default 600): a "
                                "rank stuck in a step ends the group, which is restarted (`--group-timeout`).",
    "DEVSPACE_RESCUE_DIR": "Set by the runner's supervisor for its ranks: the shared-memory directory of their "
                           "rescue snapshots (removed when the supervisor exits).",
    "DEVSPACE_RESCUE_EVERY_S": "Seconds between the runner's snapshots of the training state in /dev/shm (default "
                               "60, 0 = off): a group restarted after a failure resumes from the newest one "
                               "(`--rescue-every`).",
    "DEVSPACE_RESCUE_RECYCLE": "`0`: a superseded rescue snapshot's file is deleted instead of kept as the spare "
                               "the next snapshot is written into (its shared-memory pages already allocated).",
    "DEVSPACE_RESCUE_ROOT": "Where the runner keeps its rescue snapshot directories (default `/dev/shm`, the "
                            "pod's memory volume).",
    "DEVSPACE_RESCUE_STAGING": "`0`: a rescue snapshot is copied to shared memory at the step boundary even when "
                               "free HBM could hold a device copy written in the background.",
    "DEVSPACE_FUSED_RMSNORM": "`0`: the rocm-pytorch example's standalone RMSNorm runs PyTorch's fused rms_norm "
                              "instead of the gfx950 kernel (default on: 1.64x in device time, 1.03x launched one "
                              "call at a time; the residual add + RMSNorm kernel is always on).",
    "DEVSPACE_RUNNER_WAIT_CALLS": "Extra function names (comma-separated) that the runner's stuck-step rule treats as "
                                  "waits: a main thread inside one that spins the CPU is not making progress "
                                  "(`item`, `synchronize` and the collectives are built in).",
    "DEVSPACE_SUPERVISOR_PID": "Set by the runner's supervisor for its ranks: a rank ends with its supervisor "
                               "(PR_SET_PDEATHSIG, set by the rank itself) and exits at once when it started "
                               "orphaned.",
    "DEVSPACE_RUNNER_DEBUG": "`1`: every runner rank logs the code digest it loaded for each generation.",
    "DEVSPACE_RUNNER_FAULT": "Test-only fault injection of the runner (`mutate-entry-after-read`, `skew-helper`): "
                             "edits racing the ranks' reads, to exercise the code agreement.",
    "DEVSPACE_RUNNER_INPROCESS": "`1`: one rank runs in the runner's own process, without a supervisor (a debugger, "
                                 "a profiler that follows one process); a hard crash then ends the runner.",
    "DEVSPACE_RUNNER_STATUS_FD": "Set by the runner's supervisor for its ranks: the pipe they report `ready` / "
                                 "`fail` on.",
    "DEVSPACE_NPROC": "Training processes the runner starts when the pod requests no GPU (CPU runs).",
    "DEVSPACE_OPS_CACHE": "Where a project's vendored gfx950 ops are compiled and cached (default "
                          "`~/.cache/devspace_amd`).",
    "DEVSPACE_PREEMPT": "`0`: an edit never cuts the in-flight training step short at `ctx.preempt_point()`.",
    "DEVSPACE_PREEMPT_DRAIN_MS": "Steps at least this long (default 20 ms) are drained at a preemption point while "
                                 "the change feed is polled.",
    "DEVSPACE_WARM_STANDBY": "`0`: the runner keeps no second set of rank processes (torch already imported) to "
                             "replace a failed group (`--no-warm-standby`).",
    "DEVSPACE_WATCH_SETTLED": "`0`: the runner reacts to every write event, not only to finished writes.",
    # bundled local cluster (devspace_amd/localkube), set by its kubelet for pods
    "DEVSPACE_CONTAINER_ROOT": "Set by the bundled local cluster's kubelet: the pod container's root directory.",
    "DEVSPACE_LOCAL_IMAGES": "Set by the bundled local cluster's kubelet: its image store (kaniko emulation).",
}

# ------------------------------------------------------------------------ generators


def _help(args):
    r = subprocess.run([BIN] + args + ["--help"], capture_output=True, text=True, timeout=30,
                       env=dict(os.environ, DEVSPACE_SKIP_UPDATE_CHECK="1", DEVSPACE_NONINTERACTIVE="1",
                                NO_COLOR="1"))
    return (r.stdout + r.stderr).rstrip() + "\n"


def _subcommands(text):
    m = re.search(r"Available Commands:\n((?:  \S.*\n)+)", text)
    return [line.split()[0] for line in m.group(1).splitlines()] if m else []


def gen_cli():
    out = ["# CLI reference", "",
           "Generated from `devspace <command> --help` by `scripts/gen_docs.py`; do not edit by hand.", ""]
    todo = [[]]
    while todo:
        path = todo.pop(0)
        text = _help(path)
        title = " ".join(["devspace"] + path)
        out += [f"## `{title}`", "", "```", text.rstrip(), "```", ""]
        subs = [s for s in _subcommands(text) if s not in ("help", "completion")]
        todo = [path + [s] for s in subs] + todo if path else todo + [[s] for s in subs]
    return "\n".join(out)


def _schema_paths(s, p, out):
    k = s["kind"]
    if k == "struct":
        if p:
            out.append((p, "object"))
        for name, sub in s["fields"]:
            _schema_paths(sub, f"{p}.{name}" if p else name, out)
    elif k == "list":
        e = s["elem"]
        if e["kind"] == "struct":
            out.append((p, "list of objects"))
            _schema_paths(e, p + "[]", out)
        else:
            out.append((p, f"list of {e['kind']}s"))
    elif k == "map":
        e = s["elem"]
        if e["kind"] == "struct":
            out.append((p, "map of objects"))
            _schema_paths(e, p + ".<name>", out)
        else:
            out.append((p, f"map of {e['kind']}s"))
    else:
        out.append((p, k))


def gen_config():
    sys.path.insert(0, ROOT)
    from devspace_amd import _native

    paths = []
    _schema_paths(_native.config_schema("latest"), "", paths)
    missing = [p for p, _ in paths if p not in CONFIG]
    stale = sorted(set(CONFIG) - {p for p, _ in paths})
    if missing or stale:
        raise SystemExit(f"config descriptions out of sync with the schema: missing {missing}, stale {stale}")
    out = ["# Configuration reference (`.devspace/config.yaml`, `version: v1alpha2`)", "",
           "Generated from the CLI's strict schema by `scripts/gen_docs.py`; do not edit by hand. Unknown keys are "
           "an error, as in the original (`yaml.UnmarshalStrict`). `[]` marks list elements, `<name>` map keys. "
           "`${VAR}` anywhere in a value is a config variable (asked once, or `DEVSPACE_VAR_<NAME>`; see "
           "[configs and variables](../configuration.md)).", "",
           "| key | type | description |", "|---|---|---|"]
    for p, kind in paths:
        out.append(f"| `{p}` | {kind} | {CONFIG[p]} |")
    return "\n".join(out) + "\n"


def _env_used():
    names = set()
    for base, exts in ((os.path.join(ROOT, "src"), (".cc", ".h")), (os.path.join(ROOT, "devspace_amd"), (".py",))):
        for d, _, files in os.walk(base):
            for f in files:
                if f.endswith(exts):
                    text = open(os.path.join(d, f), errors="replace").read()
                    names.update(re.findall(r"\bDEVSPACE_[A-Z0-9_]*[A-Z0-9]\b", text))
    # the config-variable prefix ("DEVSPACE_VAR_" + name) is documented as one entry
    return {n for n in names if n != "DEVSPACE_VAR" and not n.startswith("DEVSPACE_VAR_")} | {"DEVSPACE_VAR_<NAME>"}


def gen_env():
    used = _env_used()
    missing = sorted(used - set(ENV))
    stale = sorted(set(ENV) - used)
    if missing or stale:
        raise SystemExit(f"environment descriptions out of sync with the sources: missing {missing}, stale {stale}")
    out = ["# Environment variables", "",
           "Every `DEVSPACE_*` variable the CLI and the workload kit read. Generated by `scripts/gen_docs.py` from "
           "the sources; do not edit by hand.", "",
           "| variable | effect |", "|---|---|"]
    for k in sorted(ENV):
        out.append(f"| `{k}` | {ENV[k]} |")
    return "\n".join(out) + "\n"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args(argv)
    pages = {"cli.md": gen_cli(), "configuration.md": gen_config(), "environment.md": gen_env()}
    os.makedirs(OUT, exist_ok=True)
    drift = []
    for name, text in pages.items():
        path = os.path.join(OUT, name)
        old = open(path).read() if os.path.exists(path) else None
        if old != text:
            if a.check:
                drift.append(name)
            else:
                with open(path, "w") as f:
                    f.write(text)
    if drift:
        print("out of date: " + ", ".join(drift) + " (run python scripts/gen_docs.py)", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
