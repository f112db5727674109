"""The ported sync behaviour matrix (sync/sync_config_test.go: TestInitialSync, TestNormalSync with
the remove/rename matrix) over the Kubernetes exec WebSocket transport instead of a local shell —
the "FakeKube" leg of SURVEY §7.9: every shell the engine opens is a `pods/exec` stream to a
pod on the bundled API server, over TLS (wss, client certificates), in all three protocols."""

import json
import os
import subprocess
import time

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def tls_pod(tmp_path_factory):
    from devspace_amd.localkube import LocalCluster

    base = str(tmp_path_factory.mktemp("matrix"))
    cluster = LocalCluster(os.path.join(base, "state"), gpus=0, tls=True).start()
    try:
        kc = cluster.write_kubeconfig(os.path.join(base, "kubeconfig"))
        pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "matrix", "namespace": "default"},
               "spec": {"containers": [{"name": "main", "image": "busybox", "command": ["sleep", "3600"]}]}}
        cluster.store.create("", "pods", "default", pod, "v1")
        deadline = time.time() + 60
        while time.time() < deadline:
            p = cluster.store.get("", "pods", "default", "matrix")
            if (p.get("status") or {}).get("phase") == "Running":
                break
            time.sleep(0.05)
        roots = json.loads(p["metadata"]["annotations"]["devspace.sh/local-roots"])
        yield {"KUBECONFIG": kc, "DS_SYNC_KUBE_NS": "default", "DS_SYNC_KUBE_POD": "matrix",
               "DS_SYNC_KUBE_CONTAINER": "main", "DS_SYNC_KUBE_ROOT": roots["main"]}
    finally:
        cluster.stop()


CASES = ["sync_initial_fast", "sync_initial_helper", "sync_initial_compat", "sync_normal_fast", "sync_normal_helper",
         "sync_normal_compat"]


# DEVSPACE_TESTS_BIN: the same matrix against another build (scripts/ci.sh runs the portable one).
# The scan leg runs the edit matrix with the portable stat-scan watcher in this build too.
@pytest.mark.parametrize("case,watcher", [(c, "native") for c in CASES] +
                         [(c, "scan") for c in CASES if "normal" in c])
def test_sync_matrix_over_exec_websocket(tls_pod, case, watcher, tmp_path):
    env = dict(os.environ, HOME=str(tmp_path), DEVSPACE_WATCHER=watcher, **tls_pod)
    exe = os.environ.get("DEVSPACE_TESTS_BIN") or os.path.join(ROOT, "bin", "devspace_tests")
    p = subprocess.run([exe, case], capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    assert f"PASS {case}" in p.stdout and "1 passed, 0 failed" in p.stdout, p.stdout[-2000:]
