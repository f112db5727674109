"""DEVSPACE_NONINTERACTIVE=1 never reads stdin, and `init` answers every question from flags.

CI runners and `docker exec -i` leave stdin an open pipe that nobody writes to. Every command
below runs with such a pipe (a Popen stdin that is never closed) and must end within 5 s,
either successfully or with a one-line error that names the flag or variable to set.
The reference reads answers from stdin (/root/reference/pkg/util/stdinutil/stdin.go:26-88);
the non-interactive variable and the init flags are this build's additions
(docs/reference/environment.md).
"""

import os
import subprocess
import time

import pytest

from test_e2e_cli import _make_chart_repo


def _run_open_stdin(lk, args, cwd, timeout=5.0, env=None):
    """Runs devspace with stdin an open, silent pipe; returns (rc, output, seconds)."""
    import tempfile

    e = dict(lk.env, DEVSPACE_NONINTERACTIVE="1", DEVSPACE_INIT_NO_NODE_DISCOVERY="1", **(env or {}))
    with tempfile.TemporaryFile("w+") as log:
        t0 = time.monotonic()
        p = subprocess.Popen([lk.bin] + list(args), cwd=cwd, env=e, stdin=subprocess.PIPE, stdout=log,
                             stderr=subprocess.STDOUT, text=True, start_new_session=True)
        try:
            p.wait(timeout=timeout)
            timed_out = False
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
            timed_out = True
        elapsed = time.monotonic() - t0
        p.stdin.close()
        log.seek(0)
        out = log.read()
    if timed_out:
        pytest.fail(f"devspace {' '.join(args)} waited on stdin for more than {timeout} s:\n{out}")
    return p.returncode, out, elapsed


def _project(lk, name):
    proj = os.path.join(lk.base, name)
    os.makedirs(proj, exist_ok=True)
    with open(os.path.join(proj, "index.js"), "w") as f:
        f.write("require('http').createServer((q,s)=>s.end('hi')).listen(3020);\n")
    with open(os.path.join(proj, "package.json"), "w") as f:
        f.write('{"name":"ni","version":"1.0.0","scripts":{"start":"node index.js"}}\n')
    return proj


def test_init_without_an_image_fails_fast_naming_the_flag(localkube):
    proj = _project(localkube, "ni-noimage")
    rc, out, secs = _run_open_stdin(localkube, ["init"], proj)
    assert rc != 0, out
    fatal = [l for l in out.splitlines() if "[fatal]" in l]
    assert len(fatal) == 1 and "--image" in fatal[0] and "DEVSPACE_INIT_IMAGE" in fatal[0], out
    assert secs < 5


def test_init_reset_add_package_purge_never_read_stdin(localkube):
    lk = localkube
    proj = _project(lk, "ni-full")
    rc, out, _ = _run_open_stdin(lk, ["init", "--image", "local.registry/ni", "--namespace", "ni-ns", "--port",
                                      "3020", "--registry", "local.registry", "--pullSecret", "no"], proj)
    assert rc == 0, out
    assert "Project successfully initialized" in out
    cfg = open(os.path.join(proj, ".devspace", "config.yaml")).read()
    assert "image: local.registry/ni" in cfg and "namespace: ni-ns" in cfg and "createPullSecret" not in cfg
    assert "containerPort: 3020" in open(os.path.join(proj, "chart", "values.yaml")).read()

    repo = _make_chart_repo(lk.base)
    helm_home = os.path.join(lk.base, "ni-helm-home")
    os.makedirs(helm_home, exist_ok=True)
    with open(os.path.join(helm_home, "repositories.yaml"), "w") as f:
        f.write(f"apiVersion: v1\nrepositories:\n- name: local\n  url: file://{repo}\n")
    rc, out, _ = _run_open_stdin(lk, ["add", "package", "cache"], proj, env={"DEVSPACE_HELM_HOME": helm_home})
    assert rc == 0 and "Successfully added package cache" in out, out

    rc, out, _ = _run_open_stdin(lk, ["purge"], proj)
    assert rc == 0, out
    rc, out, _ = _run_open_stdin(lk, ["reset"], proj)
    assert rc == 0, out
    assert not os.path.exists(os.path.join(proj, ".devspace"))


def test_init_flags_are_checked_like_answers(localkube):
    proj = _project(localkube, "ni-badflag")
    rc, out, _ = _run_open_stdin(localkube, ["init", "--image", "local.registry/ni", "--language", "cobol"], proj)
    assert rc != 0 and "cobol" in out and "--language" in out, out
    rc, out, _ = _run_open_stdin(localkube, ["init", "--image", "local.registry/ni", "--language", "rocm-pytorch",
                                             "--gpus", "9"], proj)
    assert rc != 0 and "--gpus" in out, out


def test_environment_variables_answer_init(localkube):
    proj = _project(localkube, "ni-env")
    rc, out, _ = _run_open_stdin(localkube, ["init"], proj, env={
        "DEVSPACE_INIT_IMAGE": "local.registry/from-env", "DEVSPACE_INIT_NAMESPACE": "env-ns",
        "DEVSPACE_INIT_LANGUAGE": "javascript"})
    assert rc == 0, out
    cfg = open(os.path.join(proj, ".devspace", "config.yaml")).read()
    assert "image: local.registry/from-env" in cfg and "namespace: env-ns" in cfg


def test_piped_answers_still_work_without_the_variable(localkube):
    """The scripted-answers path the other init tests use: the variable unset, answers on stdin."""
    proj = _project(localkube, "ni-piped")
    env = {k: v for k, v in localkube.env.items() if k != "DEVSPACE_NONINTERACTIVE"}
    env["DEVSPACE_INIT_NO_NODE_DISCOVERY"] = "1"
    p = subprocess.run([localkube.bin, "init"], cwd=proj, env=env, capture_output=True, text=True, timeout=60,
                       input="\npiped-ns\n3020\nlocal.registry\nlocal.registry/piped\nno\n")
    assert p.returncode == 0, p.stdout + p.stderr
    assert "namespace: piped-ns" in open(os.path.join(proj, ".devspace", "config.yaml")).read()
