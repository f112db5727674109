"""CLI surface parity with the reference (one row per command), plus the
multi-config commands (`list configs`, `use config`, `list vars`) and the offline
`install`/`upgrade`/`update config` paths that the e2e suites do not reach.

Reference command registrations: cmd/init.go:67-105, cmd/deploy.go:38-64, cmd/dev.go:71-120,
cmd/enter.go:33-61, cmd/logs.go:25-56, cmd/analyze.go:21-47, cmd/purge.go:34-62,
cmd/reset.go:39-61, cmd/login.go:16-41, cmd/add/*.go, cmd/create/space.go:21-45,
cmd/list/list.go:20-26, cmd/remove/remove.go:20-28, cmd/status/status.go:20-21,
cmd/update/update.go:20, cmd/use/use.go:20-23. Config files: config/configs/schema.go:4-31,
config/configutil/get.go:193-221, config/configutil/load.go:23-72.
"""

import json
import os
import re
import shutil
import subprocess

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.environ.get("DEVSPACE_BIN") or os.path.join(ROOT, "bin", "devspace")

# (command path, [(long flag, shorthand or None, default or None)]) — SURVEY.md §2.4.
# `init --cloud` deliberately defaults to false (the hosted service is gone; PARITY.md).
SURFACE = [
    ("init", [("reconfigure", "r", None), ("overwrite", "o", None), ("templateRepoUrl", None, None),
              ("templateRepoPath", None, None), ("cloud", None, None)]),
    ("deploy", [("namespace", None, None), ("kube-context", None, None), ("config", None, ".devspace/config.yaml"),
                ("docker-target", None, None), ("switch-context", None, None), ("force-build", "b", None),
                ("force-deploy", "d", None)]),
    ("dev", [("init-registries", None, "true"), ("force-build", "b", None), ("force-deploy", "d", None),
             ("skip-pipeline", "x", None), ("sync", None, "true"), ("verbose-sync", None, None),
             ("portforwarding", None, "true"), ("terminal", None, "true"), ("selector", "s", None),
             ("container", "c", None), ("label-selector", "l", None), ("namespace", "n", None),
             ("switch-context", None, None), ("exit-after-deploy", None, None), ("config", None, None)]),
    ("up", [("force-build", "b", None), ("sync", None, "true")]),
    ("enter", [("selector", "s", None), ("container", "c", None), ("label-selector", "l", None),
               ("namespace", "n", None), ("switch-context", None, None), ("pick", "p", None), ("config", None, None)]),
    ("logs", [("selector", "s", None), ("container", "c", None), ("label-selector", "l", None),
              ("namespace", "n", None), ("pick", "p", None), ("follow", "f", None), ("lines", None, "200"),
              ("config", None, None)]),
    ("analyze", [("namespace", "n", None), ("wait", None, "true")]),
    ("purge", [("deployment", "d", None), ("config", None, None)]),
    ("down", [("deployment", "d", None)]),
    ("reset", [("config", None, None)]),
    ("install", []),
    ("upgrade", []),
    ("login", [("token", None, None), ("provider", None, "app.devspace.cloud")]),
    ("add sync", [("local", None, None), ("container", None, None), ("label-selector", None, None),
                  ("namespace", None, None), ("exclude", None, None), ("selector", None, None)]),
    ("add selector", [("namespace", None, None), ("label-selector", None, None)]),
    ("add provider", [("name", None, None)]),
    ("add port", [("namespace", None, None), ("label-selector", None, None), ("selector", None, None)]),
    ("add package", [("app-version", None, None), ("chart-version", None, None), ("deployment", "d", None),
                     ("skip-question", None, None)]),
    ("add image", [("image", None, None), ("tag", None, None), ("context", None, None), ("dockerfile", None, None),
                   ("buildengine", None, None)]),
    ("add deployment", [("namespace", None, None), ("manifests", None, None), ("chart", None, None)]),
    ("create space", [("context", None, "true"), ("active", None, "true")]),
    ("list sync", []), ("list spaces", [("name", None, None)]), ("list selectors", []), ("list ports", []),
    ("list packages", []), ("list configs", []), ("list vars", []),
    ("remove context", [("all", None, None)]), ("remove deployment", [("all", None, None)]),
    ("remove image", [("all", None, None)]), ("remove package", [("all", None, None)]),
    ("remove port", [("label-selector", None, None), ("all", None, None)]),
    ("remove provider", []), ("remove selector", [("all", None, None)]),
    ("remove space", [("id", None, None), ("provider", None, None), ("all", None, None)]),
    ("remove sync", [("local", None, None), ("container", None, None), ("label-selector", None, None),
                     ("all", None, None)]),
    ("status sync", []), ("status deployments", []),
    ("update config", []),
    ("use config", []), ("use space", [("context", None, "true")]), ("use registry", []), ("use context", []),
]


def _help(path):
    p = subprocess.run([BIN] + path.split() + ["--help"], capture_output=True, text=True, timeout=30,
                       env=dict(os.environ, DEVSPACE_NONINTERACTIVE="1"))
    assert p.returncode == 0, f"devspace {path} --help failed: {p.stdout}{p.stderr}"
    return p.stdout + p.stderr


@pytest.mark.parametrize("path,flags", SURFACE, ids=[s[0].replace(" ", "_") for s in SURFACE])
def test_command_and_flags_exist(path, flags):
    out = _help(path)
    assert f"devspace {path}" in out, out
    for long, short, default in flags:
        # cobra-style line: "  -b, --force-build   ..." or "      --sync   ... (default true)"
        pat = (rf"^\s+-{short}, --{re.escape(long)}\b" if short else rf"^\s+--{re.escape(long)}\b")
        lines = [l for l in out.splitlines() if re.search(pat, l)]
        assert lines, f"devspace {path}: flag --{long}" + (f"/-{short}" if short else "") + f" missing\n{out}"
        if default is not None:
            assert f'(default {default})' in lines[0] or f'(default "{default}")' in lines[0], lines[0]


def _project(tmp_path):
    proj = tmp_path / "proj"
    shutil.copytree(os.path.join(ROOT, "examples", "quickstart"), proj, symlinks=True)
    return str(proj)


def _run(args, cwd, home, env=None, check=True):
    e = dict(os.environ, HOME=home, DEVSPACE_NONINTERACTIVE="1")
    e.update(env or {})
    p = subprocess.run([BIN] + args, cwd=cwd, env=e, capture_output=True, text=True, timeout=60)
    if check:
        assert p.returncode == 0, f"devspace {' '.join(args)} rc={p.returncode}\n{p.stdout}{p.stderr}"
    return p


def test_multi_config_list_use_and_vars(tmp_path):
    """configs.yaml with a data override and a ${VAR}: list configs, use config, list vars
    (DEVSPACE_VAR_<NAME> resolves the variable; the answer is cached in generated.yaml)."""
    proj = _project(tmp_path)
    home = str(tmp_path / "home")
    os.makedirs(home)
    dsdir = os.path.join(proj, ".devspace")
    configs = {
        "default": {"config": {"path": ".devspace/config.yaml"}},
        "staging": {
            "config": {"path": ".devspace/config.yaml"},
            "vars": {"data": [{"name": "NS", "question": "Namespace?"}]},
            "overrides": [{"data": {"cluster": {"namespace": "${NS}"}}}],
        },
    }
    with open(os.path.join(dsdir, "configs.yaml"), "w") as f:
        yaml.safe_dump(configs, f)

    out = _run(["list", "configs"], proj, home).stdout
    rows = {l.split()[0]: l.split() for l in out.splitlines() if l.strip().startswith(("default", "staging"))}
    assert set(rows) == {"default", "staging"}, out
    assert rows["staging"][2:] == [".devspace/config.yaml", "true", "1"], out

    out = _run(["use", "config", "staging"], proj, home).stdout
    assert "Successfully switched to config 'staging'" in out
    gen = yaml.safe_load(open(os.path.join(dsdir, "generated.yaml")))
    assert gen["activeConfig"] == "staging"
    active = [l for l in _run(["list", "configs"], proj, home).stdout.splitlines() if "staging" in l][0]
    assert "true" in active.split()[1]

    out = _run(["list", "vars"], proj, home, env={"DEVSPACE_VAR_NS": "team-a"}).stdout
    assert re.search(r"NS\s+team-a", out), out
    # cached answer is reused without the env var
    out = _run(["list", "vars"], proj, home).stdout
    assert re.search(r"NS\s+team-a", out), out

    p = _run(["use", "config", "nope"], proj, home, check=False)
    assert p.returncode != 0 and "does not exist" in p.stdout + p.stderr


def test_update_config_rewrites_v1alpha1(tmp_path):
    """`update config` re-saves a v1alpha1 config in the latest schema (cmd/update/config.go)."""
    proj = _project(tmp_path)
    home = str(tmp_path / "home")
    os.makedirs(home)
    cfg_path = os.path.join(proj, ".devspace", "config.yaml")
    # v1alpha1 layout (config/versions/v1alpha1/schema.go): everything dev-related under
    # `devSpace`, images reference `registries` by name, helm `devOverwrite`
    old = {
        "version": "v1alpha1",
        "devSpace": {
            "deployments": [{"name": "app", "helm": {"chartPath": "chart/", "devOverwrite": "dev-values.yaml"}}],
            "services": [{"name": "default", "labelSelector": {"app": "web"}}],
            "ports": [{"service": "default", "portMappings": [{"localPort": 3000, "remotePort": 3000}]}],
        },
        "images": {"default": {"name": "web", "registry": "local"}},
        "registries": {"local": {"url": "registry.local:5000"}},
    }
    with open(cfg_path, "w") as f:
        yaml.safe_dump(old, f)
    out = _run(["update", "config"], proj, home).stdout
    assert "Successfully converted" in out
    new = yaml.safe_load(open(cfg_path))
    assert new["version"] == "v1alpha2"
    assert "devSpace" not in new and "registries" not in new
    assert new["deployments"][0]["helm"]["overrides"] == ["dev-values.yaml"]
    assert new["images"]["default"]["image"] == "registry.local:5000/web"
    assert new["dev"]["selectors"][0]["name"] == "default"
    assert new["dev"]["ports"][0]["selector"] == "default"
    # the rewritten file loads strictly under the latest schema
    assert "default" in _run(["list", "selectors"], proj, home).stdout


def test_install_adds_path_idempotently(tmp_path):
    home = str(tmp_path / "home")
    os.makedirs(home)
    open(os.path.join(home, ".bashrc"), "w").write("# rc\n")
    for _ in range(2):
        out = _run(["install"], str(tmp_path), home).stdout + ""
    rc = open(os.path.join(home, ".bashrc")).read()
    assert rc.count("added by devspace install") == 1, rc
    assert os.path.dirname(os.path.realpath(BIN)) in rc or os.path.dirname(BIN) in rc
    assert "added by devspace install" in open(os.path.join(home, ".profile")).read()
    assert out is not None


def test_upgrade_from_local_release(tmp_path):
    """`upgrade --from <binary>`: replaces the running binary only when the candidate is newer."""
    home = str(tmp_path / "home")
    os.makedirs(home)
    exe = tmp_path / "devspace"
    shutil.copy2(BIN, exe)
    ver = subprocess.run([str(exe), "version"], capture_output=True, text=True).stdout.split()
    assert ver[:2] == ["devspace", "version"] and ver[-1] == "(devspace-mi355x)", ver
    # a "newer release": a script that reports a higher version of this product
    newer = tmp_path / "devspace-next"
    newer.write_text("#!/bin/sh\necho 'devspace version v99.0.0 (devspace-mi355x)'\n")
    newer.chmod(0o755)
    # another product's binary (an upstream devspace) is refused whatever its version
    upstream = tmp_path / "devspace-upstream"
    upstream.write_text("#!/bin/sh\necho 'devspace version v5.18.5'\n")
    upstream.chmod(0o755)
    p = subprocess.run([str(exe), "upgrade", "--from", str(upstream)], capture_output=True, text=True,
                       env=dict(os.environ, HOME=home), timeout=60, cwd=tmp_path)
    assert p.returncode != 0 and "is not a devspace-mi355x binary" in p.stdout + p.stderr, p.stdout + p.stderr
    same = subprocess.run([str(exe), "upgrade", "--from", str(exe)], capture_output=True, text=True,
                          env=dict(os.environ, HOME=home), timeout=60, cwd=tmp_path)
    assert same.returncode == 0 and "latest version" in same.stdout + same.stderr, same.stdout + same.stderr
    p = subprocess.run([str(exe), "upgrade", "--from", str(newer)], capture_output=True, text=True,
                       env=dict(os.environ, HOME=home), timeout=60, cwd=tmp_path)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "Successfully updated to version v99.0.0" in p.stdout + p.stderr
    assert "v99.0.0" in subprocess.run([str(exe)], capture_output=True, text=True).stdout
    assert ver
    # no release channel configured: never the upstream repository, a clear error instead
    clean = {k: v for k, v in os.environ.items() if k not in ("DEVSPACE_RELEASE_URL", "DEVSPACE_RELEASE_REPO")}
    no_ch = subprocess.run([BIN, "upgrade"], capture_output=True, text=True, env={**clean, "HOME": home},
                           timeout=60, cwd=tmp_path)
    assert no_ch.returncode != 0 and "no release channel" in no_ch.stdout + no_ch.stderr, no_ch.stdout + no_ch.stderr
    # no reachable release server: a clear error, not a hang
    no_src = subprocess.run([BIN, "upgrade"], capture_output=True, text=True,
                            env={**clean, "HOME": home, "DEVSPACE_RELEASE_REPO": "acme/devspace-mi355x",
                                 "DEVSPACE_GITHUB_API": "http://127.0.0.1:9"},
                            timeout=60, cwd=tmp_path)
    assert no_src.returncode != 0 and "Couldn't upgrade" in no_src.stdout + no_src.stderr


class _FakeGithub:
    """GitHub releases API + asset downloads (redirected, as GitHub does to object storage)."""

    def __init__(self, releases, files):
        import http.server
        import threading

        outer = self
        self.releases, self.files, self.hits = releases, files, []

        class H(http.server.BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                outer.hits.append((self.path, self.headers.get("User-Agent"), self.headers.get("Authorization")))
                if self.path.startswith("/repos/acme/devspace-mi355x/releases"):
                    body = json.dumps(outer.releases).encode()
                    self.send_response(200)
                    self.send_header("Content-Type", "application/json")
                elif self.path.startswith("/dl/"):
                    self.send_response(302)
                    self.send_header("Location", "/blob/" + self.path[4:])
                    self.send_header("Content-Length", "0")
                    self.end_headers()
                    return
                elif self.path.startswith("/blob/") and self.path[6:] in outer.files:
                    body = outer.files[self.path[6:]]
                    self.send_response(200)
                else:
                    body = b"not found"
                    self.send_response(404)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def close(self):
        self.srv.shutdown()


def _release(tag, assets, base, draft=False, prerelease=False):
    return {"tag_name": tag, "name": tag, "body": f"notes for {tag}", "draft": draft, "prerelease": prerelease,
            "assets": [{"name": a, "browser_download_url": f"{base}/dl/{a}"} for a in assets]}


def test_upgrade_from_github_releases(tmp_path):
    """`upgrade` from this product's release channel: newest non-draft, non-prerelease release
    with a linux/amd64 asset (go-github-selfupdate rules) whose SHA-256 matches the published
    checksums, tarball extracted, running binary swapped atomically; an upstream devspace
    binary, a checksum mismatch or a release without checksums are refused."""
    import hashlib
    import io
    import tarfile

    home = str(tmp_path / "home")
    os.makedirs(home)
    exe = tmp_path / "devspace"
    shutil.copy2(BIN, exe)
    new_bin = open(BIN, "rb").read() + b"\n# release v2.5.0\n"  # still a runnable ELF
    tgz = io.BytesIO()
    with tarfile.open(fileobj=tgz, mode="w:gz") as tf:
        ti = tarfile.TarInfo("devspace-v2.5.0/devspace")
        ti.size, ti.mode = len(new_bin), 0o755
        tf.addfile(ti, io.BytesIO(new_bin))
    sums = hashlib.sha256(tgz.getvalue()).hexdigest() + "  devspace_linux_amd64.tar.gz\n"
    gh = _FakeGithub([], {"devspace_linux_amd64.tar.gz": tgz.getvalue(), "devspace-darwin-amd64": b"x",
                          "checksums.txt": sums.encode()})
    gh.releases = [
        _release("v9.0.0-rc1", ["devspace-linux-amd64"], gh.url, prerelease=True),  # prerelease: skipped
        _release("v8.0.0", ["devspace-linux-amd64"], gh.url, draft=True),  # draft: skipped
        _release("v3.0.0", ["devspace-darwin-amd64"], gh.url),  # no asset for this platform
        _release("v2.5.0", ["devspace_linux_amd64.tar.gz", "checksums.txt"], gh.url),
        _release("v1.0.0", ["devspace-linux-amd64"], gh.url),
        _release("nightly", ["devspace-linux-amd64"], gh.url),  # not semver
    ]
    env = {**os.environ, "HOME": home, "DEVSPACE_GITHUB_API": gh.url, "GITHUB_TOKEN": "t0k",
           "DEVSPACE_RELEASE_REPO": "acme/devspace-mi355x"}
    env.pop("DEVSPACE_RELEASE_URL", None)
    try:
        p = subprocess.run([str(exe), "upgrade"], capture_output=True, text=True, env=env, timeout=60, cwd=tmp_path)
        out = p.stdout + p.stderr
        assert p.returncode == 0, out
        assert "Successfully updated to version 2.5.0" in out and "notes for v2.5.0" in out, out
        assert open(exe, "rb").read() == new_bin
        assert os.access(exe, os.X_OK) and not os.path.exists(str(exe) + ".old")
        assert subprocess.run([str(exe), "version"], capture_output=True, text=True).returncode == 0
        api = [h for h in gh.hits if h[0].startswith("/repos/")]
        assert api and api[0][1] and api[0][2] == "token t0k"  # User-Agent + token sent to the API
        # already newest: nothing downloaded
        gh.releases = [_release("v0.0.1", ["devspace-linux-amd64"], gh.url)]
        n = len(gh.hits)
        p = subprocess.run([str(exe), "upgrade"], capture_output=True, text=True, env=env, timeout=60, cwd=tmp_path)
        assert p.returncode == 0 and "latest version" in p.stdout + p.stderr
        assert not any(h[0].startswith("/dl/") for h in gh.hits[n:])
        def offer(tag, data, checksum):
            gh.files["devspace-linux-amd64"] = data
            assets = ["devspace-linux-amd64"]
            if checksum is not None:
                gh.files["devspace-linux-amd64.sha256"] = checksum.encode()
                assets.append("devspace-linux-amd64.sha256")
            gh.releases = [_release(tag, assets, gh.url)]
            return subprocess.run([str(exe), "upgrade"], capture_output=True, text=True, env=env, timeout=60,
                                  cwd=tmp_path)

        # a non-executable asset is refused and the binary is left in place
        bad = b"<html>oops</html>"
        p = offer("v7.0.0", bad, hashlib.sha256(bad).hexdigest())
        assert p.returncode != 0 and "not an executable" in p.stdout + p.stderr, p.stdout + p.stderr
        # an upstream devspace release (an ELF without this product's id) is refused
        upstream = b"\x7fELF" + b"\0" * 4096 + b"devspace version v6.3.2"
        p = offer("v7.1.0", upstream, hashlib.sha256(upstream).hexdigest())
        assert p.returncode != 0 and "is not a devspace-mi355x build" in p.stdout + p.stderr, p.stdout + p.stderr
        # a checksum mismatch, and a release without any checksum, are refused
        good = open(BIN, "rb").read() + b"\n# release v7.2.0\n"
        p = offer("v7.2.0", good, "0" * 64)
        assert p.returncode != 0 and "checksum mismatch" in p.stdout + p.stderr, p.stdout + p.stderr
        p = offer("v7.3.0", good, None)
        assert p.returncode != 0 and "publishes no SHA-256" in p.stdout + p.stderr, p.stdout + p.stderr
        assert open(exe, "rb").read() == new_bin
        # and a verified one goes in (a lone digest in <asset>.sha256)
        p = offer("v7.4.0", good, hashlib.sha256(good).hexdigest() + "\n")
        assert p.returncode == 0 and open(exe, "rb").read() == good, p.stdout + p.stderr
    finally:
        gh.close()


def test_newer_version_notice_from_daily_cache(tmp_path):
    """root.go:38: interactive runs print a "newer version" notice. Here it comes from a daily
    cache that a detached `devspace upgrade-check` refreshes, so no command waits on GitHub."""
    import pty
    import time

    home = tmp_path / "home"
    (home / ".devspace").mkdir(parents=True)
    gh = _FakeGithub([], {})
    gh.releases = [_release("v42.0.0", ["devspace-linux-amd64"], gh.url)]
    env = {k: v for k, v in os.environ.items() if k not in ("DEVSPACE_NONINTERACTIVE", "DEVSPACE_SKIP_UPDATE_CHECK")}
    env.update(HOME=str(home), DEVSPACE_GITHUB_API=gh.url, DEVSPACE_RELEASE_REPO="acme/devspace-mi355x")

    def run_tty():
        master, slave = pty.openpty()
        p = subprocess.run([BIN, "version"], stdin=slave, stdout=slave, stderr=slave, env=env, timeout=30)
        os.close(slave)
        out = b""
        while True:
            try:
                chunk = os.read(master, 65536)
            except OSError:
                break
            if not chunk:
                break
            out += chunk
        os.close(master)
        return p.returncode, out.decode(errors="replace")

    try:
        cache = home / ".devspace" / "upgrade-check.json"
        # no cache yet: nothing printed, a background check fills the cache
        rc, out = run_tty()
        assert rc == 0 and "newer version" not in out, out
        deadline = time.time() + 20
        while time.time() < deadline and not cache.exists():
            time.sleep(0.1)
        assert json.loads(cache.read_text())["latest"] == "42.0.0"
        # next interactive run tells the user, without asking GitHub again (cache is fresh)
        n = len(gh.hits)
        rc, out = run_tty()
        assert rc == 0 and "There is a newer version of DevSpace v42.0.0" in out, out
        time.sleep(0.5)
        assert len(gh.hits) == n
        # non-interactive (CI) runs stay silent
        p = subprocess.run([BIN, "version"], capture_output=True, text=True, env=env, timeout=30)
        assert "newer version" not in p.stdout + p.stderr
    finally:
        gh.close()


def test_errors_also_land_in_errors_log(tmp_path):
    """.devspace/logs/errors.log gets the command's errors (the reference routes runtime errors
    there: util/log/file_logger.go OverrideRuntimeErrorHandler), besides default.log."""
    (tmp_path / ".devspace").mkdir()
    (tmp_path / ".devspace" / "config.yaml").write_text("version: v1alpha2\nbogusKey: 1\n")
    r = subprocess.run([BIN, "deploy"], cwd=tmp_path, capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, DEVSPACE_NONINTERACTIVE="1"))
    assert r.returncode != 0
    logs = tmp_path / ".devspace" / "logs"
    errs = [json.loads(l) for l in (logs / "errors.log").read_text().splitlines()]
    assert any("bogusKey" in e["msg"] and e["level"] == "fatal" for e in errs), errs
    assert "bogusKey" in (logs / "default.log").read_text()
