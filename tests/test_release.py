"""Release artefacts (the reference's scripts/build-all.bash:24-62 ships stripped
static binaries): scripts/release.sh packages a static, stripped devspace and helper with
SHA-256 files, and a self-update from a release mirror swaps in a binary that runs with an
empty environment in a root file system that holds nothing but that binary."""

import http.server
import os
import shutil
import subprocess
import threading

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def dist(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("dist"))
    # package the in-tree static build (a fresh Release build is the script's default path)
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "release.sh")], capture_output=True, text=True,
                       env=dict(os.environ, RELEASE_BUILD_DIR="build", DIST_DIR=d), timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return d


def test_release_binaries_are_static_stripped_and_summed(dist):
    import hashlib

    for name in ("devspace-linux-amd64", "devspace-helper-linux-amd64"):
        path = os.path.join(dist, name)
        ldd = subprocess.run(["ldd", path], capture_output=True, text=True)
        assert "not a dynamic executable" in ldd.stdout + ldd.stderr, ldd.stdout + ldd.stderr
        syms = subprocess.run(["nm", path], capture_output=True, text=True)
        assert "no symbols" in syms.stderr, syms.stdout[:500]  # stripped
        digest, fname = open(path + ".sha256").read().split()
        assert fname == name and digest == hashlib.sha256(open(path, "rb").read()).hexdigest()
        assert f"{digest}  {name}" in open(os.path.join(dist, "checksums.txt")).read()
    # uploaded into every pod by the sync: small
    assert os.path.getsize(os.path.join(dist, "devspace-helper-linux-amd64")) < 1.5 * 2**20
    assert ldd_static(os.path.join(ROOT, "bin", "devspace"))
    assert open(os.path.join(dist, "latest")).read().strip() == "0.1.0-mi355x"


def ldd_static(path):
    r = subprocess.run(["ldd", path], capture_output=True, text=True)
    return "not a dynamic executable" in r.stdout + r.stderr


def _chroot_ok():
    if not shutil.which("chroot"):
        return False
    try:
        return subprocess.run(["chroot", "/", "true"], capture_output=True, timeout=10).returncode == 0
    except (OSError, subprocess.TimeoutExpired):
        return False


def test_self_update_swaps_in_a_binary_that_runs_in_an_empty_rootfs(dist, tmp_path):
    # a plain release mirror (DEVSPACE_RELEASE_URL): <url>/latest, the binary and its .sha256
    mirror = tmp_path / "mirror"
    mirror.mkdir()
    for f in ("devspace-linux-amd64", "devspace-linux-amd64.sha256"):
        shutil.copy2(os.path.join(dist, f), mirror / f)
    (mirror / "latest").write_text("99.0.0\n")

    class H(http.server.SimpleHTTPRequestHandler):
        def __init__(self, *a, **kw):
            super().__init__(*a, directory=str(mirror), **kw)

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        root = tmp_path / "rootfs"  # nothing but the binary: no libc, no /etc, no /tmp
        root.mkdir()
        exe = root / "devspace"
        shutil.copy2(os.path.join(ROOT, "bin", "devspace"), exe)
        home = tmp_path / "home"
        home.mkdir()
        env = {"HOME": str(home), "PATH": "/usr/bin:/bin",
               "DEVSPACE_RELEASE_URL": f"http://127.0.0.1:{srv.server_address[1]}"}
        p = subprocess.run([str(exe), "upgrade"], capture_output=True, text=True, env=env, timeout=60, cwd=tmp_path)
        assert p.returncode == 0 and "Successfully updated to version 99.0.0" in p.stdout + p.stderr, p.stdout + p.stderr
        assert open(exe, "rb").read() == open(os.path.join(dist, "devspace-linux-amd64"), "rb").read()
        # the swapped binary needs nothing from the system: empty environment ...
        out = subprocess.run(["env", "-i", str(exe), "version"], capture_output=True, text=True, timeout=30)
        assert out.returncode == 0 and "(devspace-mi355x)" in out.stdout, out.stdout + out.stderr
        # ... and a root file system that holds only itself
        if not _chroot_ok():
            pytest.skip("chroot not permitted here; the env -i run above passed")
        out = subprocess.run(["env", "-i", shutil.which("chroot"), str(root), "/devspace", "version"], capture_output=True,
                             text=True, timeout=30)
        assert out.returncode == 0 and "(devspace-mi355x)" in out.stdout, out.stdout + out.stderr
        # a tampered mirror binary is refused
        data = bytearray(open(mirror / "devspace-linux-amd64", "rb").read())
        data[-100] ^= 0xFF
        (mirror / "devspace-linux-amd64").write_bytes(bytes(data))
        (mirror / "latest").write_text("100.0.0\n")
        p = subprocess.run([str(exe), "upgrade"], capture_output=True, text=True, env=env, timeout=60, cwd=tmp_path)
        assert p.returncode != 0 and "does not match its published SHA-256" in p.stdout + p.stderr
    finally:
        srv.shutdown()


def test_a_target_without_a_toolchain_releases_nothing(tmp_path):
    """Cross targets (darwin-*, ...) need cmake/toolchains/<target>.cmake; without one the run
    fails before building or writing anything, rather than shipping a partial release."""
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "release.sh")], capture_output=True, text=True,
                       env=dict(os.environ, RELEASE_TARGETS="darwin-arm64", DIST_DIR=str(tmp_path / "d")),
                       timeout=120)
    assert r.returncode != 0 and "no toolchain for darwin-arm64" in r.stderr, r.stdout + r.stderr
    assert not any((tmp_path / "d").iterdir())
