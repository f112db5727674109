"""The client's OS seam (src/platform/) and the portable build.

The reference ships darwin, windows and linux clients (/root/reference/scripts/build-all.bash:27-62,
/root/reference/.travis.yml:21-47). Here every Linux-only interface of the CLI sits in
src/platform/linux*.cc; -DDEVSPACE_PORTABLE=ON builds the client from POSIX calls only
(src/platform/posix*.cc and the stat-scan watcher). scripts/ci.sh builds that variant and runs the
C++ suite, the sync matrix and the e2e suite with it; here the rule itself is checked, and the
scanner runs the end-to-end sync in this build (DEVSPACE_WATCHER=scan).
"""

import os
import re
import subprocess
import time

from conftest import ROOT

LINUX_ONLY = [r"inotify_", r"epoll_", r"prctl\(", r"pipe2\(", r"accept4\(", r"eventfd\(", r"MSG_NOSIGNAL",
              r"SOCK_CLOEXEC", r"O_TMPFILE", r"/proc/self", r"sys/inotify\.h", r"sys/epoll\.h", r"sys/prctl\.h",
              r"sys/eventfd\.h", r"signalfd", r"timerfd"]


def test_linux_only_calls_stay_behind_the_platform_layer():
    bad = []
    src = os.path.join(ROOT, "src")
    for d, _, files in os.walk(src):
        rel_d = os.path.relpath(d, src)
        if rel_d.startswith("helper"):
            continue  # the in-container agent: Linux by design, it runs in the pod
        for f in files:
            if not f.endswith((".cc", ".h")):
                continue
            if rel_d == "platform" and f.startswith("linux"):
                continue
            for n, line in enumerate(open(os.path.join(d, f), encoding="utf-8"), 1):
                if line.lstrip().startswith("//"):
                    continue
                for p in LINUX_ONLY:
                    if re.search(p, line):
                        bad.append(f"src/{rel_d}/{f}:{n}: {line.strip()}")
    assert not bad, "Linux-only calls outside src/platform/linux*:\n" + "\n".join(bad)


def test_cmake_selects_one_platform_layer():
    cm = open(os.path.join(ROOT, "CMakeLists.txt")).read()
    assert 'option(DEVSPACE_PORTABLE' in cm
    assert re.search(r"EXCLUDE REGEX .*platform/linux", cm) and re.search(r"EXCLUDE REGEX .*platform/posix", cm)
    assert "enable_testing()" in cm and "add_test(NAME devspace_tests" in cm


def test_scan_watcher_drives_the_cli_sync(tmp_path):
    """`devspace sync` on a local directory pair with the portable watcher: an edit, a new
    directory and a removal arrive, as with inotify."""
    src = tmp_path / "src"
    src.mkdir()
    (src / "a.txt").write_text("one")
    env = dict(os.environ, DEVSPACE_WATCHER="scan", HOME=str(tmp_path))
    exe = os.environ.get("DEVSPACE_BIN") or os.path.join(ROOT, "bin", "devspace")
    root = tmp_path / "root"
    dst = root / "app"
    p = subprocess.Popen([exe, "sync", "--local", str(src), "--container", "/app", "--local-root", str(root)], env=env,
                         cwd=str(tmp_path),
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, start_new_session=True)

    def wait(cond, what, t=15):
        end = time.time() + t
        while time.time() < end:
            if cond():
                return
            time.sleep(0.02)
        raise AssertionError(f"timed out waiting for {what}")

    try:
        wait(lambda: (dst / "a.txt").exists(), "initial sync")
        (src / "a.txt").write_text("two")
        wait(lambda: (dst / "a.txt").read_text() == "two", "edit")
        (src / "d" / "e").mkdir(parents=True)
        (src / "d" / "e" / "f.txt").write_text("deep")
        wait(lambda: (dst / "d" / "e" / "f.txt").exists(), "new directory")
        (src / "a.txt").unlink()
        wait(lambda: not (dst / "a.txt").exists(), "removal")
    finally:
        os.killpg(p.pid, 9)
        p.wait()
