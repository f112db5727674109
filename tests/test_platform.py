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
              r"sys/eventfd\.h", r"signalfd", r"timerfd",
              # Linux or glibc only, found by an audit of src/ for what macOS's headers lack
              r"F_SETPIPE_SZ", r"TCP_QUICKACK", r"TCP_USER_TIMEOUT", r"TCP_KEEPIDLE", r"SO_PEERCRED",
              r"\bsplice\(", r"memfd_create", r"getrandom\(", r"CLOCK_BOOTTIME", r"posix_fadvise",
              r"\bfallocate\(", r"\bstatx\(", r"SOCK_NONBLOCK", r"O_PATH\b", r"renameat2", r"copy_file_range",
              r"MSG_MORE", r"<endian\.h>", r"<byteswap\.h>", r"<malloc\.h>", r"<sys/sendfile\.h>",
              r"<linux/", r"be64toh|htobe64|be32toh|htobe32", r"strchrnul", r"memrchr", r"get_nprocs",
              r"sys/sysinfo\.h", r"program_invocation_name", r"pthread_tryjoin_np", r"\bppoll\("]


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


INNER = '''
import os
import subprocess
import time


def test_hold():
    src = {src!r}
    os.makedirs(src, exist_ok=True)
    p = subprocess.Popen([{bin!r}, "sync", "--local", src, "--container", "/app", "--local-root", {root!r}],
                         cwd={cwd!r}, start_new_session=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    with open({pidfile!r} + ".tmp", "w") as f:
        f.write(str(p.pid))
    os.rename({pidfile!r} + ".tmp", {pidfile!r})
    time.sleep(600)
'''


def test_cli_children_end_with_a_killed_test_run(tmp_path):
    """a `devspace sync` a test started outlived the test run by an hour when
    pytest itself died (a timeout's os._exit skips every finally). conftest.py exports
    DEVSPACE_PARENT_PID; the CLI ties itself to that parent (PR_SET_PDEATHSIG), so SIGKILL of a
    pytest mid-test ends the CLI it started, in its own session and all."""
    import signal
    import sys

    import psutil

    pidfile = tmp_path / "cli.pid"
    inner = tmp_path / "test_inner.py"
    inner.write_text(INNER.format(src=str(tmp_path / "src"), bin=os.path.join(ROOT, "bin", "devspace"),
                                  root=str(tmp_path / "root"), cwd=str(tmp_path), pidfile=str(pidfile)))
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "tests") + os.pathsep + ROOT)
    env.pop("DEVSPACE_PARENT_PID", None)  # the inner run's conftest sets its own
    runner = subprocess.Popen([sys.executable, "-m", "pytest", "-q", "-p", "conftest", "-p", "no:cacheprovider",
                               str(inner)], cwd=str(tmp_path), env=env, stdout=subprocess.DEVNULL,
                              stderr=subprocess.DEVNULL, start_new_session=True)
    try:
        deadline = time.time() + 120
        while not pidfile.exists():
            assert runner.poll() is None and time.time() < deadline, "inner test did not start the CLI"
            time.sleep(0.05)
        cli = psutil.Process(int(pidfile.read_text()))
        assert cli.is_running() and cli.status() != psutil.STATUS_ZOMBIE
        assert cli.environ().get("DEVSPACE_PARENT_PID") == str(runner.pid)
        time.sleep(0.5)
        os.kill(runner.pid, signal.SIGKILL)
        runner.wait()
        end = time.time() + 15
        while time.time() < end:
            try:
                if cli.status() == psutil.STATUS_ZOMBIE:
                    break
            except psutil.NoSuchProcess:
                break
            time.sleep(0.05)
        else:
            cli.kill()
            raise AssertionError("the CLI outlived the killed test run")
    finally:
        if runner.poll() is None:
            os.killpg(runner.pid, signal.SIGKILL)
            runner.wait()
