"""Bounded-memory sync of multi-GB files (VERDICT r2 "Next round" #1).

The reference streams archives through temp files (`/root/reference/pkg/devspace/sync/tar.go:146-182`,
`sync/downstream.go:443-468`). Here a >= 2 GiB incompressible file (a checkpoint) goes up and
another comes back down, in all three sync protocols, through the real `devspace sync` binary
against a local "pod" directory (`--local-root`: local shells stand in for `kubectl exec`, the
reference's own test seam `sync/upstream.go:67-95`). The peak RSS (VmHWM) of `devspace` and of
the in-container helper must stay under 64 MiB: nothing holds a whole archive in memory.

A second test cuts the stream in the middle of a transfer (FaultInjectingTransport via the
`--fault-*` hooks) and checks that the session reconnects, re-sends what was in flight and ends
byte-exact, with no temp file left on either side.

Timings and peaks go to $SYNC_LARGE_OUT when set (profiles/r3_sync_large.json)."""

import hashlib
import json
import os
import re
import shutil
import signal
import subprocess
import threading
import time

import psutil
import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "bin", "devspace")
SIZE = int(os.environ.get("DS_LARGE_FILE_BYTES", str((2 << 30) + 12345)))  # > 2 GiB, not block-aligned
RSS_CAP = 64 << 20
RESULTS = {}


def _record(key, value):
    RESULTS[key] = value
    out = os.environ.get("SYNC_LARGE_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(RESULTS, f, indent=1, sort_keys=True)


def _write_random(path, size):
    h = hashlib.sha256()
    with open(path, "wb") as f:
        left = size
        while left:
            chunk = os.urandom(min(left, 16 << 20))
            f.write(chunk)
            h.update(chunk)
            left -= len(chunk)
    return h.hexdigest()


def _sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(16 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


@pytest.fixture(scope="module")
def payloads(tmp_path_factory):
    d = tmp_path_factory.mktemp("large-payloads")
    up, down = str(d / "up.bin"), str(d / "down.bin")
    out = {"up": (up, _write_random(up, SIZE)), "down": (down, _write_random(down, SIZE + 4096))}
    yield out
    shutil.rmtree(str(d), ignore_errors=True)


class PeakRss:
    """Samples VmHWM (peak RSS) of a process tree — devspace plus the "pod" side processes
    (helper, sh, tar...) — every 100 ms until stopped."""

    def __init__(self, pid):
        self.root = psutil.Process(pid)
        self.peak = {}
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        while not self._stop.is_set():
            self.sample()
            self._stop.wait(0.1)

    def sample(self):
        try:
            procs = [self.root] + self.root.children(recursive=True)
        except psutil.Error:
            return
        for p in procs:
            try:
                name = "devspace" if p.pid == self.root.pid else p.name()
                with open(f"/proc/{p.pid}/status") as f:
                    for line in f:
                        if line.startswith("VmHWM:"):
                            kb = int(line.split()[1])
                            self.peak[name] = max(self.peak.get(name, 0), kb * 1024)
            except (psutil.Error, OSError, ValueError):
                pass

    def stop(self):
        self.sample()
        self._stop.set()
        self._t.join()
        return self.peak


def _start_sync(tmp_path, src, pod, mode, *extra, warn_mb=None):
    env = dict(os.environ, HOME=str(tmp_path / "home"), DEVSPACE_NONINTERACTIVE="1", DEVSPACE_SKIP_UPDATE_CHECK="1")
    if warn_mb is not None:
        env["DEVSPACE_SYNC_WARN_FILE_MB"] = str(warn_mb)
    log = open(str(tmp_path / f"sync-{mode}.out"), "w")
    p = subprocess.Popen([BIN, "sync", "--local-root", str(pod), "--local", str(src), "--container", "/app",
                          "--mode", mode, *extra], cwd=str(tmp_path), env=env, stdout=log, stderr=subprocess.STDOUT,
                         stdin=subprocess.DEVNULL, start_new_session=True)
    return p, log


def _stop_sync(p, log):
    if p.poll() is None:
        os.killpg(p.pid, signal.SIGINT)
        try:
            p.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
    log.close()


def _wait_file(path, size, timeout, proc, what):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        try:
            if os.path.getsize(path) == size:
                return
        except OSError:
            pass
        if proc.poll() is not None:
            raise AssertionError(f"devspace sync exited (rc={proc.returncode}) before {what}")
        time.sleep(0.05)
    raise AssertionError(f"timed out: {what}")


def _sync_log(tmp_path):
    try:
        return open(str(tmp_path / ".devspace" / "logs" / "sync.log")).read()
    except OSError:
        return ""


def _temp_leftovers(*roots):
    left = []
    for root in roots:
        for d, _, files in os.walk(root):
            left += [os.path.join(d, f) for f in files if f.endswith(".devspace-tmp")]
    return left


@pytest.mark.parametrize("mode", ["helper", "fast", "compat"])
def test_multi_gb_file_each_way_bounded_rss(mode, payloads, tmp_path):
    src, pod = tmp_path / "src", tmp_path / "pod"
    src.mkdir()
    (pod / "app").mkdir(parents=True)
    up_path, up_sha = payloads["up"]
    down_path, down_sha = payloads["down"]
    os.link(up_path, str(src / "ckpt-up.bin"))  # a 2 GiB checkpoint in the project (no copy)
    (src / "train.py").write_text("print('hello')\n")
    # the large-file warning threshold (default 1 GiB) at half the payload, whatever its size
    p, log = _start_sync(tmp_path, src, pod, mode, warn_mb=max(1, SIZE // 2 >> 20))
    mon = PeakRss(p.pid)
    try:
        t0 = time.perf_counter()
        _wait_file(str(pod / "app" / "ckpt-up.bin"), SIZE, 900, p, "upload of the 2 GiB file")
        up_s = time.perf_counter() - t0
        assert _sha(str(pod / "app" / "ckpt-up.bin")) == up_sha
        assert (pod / "app" / "train.py").read_text() == "print('hello')\n"
        # a checkpoint written in the pod comes back (appears atomically, as torch.save + rename)
        t1 = time.perf_counter()
        os.link(down_path, str(pod / "app" / "ckpt-down.bin"))
        _wait_file(str(src / "ckpt-down.bin"), SIZE + 4096, 900, p, "download of the 2 GiB file")
        down_s = time.perf_counter() - t1
        assert _sha(str(src / "ckpt-down.bin")) == down_sha
        peaks = mon.stop()
        assert p.poll() is None, "devspace sync exited"
        sync_log = _sync_log(tmp_path)
        assert "Large file /ckpt-up.bin" in sync_log and "Large file /ckpt-down.bin" in sync_log, sync_log[-2000:]
        assert not _temp_leftovers(str(src), str(pod))
        helper_peak = max([v for k, v in peaks.items() if k.startswith("devspace-helpe")], default=0)
        _record(mode, {"bytes_each_way": SIZE, "upload_s": round(up_s, 2), "download_s": round(down_s, 2),
                       "upload_MBps": round(SIZE / up_s / 1e6, 1), "download_MBps": round(SIZE / down_s / 1e6, 1),
                       "peak_rss_MiB": {k: round(v / 2**20, 1) for k, v in sorted(peaks.items())}})
        assert peaks["devspace"] < RSS_CAP, peaks
        if mode == "helper":
            assert helper_peak > 0, peaks  # the helper really ran
            assert helper_peak < RSS_CAP, peaks
    finally:
        if mon._t.is_alive():
            mon.stop()
        _stop_sync(p, log)
        shutil.rmtree(str(src), ignore_errors=True)
        shutil.rmtree(str(pod), ignore_errors=True)


@pytest.mark.parametrize("mode,direction", [("helper", "up"), ("helper", "down"), ("fast", "up"), ("fast", "down")])
def test_stream_killed_mid_transfer_resumes(mode, direction, tmp_path):
    size = 384 << 20
    src, pod = tmp_path / "src", tmp_path / "pod"
    src.mkdir()
    (pod / "app").mkdir(parents=True)
    (src / "keep.txt").write_text("small file\n")
    if direction == "up":
        sha = _write_random(str(src / "big.bin"), size)
        # the first shell carries the uploads in both protocols
        fault = ["--fault-stdin-bytes", str(128 << 20), "--fault-shell", "1"]
    else:
        # fast: the downstream shell (2nd) carries it; helper: a big file comes down on the
        # bulk download channel, opened for it (3rd)
        fault = ["--fault-stdout-bytes", str(128 << 20), "--fault-shell", "3" if mode == "helper" else "2"]
    p, log = _start_sync(tmp_path, src, pod, mode, *fault)
    try:
        if direction == "up":
            target = pod / "app" / "big.bin"
        else:
            _wait_file(str(pod / "app" / "keep.txt"), len("small file\n"), 120, p, "initial sync")
            tmp = pod / "app" / "big.bin.partial"
            sha = _write_random(str(tmp), size)
            os.rename(str(tmp), str(pod / "app" / "big.bin"))
            target = src / "big.bin"
        _wait_file(str(target), size, 300, p, "transfer after the cut stream")
        # the resumed copy is complete and exact (not the half sent before the cut)
        deadline = time.monotonic() + 60
        while _sha(str(target)) != sha:
            assert time.monotonic() < deadline, "content never converged"
            time.sleep(0.5)
        sync_log = _sync_log(tmp_path)
        assert "reconnecting" in sync_log, sync_log[-3000:]
        assert "Reconnected" in sync_log, sync_log[-3000:]
        time.sleep(0.5)
        assert not _temp_leftovers(str(src), str(pod))
        assert p.poll() is None
        # and the session keeps working after the reconnect
        (src / "after.txt").write_text("after the fault\n")
        _wait_file(str(pod / "app" / "after.txt"), len("after the fault\n"), 60, p, "edit after the reconnect")
    finally:
        _stop_sync(p, log)


def test_helper_frame_lengths_are_64_bit():
    """The helper request header carries a u64 length (a >4 GiB value survives); the archive
    chunk stream has no total length at all (tests/cpp/test_sync.cc streams 4.5 GiB through it)."""
    from devspace_amd import _native

    for n in (0, 1, (1 << 32) - 1, 1 << 32, (5 << 30) + 7, (1 << 63) + 3):
        h = _native.frame_header("U", n)
        assert len(h) == 9 and h[0:1] == b"U"
        assert int.from_bytes(h[1:], "big") == n
        assert _native.frame_parse(h) == ("U", n)


def test_multi_gb_build_context_streams_to_the_daemon(payloads, tmp_path):
    """`devspace deploy` of a project whose Docker build context holds a > 2 GiB file (VERDICT r2
    #5): the context tar streams to the Docker Engine API as a chunked POST /build body while the
    tree is walked (the reference streams a tar reader, builder/docker/docker.go:94-158), so the
    CLI's peak RSS stays under 64 MiB; the daemon receives every byte."""
    from conftest import DevspaceEnv
    from devspace_amd.localkube import LocalCluster

    cluster = LocalCluster(str(tmp_path / "state"), gpus=0).start()
    try:
        lk = DevspaceEnv(cluster, str(tmp_path))
        proj = lk.project("quickstart", "qs-bigctx")
        up_path, up_sha = payloads["up"]
        os.link(up_path, os.path.join(proj, "weights.bin"))
        # the chart's pod would copy the image rootfs (2 GiB more disk): the build is the point
        cfg = os.path.join(proj, ".devspace", "config.yaml")
        text = open(cfg).read().replace("chartPath: ./chart", "chartPath: ./chart\n    wait: false")
        with open(cfg, "w") as f:
            f.write(text)
        p = subprocess.Popen([lk.bin, "deploy"], cwd=proj, env=lk.env, stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, text=True)
        mon = PeakRss(p.pid)
        out, _ = p.communicate(timeout=900)
        peaks = mon.stop()
        assert p.returncode == 0, out[-3000:]
        assert "Sending build context to Docker daemon" in out and "Sent build context" in out, out[-3000:]
        sent_kb = float(re.search(r"Sent build context: ([\d.]+)kB", out).group(1))
        assert sent_kb * 1000 > SIZE, out[-2000:]
        # the image the daemon built holds the whole file, byte for byte
        img_root = None
        for d, _, files in os.walk(str(tmp_path / "state")):
            if "weights.bin" in files and os.path.getsize(os.path.join(d, "weights.bin")) == SIZE:
                img_root = d
                break
        assert img_root, "weights.bin not in any image rootfs"
        assert _sha(os.path.join(img_root, "weights.bin")) == up_sha
        _record("docker_build_context", {"bytes": SIZE, "devspace_peak_rss_MiB": round(peaks["devspace"] / 2**20, 1)})
        assert peaks["devspace"] < RSS_CAP, peaks
    finally:
        cluster.stop()


def test_small_edit_overtakes_a_multi_gb_upload(payloads, tmp_path):
    """a 1 KiB edit made while a >= 2 GiB file is uploading lands in the pod within
    200 ms (the helper's interactive lane, interleaved frame by frame with the bulk one), and a
    pod-side change comes back meanwhile (no index lock across the upload) — through the real
    `devspace sync` binary."""
    src, pod = tmp_path / "src", tmp_path / "pod"
    src.mkdir()
    (pod / "app").mkdir(parents=True)
    (src / "train.py").write_text("MARKER = 0\n")
    up_path, up_sha = payloads["up"]
    p, log = _start_sync(tmp_path, src, pod, "helper")
    try:
        deadline = time.monotonic() + 60
        while not (pod / "app" / "train.py").exists():
            assert time.monotonic() < deadline and p.poll() is None, "initial sync"
            time.sleep(0.02)
        os.link(up_path, str(src / "ckpt-up.bin"))
        tmp = pod / "app" / "ckpt-up.bin.devspace-tmp"
        deadline = time.monotonic() + 60
        while not (tmp.exists() and tmp.stat().st_size > (16 << 20)):
            assert time.monotonic() < deadline and p.poll() is None, "bulk upload never started"
            time.sleep(0.005)
        t0 = time.perf_counter()
        (src / "train.py").write_text("MARKER = 1\n" + "#" * 1024 + "\n")
        deadline = time.monotonic() + 10
        while not (pod / "app" / "train.py").read_bytes().startswith(b"MARKER = 1"):
            assert time.monotonic() < deadline, "edit never landed"
            time.sleep(0.001)
        edit_ms = (time.perf_counter() - t0) * 1000
        bulk_in_flight = tmp.exists() and tmp.stat().st_size < SIZE
        (pod / "app" / "metrics.json").write_text('{"step": 7}\n')
        t_down = time.perf_counter()
        deadline = time.monotonic() + 20
        while not ((src / "metrics.json").exists() and (src / "metrics.json").read_text() == '{"step": 7}\n'):
            assert time.monotonic() < deadline, "pod-side change never came back"
            time.sleep(0.005)
        down_in_flight = tmp.exists()
        down_ms = (time.perf_counter() - t_down) * 1000
        _wait_file(str(pod / "app" / "ckpt-up.bin"), SIZE, 900, p, "the bulk upload")
        upload_s = time.perf_counter() - t0
        assert _sha(str(pod / "app" / "ckpt-up.bin")) == up_sha
        _record("helper_lanes", {"bytes": SIZE, "edit_during_upload_ms": round(edit_ms, 2),
                                 "bulk_in_flight_at_edit": bulk_in_flight,
                                 "bulk_in_flight_at_download": down_in_flight})
        assert bulk_in_flight, "the upload finished before the edit landed: nothing was measured"
        assert edit_ms < 200, edit_ms
        assert down_in_flight, (f"the upload finished before the pod-side change came back (pod-side change "
                                f"back after {down_ms:.0f} ms, upload done {upload_s:.2f} s after the edit)")
        assert (pod / "app" / "train.py").read_bytes().startswith(b"MARKER = 1")
    finally:
        _stop_sync(p, log)
        shutil.rmtree(str(src), ignore_errors=True)
        shutil.rmtree(str(pod), ignore_errors=True)
