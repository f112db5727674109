#!/usr/bin/env python3
"""Node start-up costs on this machine (input for examples/quickstart/watch.js's standby pool):
plain `node -e 0`, a standby boot with watch.js's preload list up to its 'ready' message, and
the time a booted standby takes to load + listen the quickstart server."""
import os
import re
import shutil
import socket
import statistics
import subprocess
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")


def main():
    print("node", subprocess.run([NODE, "--version"], capture_output=True, text=True).stdout.strip())
    t = []
    for _ in range(15):
        t0 = time.perf_counter()
        subprocess.run([NODE, "-e", "0"])
        t.append((time.perf_counter() - t0) * 1000)
    print("node -e 0: p50 %.1f ms" % statistics.median(t))
    src = open(os.path.join(ROOT, "examples", "quickstart", "watch.js")).read()
    preload = re.search(r"const PRELOAD = (\[[^\]]*\]);", src, re.S).group(1)
    # the boot's warm-up statement (a JS string expression in watch.js), evaluated by node
    warm_expr = re.search(r"const WARM = (.*?);\n", src, re.S).group(1)
    warm = subprocess.run([NODE, "-e", "process.stdout.write(%s)" % warm_expr], capture_output=True,
                          text=True).stdout.replace("ready", "go")
    for label, mods in (("full preload", preload), ("no preload", "[]")):
        boot = ("const T0 = Date.now(); for (const m of %s) { try { require(m); } catch (e) {} }\n"
                "process.stdout.write('ready ' + (Date.now() - T0) + '\\n');" % mods)
        t = []
        for _ in range(15):
            t0 = time.perf_counter()
            p = subprocess.run([NODE, "-e", boot], capture_output=True, text=True)
            t.append((time.perf_counter() - t0) * 1000)
        print("%s: process p50 %.1f ms (preload itself %s ms)" % (label, statistics.median(t), p.stdout.split()[-1]))
    # booted standby -> listening
    d = tempfile.mkdtemp()
    shutil.copy(os.path.join(ROOT, "examples", "quickstart", "index.js"), d)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    for label, mods, warmup in (("full preload + warm-up", preload, warm), ("full preload", preload, ""),
                                ("no preload", "[]", "")):
        t = []
        for _ in range(10):
            code = ("for (const m of %s) { try { require(m); } catch (e) {} }\n"
                    "function go() {}\n" % mods) + warmup + (
                    "process.stdin.once('data', () => { const t0 = Date.now(); process.argv[1] = %r; "
                    "const http = require('http'); const L = http.Server.prototype.listen; "
                    "http.Server.prototype.listen = function (...a) { const cb = a[a.length - 1]; "
                    "a[a.length - 1] = () => { process.stderr.write('L ' + (Date.now() - t0) + '\\n'); process.exit(0); }; "
                    "return L.apply(this, a); }; require('module').runMain(); });" % os.path.join(d, "index.js"))
            p = subprocess.Popen([NODE, "-e", code], stdin=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                 env=dict(os.environ, PORT=str(port)))
            time.sleep(0.3)
            p.stdin.write("go\n")
            p.stdin.flush()
            err = p.stderr.read()
            p.wait()
            m = re.search(r"L (\d+)", err)
            if m:
                t.append(float(m.group(1)))
        print("%s: handoff -> listening p50 %.1f ms" % (label, statistics.median(t) if t else -1))


if __name__ == "__main__":
    main()
