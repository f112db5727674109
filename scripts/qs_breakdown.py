#!/usr/bin/env python3
"""Where the quickstart edit -> response time goes (the bench headline's loop, instrumented).

Runs bench.quickstart_loop with timestamped copies of the example's watch.js / index.js and
prints per-edit phases on one clock (ms): edit -> synced into the pod, -> watcher saw the
change, -> old server killed, -> new process handed the script (old one exited), -> new
server listening, -> response through the port-forward.

    python scripts/qs_breakdown.py [--steps 20] [--warmup 3]
"""
import argparse
import glob
import json
import os
import re
import shutil
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default="")
    ap.add_argument("--standby", type=int, default=None, help="watch.js standby count (default: its own)")
    a = ap.parse_args()
    NOW = "(require('perf_hooks').performance.timeOrigin + require('perf_hooks').performance.now())"
    trace = tempfile.mktemp(prefix="qs-trace-")
    real_copytree = shutil.copytree

    def copytree(src, dst, *args, **kw):
        r = real_copytree(src, dst, *args, **kw)
        if str(getattr(src, "path", src)).endswith(os.path.join("examples", "quickstart")):
            # sub-millisecond epoch clock shared by every node process (Date.now() is whole ms)
            t = "const T = (m) => require('fs').appendFileSync(%s, m + ' ' + %s + '\\n');\n" % (json.dumps(trace), NOW)
            w = os.path.join(dst, "watch.js")
            s = open(w).read()
            s = s.replace("const {spawn} = require('child_process');", "const {spawn} = require('child_process');\n" + t)
            s = s.replace("  restarting = true;\n  child.kill('SIGTERM');", "  restarting = true;\n  T('kill');\n  child.kill('SIGTERM');")
            s = s.replace("    const go = () => s.kill('SIGUSR2');", "    const go = () => T('handoff') || s.kill('SIGUSR2');")
            s = s.replace("  if (!name || ignored.test(name)", "  T('event');\n  if (!name || ignored.test(name)")
            # inside the standby (its program is a string in watch.js): go message in, app start
            mark = "require('fs').appendFileSync('%s', '%%s ' + %s + '\\\\n'); " % (trace, NOW)
            s = s.replace('"sent = true; if (warm)', '"' + mark % "go" + 'sent = true; if (warm)')
            s = s.replace('"require(\'module\').runMain(); });\\n"', '"' + mark % "main" + 'require(\'module\').runMain(); });\\n"')
            if a.standby is not None:
                s, n = re.subn(r"process\.env\.WATCH_STANDBY \|\| '\d+'", "'%d'" % a.standby, s)
                assert n == 1, "watch.js no longer reads WATCH_STANDBY this way"
            s = s.replace("  console.log('[watch] started gen='", "  T(s && s.ready ? 'ready' : 'booting');\n  console.log('[watch] started gen='")
            open(w, "w").write(s)
            i = os.path.join(dst, "index.js")
            s = open(i).read()
            s = s.replace("}).listen(port, () => console.log(",
                          "}).listen(port, () => require('fs').appendFileSync(%s, 'listening ' + %s + '\\n') || "
                          "console.log(" % (json.dumps(trace), NOW))
            open(i, "w").write(s)
        return r

    shutil.copytree = copytree
    marks = []
    orig_edit, orig_wait, orig_get = bench._qs_edit, bench._wait_file_contains, bench._http_get

    def edit(path, marker):
        marks.append({"edit": time.time() * 1000})
        return orig_edit(path, marker)

    def wait(*args, **kw):
        r = orig_wait(*args, **kw)
        marks[-1]["synced"] = time.time() * 1000
        return r

    def get(port, timeout=2.0):
        body = orig_get(port, timeout)
        if marks and body and "got" not in marks[-1] and "[q" in body:
            m = body.split("[", 1)[1].split("]", 1)[0]
            if m == f"q{len(marks) - 1}" + ("_" * ((len(marks) - 1) % 2)):
                marks[-1]["got"] = time.time() * 1000
        return body

    bench._qs_edit, bench._wait_file_contains, bench._http_get = edit, wait, get
    with tempfile.TemporaryDirectory() as d:
        r = bench.quickstart_loop(d, a.steps, a.warmup)
        spans = []
        for tp in glob.glob(os.path.join(d, "*", "quickstart", ".devspace", "logs", "trace.jsonl")):
            spans += [json.loads(l) for l in open(tp) if '"portforward.stream"' in l]
    events = []
    for line in open(trace):
        k, v = line.split()
        events.append((float(v), k))
    rows = []
    for m in marks[a.warmup:]:
        after = [(t, k) for t, k in events if t >= m["edit"] - 1]
        first = {}
        for t, k in after:
            first.setdefault(k, t)
        row = {"sync": m.get("synced", 0) - m["edit"]}
        for k in ("event", "kill", "handoff", "go", "main", "listening"):
            if k in first:
                row[k] = first[k] - m["edit"]
        # the restart's hand-off went to a booted standby, or to one still booting
        pick = next((k for _, k in after if k in ("ready", "booting")), None)
        if pick:
            row["standby"] = pick
        if "got" in m:
            row["response"] = m["got"] - m["edit"]
        rows.append(row)
    keys = ["sync", "event", "kill", "handoff", "go", "main", "listening", "response"]
    print("ms after the edit (p50 over %d edits): " % len(rows) +
          ", ".join("%s %.2f" % (k, statistics.median([x[k] for x in rows if k in x])) for k in keys
                    if any(k in x for x in rows)))
    print("bench p50 %.2f ms p90 %.2f ms; handoffs to a booted standby: %d of %d" % (
        statistics.median(r["reload_ms"]), bench._pct(r["reload_ms"], 0.9), sum(1 for x in rows if x.get("standby") == "ready"),
        len(rows)))
    # port-forward streams (trace.jsonl spans): how long a held connection's attempts take
    for outcome in ("refused", "reply"):
        v = [x for x in spans if x["outcome"] == outcome]
        if v:
            print("portforward %s streams: %d, open p50 %.2f ms, first byte/refusal p50 %.2f ms, preopened %d" % (
                outcome, len(v), statistics.median(int(x["open_us"]) for x in v) / 1000,
                statistics.median(int(x["first_us"]) for x in v) / 1000,
                sum(1 for x in v if x.get("preopened") == "1")))
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"rows": rows, "reload_ms": r["reload_ms"]}, f, indent=1)
    os.unlink(trace)


if __name__ == "__main__":
    main()
