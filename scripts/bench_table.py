#!/usr/bin/env python3
"""Renders the README benchmark table from a driver-written ``BENCH_rNN.json`` (never from the
builder's own runs under ``profiles/``), so the README quotes exactly what the driver measured.

    python scripts/bench_table.py BENCH_r02.json            # print the table
    python scripts/bench_table.py BENCH_r03.json --update   # rewrite README.md's bench block

The README block sits between ``<!-- bench-table source=FILE -->`` and ``<!-- /bench-table -->``;
``tests/test_readme_bench.py`` checks that it equals what this script renders from FILE.
Handles the bench.py line formats: round 2 (``value`` = rocm-pytorch pod reload, quickstart
under ``quickstart``), round 3 (``value`` = quickstart reload with the example's standby pool,
cold restarts under ``cold_restart``) and round 4+ (``value`` = quickstart with cold restarts,
``config.restart == "cold"``, the pool under ``standby_pool``); extras under ``gpu_pod``,
``deploy``, ``php_mysql``, ``microservices``, ``kaniko``.
"""

import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BEGIN = re.compile(r"<!-- bench-table source=(\S+) -->\n")
END = "<!-- /bench-table -->"


def load_line(path):
    """The bench.py JSON line out of a driver BENCH file (or a bare bench.py output file)."""
    with open(path) as f:
        doc = json.load(f)
    if "metric" in doc:
        return doc, {}
    tail = doc.get("run", {}).get("stdout_tail", "")
    for line in tail.splitlines():
        line = line.strip()
        if line.startswith('{"metric"'):
            return json.loads(line), doc
    raise ValueError(f"{path}: no bench.py JSON line in run.stdout_tail")


def _ms(v):
    return "—" if v is None else (f"{v:.2f} ms" if v < 100 else f"{v:.0f} ms")


def _s(v):
    return "—" if v is None else f"{v:.3f} s"


def _x(a, b):
    return f" (**{b / a:.1f}x**)" if a and b else ""


def render(path):
    b, doc = load_line(path)
    name = os.path.basename(path)
    rows = []
    round3 = "gpu_pod" in b or "php_mysql" in b or b.get("config", {}).get("app") == "examples/quickstart"
    if round3:
        ref = b.get("reference_equivalent", {})
        cold_headline = b.get("config", {}).get("restart") == "cold"
        rows.append(("edit → new response p50, quickstart, cold restarts as nodemon (headline `value`: the tool's loop)"
                     if cold_headline else "edit → new response p50, quickstart (headline `value`)",
                     f"**{_ms(b['value'])}** (p90 {_ms(b.get('p90_ms'))}; sync {_ms(b.get('sync_p50_ms'))})",
                     _ms(ref.get("p50_ms")) + _x(b["value"], ref.get("p50_ms"))))
        pool = b.get("standby_pool")
        if isinstance(pool, dict) and "p50_ms" in pool:
            rows.append(("edit → new response p50, quickstart with the example app's pre-booted node standbys "
                         "(app-side, not the tool)",
                         f"{_ms(pool['p50_ms'])} (p90 {_ms(pool.get('p90_ms'))})", "—"))
        cold = b.get("cold_restart")
        if isinstance(cold, dict) and "p50_ms" in cold:
            rows.append(("edit → new response p50, quickstart with cold restarts (the tool alone, no standby pool)",
                         f"**{_ms(cold['p50_ms'])}** (p90 {_ms(cold.get('p90_ms'))})",
                         _ms(ref.get("p50_ms")) + _x(cold["p50_ms"], ref.get("p50_ms"))))
        rows.append(("sync p50, quickstart (edit → bytes in the pod)", f"**{_ms(b.get('sync_p50_ms'))}**",
                     _ms(ref.get("sync_p50_ms")) + _x(b.get("sync_p50_ms"), ref.get("sync_p50_ms"))))
        if b.get("dev_start_s") is not None:
            rows.append(("`devspace dev` start → app answering through the forward, quickstart",
                         f"{_s(b['dev_start_s'])}",
                         _s(ref.get("dev_start_s")) + _x(b["dev_start_s"], ref.get("dev_start_s"))
                         if ref.get("dev_start_s") else "—"))
        g = b.get("gpu_pod")
        if isinstance(g, dict) and "reload_p50_ms" in g:
            gr = g.get("reference_equivalent", {})
            rows.append((f"edit → pod hot-reload p50, rocm-pytorch ({g.get('parallelism')}, fused={g.get('fused_ops')})",
                         f"**{_ms(g['reload_p50_ms'])}** (sync {_ms(g.get('sync_p50_ms'))})",
                         _ms(gr.get("p50_ms")) + " (compat sync + cold workload restart)" if gr else "—"))
        drill = g.get("fault_drill") if isinstance(g, dict) else None
        if isinstance(drill, dict) and drill.get("recovered"):
            rows.append((f"rocm-pytorch fault drill ({drill.get('failure', 'one rank fails')}): failure → training again",
                         f"{_s(drill.get('failure_to_training_s'))} (warm standby: "
                         f"{'yes' if drill.get('warm_standby') else 'no'}; resumed at step "
                         f"{drill.get('resumed_from_step')})", "— (the process restarts from step 0)"))
        w = b.get("wan")
        if isinstance(w, dict) and "p50_ms" in w:
            wr = w.get("reference_equivalent", {})
            rows.append((f"edit → new response p50, quickstart, cluster behind {w.get('rtt_ms')} ms RTT / "
                         f"{w.get('mbit')} Mbit/s (sync p50)",
                         f"**{_ms(w['p50_ms'])}** (sync {_ms(w.get('sync_p50_ms'))})",
                         (f"{_ms(wr.get('p50_ms'))} (sync {_ms(wr.get('sync_p50_ms'))})" + _x(w["p50_ms"], wr.get("p50_ms")))
                         if wr else "—"))
            gw = g.get("wan") if isinstance(g, dict) else None
            if isinstance(gw, dict) and "reload_p50_ms" in gw:
                rows.append((f"edit → pod hot-reload p50, rocm-pytorch, across that link (sync p50)",
                             f"**{_ms(gw['reload_p50_ms'])}** (sync {_ms(gw.get('sync_p50_ms'))})", "—"))
            wd = w.get("deploy")
            if isinstance(wd, dict) and "wall_clock_s" in wd:
                wdr = wd.get("reference_equivalent", {})
                rows.append((f"`devspace deploy` quickstart across that link, cold",
                             f"{_s(wd['wall_clock_s'])}",
                             _s(wdr.get("wall_clock_s")) + _x(wd["wall_clock_s"], wdr.get("wall_clock_s")) if wdr else "—"))
        for key, label in (("php_mysql", "php-mysql"), ("microservices", "microservices"), ("kaniko", "kaniko")):
            e = b.get(key)
            if isinstance(e, dict) and "edit_to_pod_p50_ms" in e:
                er = e.get("reference_equivalent", {})
                # round 4's microservices deploy ran with helm's rollout wait off in both columns
                if key == "microservices" and "rollout wait (on" not in e.get("note", ""):
                    label += " (helm wait off in both columns)"
                rows.append((f"{label}: edit → pod p50 / deploy cold",
                             f"{_ms(e['edit_to_pod_p50_ms'])} / {_s(e.get('deploy_cold_s'))}",
                             f"{_ms(er.get('edit_to_pod_p50_ms'))} / {_s(er.get('deploy_cold_s'))}" if er else "—"))
            elif isinstance(e, dict) and "error" in e:
                rows.append((f"{label}", f"failed: {e['error'][:60]}", "—"))
    else:
        qs = b.get("quickstart", {})
        rows.append(("edit → pod hot-reload p50, rocm-pytorch (headline `value`)",
                     f"**{_ms(b['value'])}** (p90 {_ms(b.get('p90_ms'))}; sync {_ms(b.get('sync_p50_ms'))})",
                     _ms(b.get("reference_equivalent", {}).get("p50_ms")) + " (compat sync + cold workload restart)"))
        rows.append(("edit → new response p50, quickstart", f"**{_ms(qs.get('reload_p50_ms'))}**",
                     _ms(qs.get("compat_reload_p50_ms")) + _x(qs.get("reload_p50_ms"), qs.get("compat_reload_p50_ms"))))
        rows.append(("sync p50, quickstart (edit → bytes in the pod)", f"**{_ms(qs.get('sync_p50_ms'))}**",
                     _ms(qs.get("compat_sync_p50_ms")) + _x(qs.get("sync_p50_ms"), qs.get("compat_sync_p50_ms"))))
    d = b.get("deploy")
    if isinstance(d, dict) and "wall_clock_s" in d:
        dr = d.get("reference_equivalent", {})
        net = d.get("net") or {}
        # round 4 and before: the image build skipped RUN steps (control_plane_only); from round 5
        # the build runs them (npm install) and an edit is redeployed from the layer cache
        what = ("control plane only: RUN steps not executed" if d.get("control_plane_only", True)
                else "image build runs the Dockerfile's RUN steps; base image not pulled")
        if d.get("edit_redeploy_s") is not None:
            rows.append((f"`devspace deploy` quickstart, cold / after an edit / unchanged ({what})",
                         f"{_s(d['wall_clock_s'])} / {_s(d['edit_redeploy_s'])} / {_s(d.get('warm_wall_clock_s'))} "
                         f"({net.get('tls_handshakes', '?')} TLS handshakes, {net.get('requests', '?')} requests)",
                         f"{_s(dr.get('wall_clock_s'))} / {_s(dr.get('edit_redeploy_s'))} / "
                         f"{_s(dr.get('warm_wall_clock_s'))}" + _x(d["wall_clock_s"], dr.get("wall_clock_s"))
                         if dr else "—"))
        else:
            rows.append((f"`devspace deploy` quickstart, cold / warm ({what})",
                         f"{_s(d['wall_clock_s'])} / {_s(d.get('warm_wall_clock_s'))} "
                         f"({net.get('tls_handshakes', '?')} TLS handshakes, {net.get('requests', '?')} requests)",
                         f"{_s(dr.get('wall_clock_s'))} / {_s(dr.get('warm_wall_clock_s'))}" if dr else "—"))
    where = doc.get("where", "bench.py output")
    cmd = doc.get("cmd", "")
    head = doc.get("head", "")
    out = [f"Driver run `{name}`: `{cmd}` on {where}" + (f", commit `{head}`" if head else "") +
           f"; {b.get('steps')} timed steps after {b.get('warmup')} warmup, `ms_per_step` {b.get('ms_per_step')}.",
           "",
           "| | this rebuild | reference-equivalent, same box |",
           "|---|---|---|"]
    out += [f"| {a} | {c} | {r} |" for a, c, r in rows]
    return "\n".join(out) + "\n"


def update_readme(path, readme=os.path.join(ROOT, "README.md")):
    text = open(readme).read()
    m = BEGIN.search(text)
    if not m:
        raise SystemExit("README.md has no <!-- bench-table source=... --> block")
    end = text.index(END, m.end())
    name = os.path.basename(path)
    new = text[:m.start()] + f"<!-- bench-table source={name} -->\n" + render(path) + text[end:]
    with open(readme, "w") as f:
        f.write(new)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("bench_file")
    ap.add_argument("--update", action="store_true", help="rewrite README.md's bench-table block")
    a = ap.parse_args(argv)
    if a.update:
        update_readme(a.bench_file)
    else:
        sys.stdout.write(render(a.bench_file))
    return 0


if __name__ == "__main__":
    sys.exit(main())
