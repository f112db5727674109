"""The README's benchmark numbers are the driver's, not the builder's: the block between
``<!-- bench-table source=FILE -->`` and ``<!-- /bench-table -->`` must equal what
``scripts/bench_table.py`` renders from that driver file (README quoted a best run)."""

import importlib.util
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bt():
    spec = importlib.util.spec_from_file_location("bench_table", os.path.join(ROOT, "scripts", "bench_table.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_readme_table_is_the_driver_bench_file():
    bt = _bt()
    text = open(os.path.join(ROOT, "README.md")).read()
    m = bt.BEGIN.search(text)
    assert m, "README.md lacks the bench-table block"
    src = m.group(1)
    assert re.fullmatch(r"BENCH_r\d\d\.json", src), src
    block = text[m.end():text.index(bt.END, m.end())]
    assert block == bt.render(os.path.join(ROOT, src))
    # every number in the table's rows comes from the driver's line
    line, _ = bt.load_line(os.path.join(ROOT, src))
    assert f"**{line['value']:.2f} ms**" in block


def test_round3_line_renders_all_extras(tmp_path):
    bt = _bt()
    line = {
        "metric": "m", "value": 48.2, "steps": 20, "warmup": 5, "ms_per_step": 60.1, "p90_ms": 55.0,
        "sync_p50_ms": 0.9, "config": {"app": "examples/quickstart"},
        "reference_equivalent": {"p50_ms": 700.0, "sync_p50_ms": 610.0},
        "deploy": {"wall_clock_s": 0.03, "warm_wall_clock_s": 0.02, "net": {"tls_handshakes": 2, "requests": 13},
                   "reference_equivalent": {"wall_clock_s": 6.1, "warm_wall_clock_s": 5.9}},
        "gpu_pod": {"reload_p50_ms": 6.0, "sync_p50_ms": 0.8, "parallelism": "dp1", "fused_ops": "hip",
                    "reference_equivalent": {"p50_ms": 5000.0}},
        "php_mysql": {"edit_to_pod_p50_ms": 3.0, "deploy_cold_s": 1.0,
                      "reference_equivalent": {"edit_to_pod_p50_ms": 650.0, "deploy_cold_s": 7.0}},
        "microservices": {"error": "boom"},
    }
    doc = {"cmd": "python3 bench.py", "where": "mi355x:1", "head": "abc",
           "run": {"stdout_tail": json.dumps(line) + "\n\n---- stderr ----\nnoise\n"}}
    p = tmp_path / "BENCH_r99.json"
    p.write_text(json.dumps(doc))
    out = bt.render(str(p))
    assert "**48.20 ms**" in out and "700 ms (**14.5x**)" in out
    assert "fused=hip" in out and "dp1" in out
    assert "php-mysql" in out and "650 ms" in out
    assert "microservices | failed: boom" in out
    assert "6.100 s / 5.900 s" in out
    readme = tmp_path / "README.md"
    readme.write_text("x\n<!-- bench-table source=BENCH_r02.json -->\nSTALE-TABLE\n<!-- /bench-table -->\ny\n")
    bt.update_readme(str(p), readme=str(readme))
    r = readme.read_text()
    assert r.startswith("x\n<!-- bench-table source=BENCH_r99.json -->\nDriver run") and r.endswith(
        "<!-- /bench-table -->\ny\n") and "STALE-TABLE" not in r


def test_round4_line_renders_the_drill_and_wan_rows():
    """A round-4 line (the builder's last MI355X run) carries the fault drill and the WAN columns;
    the table shows them once the driver's file has them."""
    out = _bt().render(os.path.join(ROOT, "profiles", "r4_bench_gpu_final.json"))
    assert "fault drill (hard crash (os._exit) of the only rank)" in out and "warm standby: yes" in out
    assert re.search(r"cluster behind 30 ms RTT / 100 Mbit/s .*\| \*\*\d+ ms\*\* \(sync [\d.]+ ms\) \|", out), out
    assert "`devspace deploy` quickstart across that link, cold" in out


def test_round5_line_renders_the_measured_deploy_and_the_wait_caveat(tmp_path):
    """Round 5: the deploy runs RUN steps (no longer control-plane only) and is measured cold, after
    an edit and unchanged; a round-4 line keeps its caveats (control plane only; microservices'
    helm wait off in both columns)."""
    bt = _bt()
    base = {"metric": "m", "value": 50.0, "steps": 20, "warmup": 5, "ms_per_step": 60.1, "p90_ms": 55.0,
            "sync_p50_ms": 1.0, "config": {"app": "examples/quickstart"},
            "reference_equivalent": {"p50_ms": 660.0, "sync_p50_ms": 605.0}}
    r5 = dict(base, deploy={"wall_clock_s": 0.96, "edit_redeploy_s": 0.12, "warm_wall_clock_s": 0.08,
                            "control_plane_only": False, "net": {"tls_handshakes": 2, "requests": 14},
                            "reference_equivalent": {"wall_clock_s": 6.05, "edit_redeploy_s": 5.22,
                                                     "warm_wall_clock_s": 5.2}},
              microservices={"edit_to_pod_p50_ms": 1.1, "deploy_cold_s": 0.15, "note": "x; the helm rollout wait "
                             "(on, as in the reference) completes", "reference_equivalent": {
                                 "edit_to_pod_p50_ms": 605.0, "deploy_cold_s": 5.26}})
    r4 = dict(base, deploy={"wall_clock_s": 0.026, "warm_wall_clock_s": 0.019, "control_plane_only": True,
                            "net": {}, "reference_equivalent": {"wall_clock_s": 5.04, "warm_wall_clock_s": 5.04}},
              microservices={"edit_to_pod_p50_ms": 0.87, "deploy_cold_s": 0.023, "note": "two deployments",
                             "reference_equivalent": {"edit_to_pod_p50_ms": 607.0, "deploy_cold_s": 0.039}})
    out = []
    for i, line in enumerate((r5, r4)):
        p = tmp_path / f"BENCH_r9{i}.json"
        p.write_text(json.dumps({"cmd": "python3 bench.py", "run": {"stdout_tail": json.dumps(line)}}))
        out.append(bt.render(str(p)))
    assert "image build runs the Dockerfile's RUN steps" in out[0] and "0.960 s / 0.120 s / 0.080 s" in out[0]
    assert "6.050 s / 5.220 s / 5.200 s (**6.3x**)" in out[0]
    assert "helm wait off" not in out[0]
    assert "control plane only: RUN steps not executed" in out[1]
    assert "microservices (helm wait off in both columns)" in out[1]


def test_wan_rows_render_the_gpu_pod_across_the_link(tmp_path):
    bt = _bt()
    line = {"metric": "m", "value": 50.0, "steps": 20, "warmup": 3, "ms_per_step": 56.0, "p90_ms": 55.0,
            "sync_p50_ms": 1.0, "config": {"app": "examples/quickstart"},
            "reference_equivalent": {"p50_ms": 660.0, "sync_p50_ms": 605.0},
            "gpu_pod": {"reload_p50_ms": 6.5, "sync_p50_ms": 1.1, "parallelism": "dp1", "fused_ops": "hip",
                        "wan": {"reload_p50_ms": 37.2, "sync_p50_ms": 16.1, "n": 10}},
            "wan": {"rtt_ms": 30, "mbit": 100, "p50_ms": 81.1, "sync_p50_ms": 16.3,
                    "reference_equivalent": {"p50_ms": 822.2, "sync_p50_ms": 723.1}}}
    p = tmp_path / "BENCH_r95.json"
    p.write_text(json.dumps({"cmd": "python3 bench.py", "run": {"stdout_tail": json.dumps(line)}}))
    out = bt.render(str(p))
    assert "cluster behind 30 ms RTT / 100 Mbit/s" in out and "**81.10 ms**" in out, out
    assert "rocm-pytorch, across that link" in out and "**37.20 ms** (sync 16.10 ms)" in out, out
