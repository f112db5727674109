"""A/B of how port-forwarded connections reach the pod on a remote cluster: the bench's WAN loop
(quickstart edit -> new HTTP response through `devspace dev`, cluster behind a 30 ms RTT /
100 Mbit link) with DEVSPACE_PORTFORWARD_VIA=kubelet (held connections retried from the laptop,
one round trip per refused attempt) against the default, `auto` (the hold done in the pod by the
in-container helper). Rounds alternate so both modes see the same box. One JSON line.

  python scripts/ab_portforward_via.py [--rounds 2] [--steps 10]
"""

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    out = {m: {"reload_ms": [], "app_requests": [], "refused_per_edit": [], "via": set()} for m in ("kubelet", "auto")}
    for r in range(args.rounds):
        for mode in (("kubelet", "auto") if r % 2 == 0 else ("auto", "kubelet")):
            os.environ["DEVSPACE_PORTFORWARD_VIA"] = mode
            d = tempfile.mkdtemp(prefix=f"ab-via-{mode}-")
            res = bench.quickstart_loop(d, args.steps, 1, tls=True, cold=True, wan=bench.WAN)
            o = out[mode]
            o["reload_ms"] += res["reload_ms"]
            o["app_requests"] += res.get("app_requests") or []
            pf = res.get("portforward") or {}
            o["refused_per_edit"].append(pf.get("refused_per_edit"))
            o["via"] |= set(pf.get("via") or [])
            print(f"round {r} {mode}: p50 {_pct(res['reload_ms'], 0.5):.1f} ms", file=sys.stderr, flush=True)
    summary = {"what": "bench WAN loop (30 ms RTT, 100 Mbit/s, cold node restarts): edit -> new HTTP response "
                       "through the port-forward; kubelet = retries from the laptop, auto = hold in the pod "
                       "(devspace-helper forward)",
               "rounds": args.rounds, "steps_per_round": args.steps}
    for mode, o in out.items():
        summary[mode] = {"p50_ms": round(_pct(o["reload_ms"], 0.5), 2), "p90_ms": round(_pct(o["reload_ms"], 0.9), 2),
                         "min_ms": round(min(o["reload_ms"]), 2), "max_ms": round(max(o["reload_ms"]), 2),
                         "n": len(o["reload_ms"]), "samples_ms": [round(x, 1) for x in o["reload_ms"]],
                         "app_requests_per_edit": round(sum(o["app_requests"]) / max(1, len(o["app_requests"])), 2),
                         "refused_per_edit": o["refused_per_edit"], "via": sorted(o["via"])}
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
