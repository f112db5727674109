#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 run (ROCm 7 writes a rocpd SQLite database by default).

    python scripts/rocpd_summary.py gpurun_out/prof_smoke/smoke_results.db [--top 30]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    total_us = sum(r[2] for r in rows)
    calls = sum(r[1] for r in rows)
    print(f"kernels: {len(rows)} distinct, {calls} dispatches, {total_us:.1f} us total GPU kernel time")
    print(f"{'calls':>6} {'total_us':>10} {'avg_us':>9} {'pct':>6}  kernel")
    for name, n, tot, avg, pct in rows[: a.top]:
        short = name if len(name) <= 110 else name[:107] + "..."
        print(f"{n:>6} {tot:>10.2f} {avg:>9.2f} {pct:>6.2f}  {short}")


if __name__ == "__main__":
    main()
