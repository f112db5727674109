#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (kernel trace) into a text table for profiles/.

rocpd's `top_kernels` view reports durations in microseconds."""
import sqlite3
import sys


def short(name, n=90):
    name = name.replace("void ", "")
    if name.startswith("Cijk_"):
        mt = [p for p in name.split("_") if p.startswith("MT")]
        return "hipBLASLt GEMM " + (mt[0] if mt else "") + " (" + name[:32] + "...)"
    return name if len(name) <= n else name[: n - 3] + "..."


def main(db, top=25):
    c = sqlite3.connect(db)
    total = c.execute("select sum(total_duration), sum(total_calls) from top_kernels").fetchone()
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels "
                     "order by total_duration desc limit ?", (top,)).fetchall()
    out = [f"# rocprofv3 --kernel-trace --stats: {db}",
           f"# total kernel time {total[0] / 1e3:.3f} ms over {total[1]} dispatches",
           f"{'calls':>7} {'total_ms':>10} {'avg_us':>9} {'pct':>6}  kernel"]
    for name, calls, dur, avg, pct in rows:
        out.append(f"{calls:>7} {dur / 1e3:>10.3f} {avg:>9.2f} {pct:>6.2f}  {short(name)}")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
