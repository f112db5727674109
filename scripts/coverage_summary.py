#!/usr/bin/env python3
"""Per-module line coverage from gcov builds (scripts/coverage.sh): runs `gcov -n` on every
.gcda under each BUILD and sums the executed / executable lines of the .cc files under SRC by
module (src/<module>/). A file built in several builds counts with its best run (the default
build and the portable one share most of src/; each has its own platform layer). Files that
never ran (no .gcda) count as 0 %.

    python scripts/coverage_summary.py build/coverage [build/coverage-portable ...] src
"""
import collections
import glob
import os
import re
import subprocess
import sys


def main(builds, src):
    src = os.path.abspath(src)
    seen = {}
    gcdas = [(b, g) for b in builds for g in glob.glob(os.path.join(b, "**", "*.gcda"), recursive=True)]
    for build, gcda in gcdas:
        r = subprocess.run(["gcov", "-n", "-o", os.path.dirname(gcda), gcda], capture_output=True, text=True,
                           cwd=build)
        for m in re.finditer(r"File '([^']+)'\nLines executed:([\d.]+)% of (\d+)", r.stdout):
            path, pct, total = os.path.abspath(os.path.join(build, m.group(1))), float(m.group(2)), int(m.group(3))
            if not path.startswith(src + os.sep) or not path.endswith(".cc"):
                continue
            hit = round(pct * total / 100)
            if hit >= seen.get(path, (0, 0))[0]:
                seen[path] = (hit, total)
    for path in glob.glob(os.path.join(src, "**", "*.cc"), recursive=True):
        if os.sep + "python" + os.sep in path or os.sep + "helper" + os.sep in path or path.endswith("main.cc"):
            continue  # the pybind11 module, the in-container helper and main are not in this build
        if path not in seen:
            with open(path, errors="replace") as f:
                seen[path] = (0, max(1, sum(1 for line in f if line.strip() and not line.strip().startswith("//"))))
    mods = collections.defaultdict(lambda: [0, 0])
    for path, (hit, total) in seen.items():
        mod = os.path.relpath(path, src).split(os.sep)[0]
        mods[mod][0] += hit
        mods[mod][1] += total
    hit_all = sum(h for h, _ in mods.values())
    tot_all = sum(t for _, t in mods.values())
    print(f"{'module':<12} {'lines':>7} {'executed':>9} {'coverage':>9}")
    for mod in sorted(mods):
        h, t = mods[mod]
        print(f"src/{mod:<8} {t:>7} {h:>9} {100.0 * h / t:>8.1f}%")
    print(f"{'total':<12} {tot_all:>7} {hit_all:>9} {100.0 * hit_all / tot_all:>8.1f}%")


if __name__ == "__main__":
    args = sys.argv[1:]
    main(args[:-1] if len(args) > 1 else args, args[-1] if len(args) > 1 else "src")
