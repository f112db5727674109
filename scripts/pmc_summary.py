#!/usr/bin/env python3
"""Mean per dispatch of each PMC counter per kernel, from rocprofv3 --pmc --output-format csv
output (every *counter_collection.csv under the given directory)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "?").replace("void ", "")
            k = k if len(k) < 80 else k[:77] + "..."
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            meta[k] = (row.get("VGPR_Count", row.get("Arch_VGPR_Count", "?")), row.get("LDS_Block_Size", "?"))
    for k in sorted(acc):
        vals = {c: round(sum(v) / len(v)) for c, v in sorted(acc[k].items())}
        print(f"{k} vgpr={meta[k][0]} lds={meta[k][1]} {vals}")


if __name__ == "__main__":
    main(sys.argv[1])
