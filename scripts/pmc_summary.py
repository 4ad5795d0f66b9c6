#!/usr/bin/env python3
"""Average per-launch rocprofv3 counters per kernel: pmc_summary.py <prof dir>..."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("__amd"):
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            acc[(k, r["Counter_Name"], r["VGPR_Count"], r["Grid_Size"])].append(float(r["Counter_Value"]))
    for (k, c, vg, gs), v in sorted(acc.items()):
        print(f"{k:48s} vgpr={vg:4s} grid={gs:10s} {c:22s} n={len(v):2d} avg={sum(v) / len(v):.6g}")
