#!/usr/bin/env python3
"""Steady-state kernel durations from a rocprofv3 --kernel-trace run of bench.py.

Usage: trace_steady.py <prof dir> <warmup launches> [bench json line file]

Per kernel (launches at its largest grid: the workload's batch; bench.py also runs small sanity
batches): the number of launches, the mean over all of them (what rocprofv3 --stats reports), the
mean and median without the first <warmup> launches (bench.py's untimed warm-up steps), and --
given the bench line of the same command -- the line's kernel_ms for comparison (VERDICT r5 item 1:
the profile's average within 3 % of the line).  Prints one JSON object."""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d, skip = sys.argv[1], int(sys.argv[2])
    line = None
    if len(sys.argv) > 3 and os.path.exists(sys.argv[3]):
        ls = [x for x in open(sys.argv[3]) if x.startswith("{")]
        line = json.loads(ls[-1]) if ls else None
    rows = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            short = name.split("(")[0].split("<")[0].replace("void ", "").split("::")[-1].strip()
            grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0) * int(r.get("Grid_Size_Y") or 1)
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            rows[short].append((int(r["Start_Timestamp"]), grid, dur))
    out = {}
    for k, rs in sorted(rows.items()):
        top = max(g for _, g, _ in rs)
        ds = [dur for _, g, dur in sorted(rs) if g == top]
        steady = ds[skip:] if len(ds) > skip else ds
        ent = {"launches": len(ds), "mean_all_ms": round(statistics.mean(ds), 4),
               "mean_steady_ms": round(statistics.mean(steady), 4), "median_steady_ms": round(statistics.median(steady), 4),
               "first_ms": round(ds[0], 4)}
        if line and k in line.get("kernel_ms", {}):
            ent["line_kernel_ms"] = line["kernel_ms"][k]
            ent["steady_vs_line"] = round(ent["mean_steady_ms"] / line["kernel_ms"][k], 4)
            ent["all_vs_line"] = round(ent["mean_all_ms"] / line["kernel_ms"][k], 4)
        out[k] = ent
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
