#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 PMC passes -> profiles/pmc_traffic.json.

Usage: make_pmc_traffic.py <workload name> <prof dir> [<workload name> <prof dir> ...]
Each prof dir holds the passes written by scripts/profile.sh with PMC2=FETCH_SIZE and
PMC3=WRITE_SIZE (one counter block each: FETCH_SIZE and WRITE_SIZE cannot share a pass).
Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE/WRITE_SIZE are KiB; FETCH_SIZE reports
half the bytes of a coalesced streaming read on gfx950, so it is doubled; WRITE_SIZE is
exact for 16-byte-per-lane streaming stores.  Averages over all launches of a kernel.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {k: k for k in ("vp8_recon_filter_kernel", "yuv_to_rgba_kernel", "vp8l_transforms_kernel", "alpha_kernel",
                           "vp8l_resolve_kernel", "emit_kernel", "anim_compose_kernel")}


def per_kernel(d):
    """Averages over the kernel's launches at its largest grid (the workload's batch; the
    bench also runs small sanity batches)."""
    rows = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            for key in KERNELS:
                if key in r["Kernel_Name"]:
                    rows[key].append((int(r["Grid_Size"]), r["Counter_Name"], float(r["Counter_Value"])))
    acc = collections.defaultdict(list)
    for key, rs in rows.items():
        top = max(g for g, _, _ in rs)
        for g, name, v in rs:
            if g == top:
                acc[(key, name)].append(v)
    out = {}
    avg = lambda key, name: sum(acc[(key, name)]) / len(acc[(key, name)]) if acc.get((key, name)) else None  # noqa: E731
    for key in KERNELS:
        fetch = acc.get((key, "FETCH_SIZE"))
        write = acc.get((key, "WRITE_SIZE"))
        ent = {}
        if fetch and write:
            fb = 2.0 * 1024 * sum(fetch) / len(fetch)
            wb = 1024.0 * sum(write) / len(write)
            ent = {"bytes": int(fb + wb), "read_bytes": int(fb), "write_bytes": int(wb),
                   "launches": len(fetch), "source": os.path.relpath(d, ROOT)}
        # instruction issue (SQ counters, per launch): VALU wave-instructions, and the share of
        # lanes active in them, VALUUtilization = SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)
        valu, act, thr = avg(key, "SQ_INSTS_VALU"), avg(key, "SQ_ACTIVE_INST_VALU"), avg(key, "SQ_THREAD_CYCLES_VALU")
        if valu:
            ent["valu"] = {"insts_valu": int(valu), "insts_salu": int(avg(key, "SQ_INSTS_SALU") or 0),
                           "insts_lds": int(avg(key, "SQ_INSTS_LDS") or 0),
                           "valu_utilization": round(thr / (64.0 * act), 4) if thr and act else None,
                           "wait_any_frac": round(avg(key, "SQ_WAIT_ANY") / avg(key, "SQ_WAVE_CYCLES"), 4)
                           if avg(key, "SQ_WAIT_ANY") and avg(key, "SQ_WAVE_CYCLES") else None,
                           "source": os.path.relpath(d, ROOT)}
        if ent:
            out[key] = ent
    return out


def main():
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    args = sys.argv[1:]
    for name, d in zip(args[0::2], args[1::2]):
        new = per_kernel(d)
        for k, v in new.items():  # a pass set with only traffic (or only SQ counters) keeps the other
            data.setdefault(name, {}).setdefault(k, {}).update(v)
    data["_note"] = ("HBM bytes per launch: 2*FETCH_SIZE + WRITE_SIZE (KiB->B), rocprofv3 --pmc in separate "
                     "passes (scripts/profile.sh); FETCH_SIZE doubling per MI355X_MICROARCH.md gfx950 note. "
                     "valu: SQ instruction counters per launch; valu_utilization = SQ_THREAD_CYCLES_VALU / "
                     "(64 * SQ_ACTIVE_INST_VALU)")
    json.dump(data, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(data, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
