#!/bin/bash
# A/B of K1 variants on the GPU box: for each variant library (built beforehand with
# `make -C go-webp_amd/csrc VARIANT=<name> K1SRC=device/<file>.hip`; "base" = the product
# library), a timed bench run and one rocprofv3 PMC pass for instruction counts.
# Usage: bash scripts/ab_k1.sh base v1 v2 ...   -> gpurun_out/ab/<name>.{json,pmc}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in "$@"; do
  if [ "$v" = base ]; then unset WG_LIB_VARIANT; else export WG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "STOP: bench $v rc=$rc"; tail -5 gpurun_out/ab/$v.err; exit $rc; fi
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES -d gpurun_out/ab/prof_$v -o p \
    --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/$v.prof.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "STOP: rocprof $v rc=$rc"; tail -5 gpurun_out/ab/$v.prof.log; exit $rc; fi
  python3 - "$v" <<'PY'
import csv, glob, json, sys, collections
v = sys.argv[1]
j = json.load(open(f"gpurun_out/ab/{v}.json"))
acc = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/ab/prof_{v}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "recon" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
c = {k: sum(x) / len(x) for k, x in acc.items()}
print(f"{v:12s} K1 {j['kernel_ms']['vp8_recon_filter_kernel']:7.3f} ms  K2 {j['kernel_ms'].get('yuv_to_rgba_kernel', 0):6.3f} ms  "
      f"VALU {c.get('SQ_INSTS_VALU', 0):.3e}  SALU {c.get('SQ_INSTS_SALU', 0):.3e}  LDS {c.get('SQ_INSTS_LDS', 0):.3e}  "
      f"value {j['value']}")
PY
done
