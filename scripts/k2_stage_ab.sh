#!/bin/bash
# Same-call A/B of the YUV->RGBA stage alone (the c3 bench line's roofline_yuv_to_rgba) between a
# committed library (variant "prev", scripts/build_prev_lib.sh <rev>) and the working tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-k2ab}; mkdir -p $OUT
for rep in 1 2 3; do
  for v in prev ""; do
    WG_LIB_VARIANT=$v timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e \
      > $OUT/c3_${v:-new}_$rep.log 2>&1 || { tail $OUT/c3_${v:-new}_$rep.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline_yuv_to_rgba']; print(sys.argv[2], d['value'], d['kernel_ms'], 'K2 stage', r['avg_launch_ms'], r['frac'])" \
      $OUT/c3_${v:-new}_$rep.log ${v:-new}
  done
done
