#!/bin/bash
# K1 timelines (timing builds) of the working tree ("timing") and of a previous revision
# ("timingprev", built by hand) on the workloads in $WLS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-tl1}; mkdir -p $OUT
export TMPDIR=/tmp
for wl in ${WLS:-c3s c3}; do
  for v in timing timingprev; do
    K1_TIMING_VARIANT=$v timeout -k 10 300 python scripts/k1_sections.py --workload $wl > $OUT/${wl}_$v.txt 2>&1 || { tail $OUT/${wl}_$v.txt; exit 1; }
    echo "== $wl $v"; grep -v amdgpu.ids $OUT/${wl}_$v.txt
  done
done
