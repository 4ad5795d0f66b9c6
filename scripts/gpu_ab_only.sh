#!/bin/bash
# Same-call A/B only (no tests): the product library against $VARIANTS on $WLS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abonly}
mkdir -p $OUT
for wl in ${WLS:-c3 c3s}; do
  WL=$wl bash scripts/ab_quick.sh base $VARIANTS > $OUT/ab_$wl.txt 2>&1 || { cat $OUT/ab_$wl.txt; exit 1; }
  cat $OUT/ab_$wl.txt
done
