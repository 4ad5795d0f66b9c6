#!/bin/bash
# Same-box A/B of the end-to-end decode (c3, automatic chunking, 16 entropy threads): the committed
# library (variant "prev", scripts/build_prev_lib.sh) against the working tree, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-e2e_prev_ab}; mkdir -p $OUT
for rep in 1 2; do
  for v in prev ""; do
    WG_LIB_VARIANT=$v timeout -k 10 300 python -u scripts/e2e_ab.py ${WL:-c3} 0 > $OUT/${v:-new}_$rep.log 2>&1 || { tail -5 $OUT/${v:-new}_$rep.log; exit 1; }
    echo "${v:-new} rep $rep:"; grep round $OUT/${v:-new}_$rep.log
  done
done
