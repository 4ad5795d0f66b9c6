#!/bin/bash
# K7 variant check: lossless parity with the variant library $V (test_gpu_k7 streams incl. far
# copies, the C5 SHAs, the lossless fuzz set), then same-call c5 A/Bs of the product library
# against $V (and $EXTRA_VARIANTS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-k7a}; mkdir -p $OUT
export TMPDIR=/tmp
for v in $V $EXTRA_VARIANTS; do
  WG_LIB_VARIANT=$v timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_k7.py tests/test_gpu_vp8l.py tests/test_gpu_fuzz.py > $OUT/pytest_$v.txt 2>&1 || { tail -30 $OUT/pytest_$v.txt; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.txt)"
done
WL=c5 bash scripts/ab_quick.sh base $V $EXTRA_VARIANTS > $OUT/ab_c5.txt 2>&1 || { cat $OUT/ab_c5.txt; exit 1; }
cat $OUT/ab_c5.txt
