#!/bin/bash
# Conversion change check: lossy + mode parity (incl. every (y, u, v) triple on the device), then
# same-call A/Bs of the working tree against libgowebp_amd_prev.so (scripts/build_prev_lib.sh) on
# c3, c3s and c2 (K1 with the fused tail; "stage" = K2 alone over the same planes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-conv1}; mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_modes.py tests/test_gpu_alpha.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 $OUT/pytest.txt
for wl in ${WLS:-c3 c3s c2}; do
  WL=$wl bash scripts/ab_quick.sh base prev $EXTRA_VARIANTS > $OUT/ab_$wl.txt 2>&1 || { cat $OUT/ab_$wl.txt; exit 1; }
  cat $OUT/ab_$wl.txt
done
