#!/bin/bash
# K1 change check: lossy parity tests with the product library, then same-call A/Bs of the
# product library against the variants named in $VARIANTS on c3 and c3s.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abk1}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_modes.py > $OUT/pytest.txt 2>&1 || { tail -20 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for wl in ${WLS:-c3 c3s}; do
  WL=$wl bash scripts/ab_quick.sh base $VARIANTS > $OUT/ab_$wl.txt 2>&1 || { cat $OUT/ab_$wl.txt; exit 1; }
  cat $OUT/ab_$wl.txt
done
