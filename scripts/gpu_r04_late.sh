#!/bin/bash
# K1 late waves: lossy parity with them on (and with 3 late waves on 11 round-robin waves), then
# same-call A/Bs on c3 / c3s / c2, then the timing build's quad timeline with and without.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-late1}; mkdir -p $OUT
export TMPDIR=/tmp
WG_K1_LATE_WAVES=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_modes.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
WG_K1_LATE_WAVES=3 WG_K1_RECON_WAVES=11 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $OUT/pytest_11_3.txt 2>&1 || { tail -30 $OUT/pytest_11_3.txt; exit 1; }
tail -2 $OUT/pytest_11_3.txt
for wl in c3 c3s c2; do
  WL=$wl bash scripts/ab_env.sh - WG_K1_LATE_WAVES=2 WG_K1_RECON_WAVES=11,WG_K1_LATE_WAVES=3 > $OUT/ab_$wl.txt 2>&1 || { cat $OUT/ab_$wl.txt; exit 1; }
  cat $OUT/ab_$wl.txt
done
WG_K1_LATE_WAVES=2 timeout -k 10 300 python scripts/k1_sections.py --workload c3 > $OUT/sections_late2.txt 2>&1 || { tail $OUT/sections_late2.txt; exit 1; }
timeout -k 10 300 python scripts/k1_sections.py --workload c3 > $OUT/sections_late0.txt 2>&1 || { tail $OUT/sections_late0.txt; exit 1; }
grep -A3 timeline $OUT/sections_late2.txt; grep "quad start" $OUT/sections_late2.txt $OUT/sections_late0.txt
