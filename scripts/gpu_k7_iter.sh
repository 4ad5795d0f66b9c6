#!/bin/bash
# K7 iteration: the K7 / lossless / alpha GPU tests, the timing build's block statistics on the
# c3a ALPH streams, and a same-call A/B of the committed library (variant "prev") against the
# working tree on c3a and c5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-k7iter}
mkdir -p $OUT
export TMPDIR=/tmp
echo "=== pytest ($(date +%T))"
timeout -k 10 400 python -u -m pytest tests/test_gpu_k7.py tests/test_gpu_vp8l.py tests/test_gpu_alpha.py tests/test_gpu_next_rows.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "=== pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 300 python -u scripts/k7_stats.py 64 c3a > $OUT/k7_stats_c3a.log 2>&1 || { tail $OUT/k7_stats_c3a.log; exit 1; }
head -14 $OUT/k7_stats_c3a.log | tail -12
for v in prev "" prev ""; do
  for w in ${AB_WLS:-c3a c5}; do
    WG_LIB_VARIANT=$v timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-e2e \
      > $OUT/ab_${w}_${v:-new}.log 2>&1 || { tail $OUT/ab_${w}_${v:-new}.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], d['value'], {k: round(x, 3) for k, x in d['kernel_ms'].items()})" \
      $OUT/ab_${w}_${v:-new}.log ${v:-new} $w
  done
done
echo K7ITER_DONE
