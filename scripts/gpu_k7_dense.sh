#!/bin/bash
# K7 dense-updater registration and direct colorspace emission: the K7 / lossless / alpha / fuzz /
# modes / next-row GPU tests on the working tree, then a same-call A/B of the committed library
# (variant "prev", scripts/build_prev_lib.sh) against the working tree on c5, c3a, c3 and c3rgb565
# (bench lines without the CPU / end-to-end legs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-k7dense}
mkdir -p $OUT
export TMPDIR=/tmp
echo "=== pytest ($(date +%T))"
timeout -k 10 500 python -u -m pytest tests/test_gpu_k7.py tests/test_gpu_vp8l.py tests/test_gpu_alpha.py tests/test_gpu_fuzz.py \
  tests/test_gpu_next_rows.py tests/test_gpu_modes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "=== pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; }
for rep in 1 2; do
  for v in prev ""; do
    for w in ${AB_WLS:-c5 c3a c3 c3rgb565}; do
      WG_LIB_VARIANT=$v timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-e2e \
        > $OUT/ab_${w}_${v:-new}_$rep.log 2>&1 || { tail $OUT/ab_${w}_${v:-new}_$rep.log; exit 1; }
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], d['value'], {k: round(x, 3) for k, x in d['kernel_ms'].items()})" \
        $OUT/ab_${w}_${v:-new}_$rep.log ${v:-new} $w
    done
  done
done
echo K7DENSE_DONE
