#!/bin/bash
# K7 on the context's side stream (beside K1 / K2 for small batches): the GPU tests that run
# alpha / lossless / animation batches, then a same-call A/B against WG_K7_SIDE=0 on anim and
# small c3a batches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-k7side}
mkdir -p $OUT
export TMPDIR=/tmp
echo "=== pytest ($(date +%T))"
timeout -k 10 500 python -u -m pytest tests/test_gpu_anim.py tests/test_gpu_alpha.py tests/test_gpu_next_rows.py tests/test_gpu_k7.py \
  tests/test_gpu_vp8l.py tests/test_gpu_pipeline.py tests/test_gpu_modes.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "=== pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; }
for side in 0 1 0 1; do
  for wb in "anim 64" "c3a 32" "c3a 64" "c3a 256"; do
    set -- $wb
    WG_K7_SIDE=$side timeout -k 10 300 python bench.py --workload $1 --batch $2 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e \
      > $OUT/ab_$1_$2_$side.log 2>&1 || { tail $OUT/ab_$1_$2_$side.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('side', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['kernel_ms'].items()})" \
      $OUT/ab_$1_$2_$side.log $side "$1x$2"
  done
done
echo K7SIDE_DONE
