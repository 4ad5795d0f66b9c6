#!/bin/bash
# Alpha-first batches (K7 -> K3 -> K4 into scratch planes before K1, whose tail / K2 take A from
# them): the whole GPU suite, the alpha / animation / modes tests again with K7 kept in stream order
# (WG_K7_SIDE=0: every alpha batch alpha-first), then a same-call A/B -- the committed library
# ("prev") vs the working tree on c3 (no alpha: the tail's default instantiation), and c3a with
# alpha-first on / off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-alphafirst}
mkdir -p $OUT
export TMPDIR=/tmp
echo "=== pytest all ($(date +%T))"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "=== pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; }
echo "=== pytest WG_K7_SIDE=0 ($(date +%T))"
WG_K7_SIDE=0 timeout -k 10 500 python -u -m pytest tests/test_gpu_alpha.py tests/test_gpu_next_rows.py tests/test_gpu_anim.py tests/test_gpu_modes.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_noside.log 2>&1
rc=$?; echo "=== pytest rc=$rc"; tail -2 $OUT/pytest_noside.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_noside.log | head; exit $rc; }
for rep in 1 2; do
  for v in prev new newoff; do
    for w in c3 c3a; do
      [ $v = newoff ] && [ $w = c3 ] && continue
      lib=$v; af=1; [ $v = newoff ] && { lib=new; af=0; }
      [ $lib = new ] && lib=""
      WG_LIB_VARIANT=$lib WG_ALPHA_FIRST=$af timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-e2e \
        > $OUT/ab_${w}_${v}_$rep.log 2>&1 || { tail $OUT/ab_${w}_${v}_$rep.log; exit 1; }
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['kernel_ms'].items()})" \
        $OUT/ab_${w}_${v}_$rep.log $v $w
    done
  done
done
echo ALPHAFIRST_DONE
