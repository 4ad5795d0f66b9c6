#!/bin/bash
# Same-call A/B of several library variants ($VARIANTS, "new" = the working tree's product library,
# others = libgowebp_amd_<name>.so) on the workloads $WLS (name or name:batch), $REPS rounds,
# alternating variants within each round.  Optional $TESTS first (GPU pytest on the product library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abmulti}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  echo "=== pytest ($(date +%T))"
  timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
  rc=$?; echo "=== pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; }
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-prev new}; do
    for w in ${WLS:-c3}; do
      lib=$v; [ $v = new ] && lib=""
      wl=${w%%:*}; bt=256; [ "$wl" != "$w" ] && bt=${w#*:}
      WG_LIB_VARIANT=$lib timeout -k 10 300 python bench.py --workload $wl --batch $bt --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-e2e $BENCH_ARGS \
        > $OUT/ab_${w}_${v}_$rep.log 2>&1 || { tail $OUT/ab_${w}_${v}_$rep.log; exit 1; }
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['kernel_ms'].items()})" \
        $OUT/ab_${w}_${v}_$rep.log $v $w
    done
  done
done
echo AB_DONE
