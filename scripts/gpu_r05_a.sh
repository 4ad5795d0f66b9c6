#!/bin/bash
# Round-5 check A: the whole GPU suite, smoke, bench lines for c3 and c5 (with the libwebp CPU
# legs), soaks of the final K7 / K1 code, then the c5 profile refresh (trace + PMC passes).
# Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05a}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
for w in ${BENCH_WLS:-c3 c5}; do
  step bench_$w 400 python bench.py --workload $w --steps 10 --warmup 3
  grep -h '^{' $OUT/bench_$w.log > $OUT/bench_$w.json
done
if [ -n "$SOAK" ]; then
  step soak_c5 300 python -u scripts/soak_fused.py ${N5:-100} c5_ll2048
  step soak_c3 300 python -u scripts/soak_fused.py ${N3:-40} c3_4k
fi
if [ -n "$PROF" ]; then
  TAG=${TAG:-r05a} WLS="$PROF" bash scripts/gpu_r04_final_prof.sh > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
  tail -3 $OUT/prof.log
fi
echo ALLDONE
