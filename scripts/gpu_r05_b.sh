#!/bin/bash
# Round-5 check B: the new-row parity tests, then bench lines + rocprof trace/PMC for the three
# "next"-row workloads (c3a: K4, c3rgb565: K6, anim: K5).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05b}
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
  step pytest_next 400 python -u -m pytest tests/test_gpu_next_rows.py tests/test_gpu_anim.py tests/test_gpu_modes.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
fi
for w in ${BENCH_WLS:-c3a c3rgb565 anim}; do
  step bench_$w 400 python bench.py --workload $w --steps 10 --warmup 3
  grep -h '^{' $OUT/bench_$w.log > $OUT/bench_$w.json
done
if [ -n "$PROF" ]; then
  TAG=${TAG:-r05b} WLS="$PROF" bash scripts/gpu_r04_final_prof.sh > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
  tail -3 $OUT/prof.log
fi
echo ALLDONE
