#!/bin/bash
# Round-5 final check: the whole GPU suite and smoke on the final code, then the bench lines of every
# workload (c3 with its end-to-end and CPU legs; c3s, c5, c2; the next rows c3a, c3rgb565, anim).
# Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05final}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
for w in ${BENCH_WLS:-c3 c3s c5 c3a c3rgb565 anim c2}; do
  step bench_$w 400 python bench.py --workload $w --steps 10 --warmup 3
  grep -h '^{' $OUT/bench_$w.log > $OUT/bench_$w.json
done
echo FINAL_DONE
