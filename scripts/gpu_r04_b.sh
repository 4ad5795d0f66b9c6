#!/bin/bash
# Round-4 check B: the whole GPU suite, smoke, then full bench lines for c3 (headline) and c3s
# (entropy stress) with their CPU baselines.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04b}
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
  step pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_c3 400 python bench.py --steps 10 --warmup 3
step bench_c3s 400 python bench.py --workload c3s --steps 10 --warmup 3
step bench_c5 400 python bench.py --workload c5 --steps 10 --warmup 3
for w in c3 c3s c5; do grep -h '^{' $OUT/bench_$w.log > $OUT/bench_$w.json; done
