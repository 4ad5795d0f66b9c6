#!/bin/bash
# K7 check: stage-entry parity, the lossless batch tests, K7 statistics, c5 bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n ${TAILN:-6} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
TAILN=4 step k7_tests 300 python -u -m pytest tests/test_gpu_k7.py tests/test_gpu_vp8l.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
TAILN=30 step k7_stats 200 python -u scripts/k7_stats.py 256
TAILN=2 step bench_c5 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e
