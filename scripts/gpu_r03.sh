#!/bin/bash
# Round-3 check: GPU tests, then c5 bench (K7 + K3), then library A/B (VARIANTS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n ${TAILN:-4} "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider
fi
step bench_c5 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e
if [ -n "$VARIANTS" ]; then
  bash scripts/ab_lib.sh || exit $?
fi
