#!/bin/bash
# GPU-box check: parity tests, smoke, short bench.  Stops at the first crash/timeout
# (exit codes other than 0/1), never retries a failing GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -x --timeout 600 -p no:cacheprovider
rc_t=$?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if [ "${RUN_BENCH:-1}" = "1" ]; then
  step bench 900 python bench.py --steps 5 --warmup 2 --cpu-seconds 8
fi
exit $rc_t
