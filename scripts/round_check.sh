#!/bin/bash
# One GPU call: parity tests, smoke, c3 bench (with CPU baselines), c2/c5 bench lines, and the
# rocprofv3 trace + PMC passes of c3 (kernel stats and HBM traffic).  Stops at the first
# crash/timeout.  Usage: TAG=r01_x bash scripts/round_check.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_c3 600 python bench.py --steps 10 --warmup 3
step bench_c2 300 python bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e
step bench_c5 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e
if [ -z "$SKIP_PROF" ]; then
  TAG=$TAG WL=c3 STEPS=3 PMC1="FETCH_SIZE" PMC2="WRITE_SIZE" \
    PMC3="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
    timeout -k 10 900 bash scripts/profile.sh > gpurun_out/profile_$TAG.log 2>&1
  rc=$?; tail -n 5 gpurun_out/profile_$TAG.log; [ $rc -eq 0 ] || { echo "STOP: profile rc=$rc"; exit $rc; }
fi
