#!/bin/bash
# rocprofv3 passes for the bench workload: kernel-trace stats, then PMC passes (separate runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
WL=${WL:-c3}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="python3 bench.py --workload $WL --steps ${STEPS:-3} --warmup ${WARMUP:-1} --no-cpu-baseline --no-e2e"
run() {  # run <name> <timeout> <rocprofv3 args...>
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 $to rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- $BENCH > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
[ -z "$PMC_ONLY" ] && run trace 240 --kernel-trace --stats
if [ -n "$PMC1" ]; then run pmc1 240 --pmc $PMC1; fi
if [ -n "$PMC2" ]; then run pmc2 240 --pmc $PMC2; fi
if [ -n "$PMC3" ]; then run pmc3 240 --pmc $PMC3; fi
if [ -n "$PMC4" ]; then run pmc4 240 --pmc $PMC4; fi
if [ -n "$PMC5" ]; then run pmc5 240 --pmc $PMC5; fi
if [ -n "$PMC6" ]; then run pmc6 240 --pmc $PMC6; fi
find $OUT -name "*.csv" | head -50
