#!/bin/bash
# Round-5 check F: soaks of the final K7 / K4 / K1 code (c5, c3a, c3), the end-to-end thread /
# split A/B and the latency / batch-size table.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05f}
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
if [ -z "$NO_SOAK" ]; then
  step soak_c5 300 python -u scripts/soak_fused.py ${N5:-100} c5_ll2048
  step soak_c3a 300 python -u scripts/soak_fused.py ${N3A:-30} c3a_4k
  step soak_c3 300 python -u scripts/soak_fused.py ${N3:-40} c3_4k
fi
[ -n "$NO_AB" ] || { TAG=${TAG:-r05f}/e2e_ab bash scripts/e2e_threads_ab.sh > $OUT/e2e_ab.log 2>&1 || { tail $OUT/e2e_ab.log; exit 1; }; cat $OUT/e2e_ab.log; }
[ -n "$NO_LAT" ] || { TAG=${TAG:-r05f} bash scripts/gpu_r05_c.sh || exit $?; }
echo CHECK_F_DONE
