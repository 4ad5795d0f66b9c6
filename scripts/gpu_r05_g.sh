#!/bin/bash
# Round-5 check G (measurement builds): K7 block statistics on the c3a ALPH streams and on c5, K1's
# per-section cycle shares on c3 and c3s (timing build), and the host entropy stage's -O2 vs
# x86-64-v3 A/B on the box's CPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05g}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 30 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
step k7_stats_c3a 300 python -u scripts/k7_stats.py 64 c3a
step k7_stats_c5 300 python -u scripts/k7_stats.py 64 c5
step k1_sections_c3 300 python -u scripts/k1_sections.py --workload c3
step k1_sections_c3s 300 python -u scripts/k1_sections.py --workload c3s
TAG=${TAG:-r05g} bash scripts/host_parse_ab.sh > $OUT/host_ab.log 2>&1 || { tail $OUT/host_ab.log; exit 1; }
cat $OUT/host_ab.log
echo CHECK_G_DONE
