#!/bin/bash
# Round-5 check C: the latency / batch-size table of the lossy path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05c}
mkdir -p $OUT
export TMPDIR=/tmp
echo "=== latency ($(date +%T))"
timeout -k 10 400 python -u scripts/latency_table.py --out $OUT/latency_table.json > $OUT/latency.log 2>&1
rc=$?; echo "=== latency rc=$rc"; tail -3 $OUT/latency.log; [ $rc -eq 0 ] || exit $rc
echo ALLDONE
