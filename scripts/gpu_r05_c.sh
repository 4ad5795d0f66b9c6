#!/bin/bash
# Round-5 check C: the latency / batch-size table of the lossy path, then a PC-sampling probe
# of K1 on c3 (rocprofv3 host-trap sampling; stops quietly if the box does not support it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05c}
mkdir -p $OUT
export TMPDIR=/tmp
echo "=== latency ($(date +%T))"
timeout -k 10 400 python -u scripts/latency_table.py --out $OUT/latency_table.json > $OUT/latency.log 2>&1
rc=$?; echo "=== latency rc=$rc"; tail -3 $OUT/latency.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PCS" ]; then
  echo "=== pcs ($(date +%T))"
  timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-host_trap} \
    --pc-sampling-unit ${PCS_UNIT:-time} --pc-sampling-interval ${PCS_INTERVAL:-1} -d $OUT/pcs -o pcs \
    --output-format csv -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
    > $OUT/pcs.log 2>&1
  rc=$?; echo "=== pcs rc=$rc"; tail -5 $OUT/pcs.log; find $OUT/pcs -type f | head; 
fi
echo ALLDONE
