#!/bin/bash
# Same-call end-to-end A/B of library variants ($VARIANTS, "new" = the working tree's product
# library): bench.py's end_to_end leg (c3 by default) alternated $REPS times; prints the value and
# the pipeline breakdown (parse, arena waits, drain) per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-e2e_lib_ab}; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-3}); do
  for v in ${VARIANTS:-prev new}; do
    lib=$v; [ $v = new ] && lib=""
    WG_LIB_VARIANT=$lib timeout -k 10 300 python bench.py --workload ${WL:-c3} --steps 3 --warmup 1 --no-cpu-baseline \
      > $OUT/e2e_${v}_$rep.log 2>&1 || { tail $OUT/e2e_${v}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])['end_to_end']; b=d['breakdown_rank0']; print(sys.argv[2], d['value'], d['seconds'], 'parse', round(b['parse_s'],4), 'wait', round(b['parse_wait_s'],4), 'drain', round(b['drain_s'],4))" $OUT/e2e_${v}_$rep.log $v
  done
done
echo E2E_AB_DONE
