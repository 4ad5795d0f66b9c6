#!/bin/bash
# c3a end to end (pipelined chunks): the default library against K7 kept in stream order
# (WG_K7_SIDE=0) and alpha-first off (WG_ALPHA_FIRST=0), alternating, same call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-e2e_c3a}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in default noside noaf; do
    env=""; [ $v = noside ] && env="WG_K7_SIDE=0"; [ $v = noaf ] && env="WG_ALPHA_FIRST=0"
    env $env timeout -k 10 300 python bench.py --workload ${WL:-c3a} --steps 10 --warmup 3 --no-cpu-baseline \
      > $OUT/${v}_$rep.log 2>&1 || { tail $OUT/${v}_$rep.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); e=d['end_to_end']; b=e['breakdown_rank0']; print(sys.argv[2], d['value'], e['value'], {k: b[k] for k in ('parse_s','parse_wait_s','kernel_ms','d2h_ms','h2d_ms','drain_s')})" \
      $OUT/${v}_$rep.log $v
  done
done
echo E2E_AB_DONE
