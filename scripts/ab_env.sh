#!/bin/bash
# Same-call A/B of environment settings on the product library: each argument is one setting
# ("-" = none, else NAME=VALUE[,NAME=VALUE...]); one timed bench run each, two alternating rounds,
# kernel times side by side.
# Usage: WL=c3 bash scripts/ab_env.sh - WG_K1_LATE_WAVES=0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abe
for round in 1 2; do
for v in "$@"; do
  envs=()
  [ "$v" != "-" ] && IFS=',' read -ra envs <<< "$v"
  tag=$(echo "$v" | tr '=,' '__')
  ( for e in "${envs[@]}"; do export "$e"; done
    timeout -k 10 240 python3 bench.py --workload ${WL:-c3} --steps ${STEPS:-10} --warmup 2 \
      --no-cpu-baseline --no-e2e > gpurun_out/abe/$tag.$round.json 2> gpurun_out/abe/$tag.$round.err )
  rc=$?; if [ $rc -ne 0 ]; then echo "STOP: bench $v rc=$rc"; tail -5 gpurun_out/abe/$tag.$round.err; exit $rc; fi
  python3 -c "
import json; j=json.load(open('gpurun_out/abe/$tag.$round.json'))
print('%-28s r$round' % '$v', ' '.join('%s %.3f' % (k[:12], x) for k, x in j['kernel_ms'].items()), ' value', j['value'])"
done
done
