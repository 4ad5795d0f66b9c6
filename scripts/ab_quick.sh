#!/bin/bash
# Quick A/B of library variants (built with `make -C go-webp_amd/csrc VARIANT=<name> K?SRC=...`;
# "base" = the product library): one timed bench run each, kernel times printed side by side.
# Usage: WL=c3 bash scripts/ab_quick.sh base v1 v2 ...   -> gpurun_out/abq/<name>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abq
for round in 1 2; do
for v in "$@"; do
  if [ "$v" = base ]; then unset WG_LIB_VARIANT; else export WG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python3 bench.py --workload ${WL:-c3} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
    > gpurun_out/abq/$v.$round.json 2> gpurun_out/abq/$v.$round.err
  rc=$?; if [ $rc -ne 0 ]; then echo "STOP: bench $v rc=$rc"; tail -5 gpurun_out/abq/$v.$round.err; exit $rc; fi
  python3 -c "
import json,sys; j=json.load(open('gpurun_out/abq/$v.$round.json'))
st = j.get('roofline_yuv_to_rgba', {}).get('avg_launch_ms')
print('%-10s r$round' % '$v', ' '.join('%s %.3f' % (k[:12], x) for k, x in j['kernel_ms'].items()),
      ' stage %.3f' % st if st else '', ' value', j['value'])"
done
done
