#!/bin/bash
# Same-call A/B of whole library variants (built beforehand into go-webp_amd/webp_amd/
# libgowebp_amd_<name>.so, e.g. from an older revision):  VARIANTS="old" bash scripts/ab_lib.sh
# Alternates the product library and each variant on c3 and c2 (kernels only, then one run
# with the end-to-end leg), ROUNDS times.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUNDS=${ROUNDS:-2}
WLS=${WLS:-"c3 c2"}
for r in $(seq 1 "$ROUNDS"); do
  for wl in $WLS; do
    for v in "" $VARIANTS; do
      name="ab_${wl}_${v:-new}_$r"
      extra="--no-e2e"
      [ "$r" = "$ROUNDS" ] && [ "$wl" = "c3" ] && extra=""
      WG_LIB_VARIANT=$v timeout -k 10 300 python bench.py --workload "$wl" --steps 10 --warmup 3 --no-cpu-baseline \
        $extra > "gpurun_out/$name.log" 2>&1
      rc=$?
      line=$(grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); \
k=d['kernel_ms']; e=d.get('end_to_end',{}); print(d['value'], k, e.get('value',''), e.get('seconds_first_call',''))" 2>/dev/null)
      echo "$name rc=$rc $line"
      [ $rc -eq 0 ] || { tail -5 "gpurun_out/$name.log"; exit $rc; }
    done
  done
done
