#!/bin/bash
# A/B of K3 variant libraries on the c5 workload: bench K3 time per variant ("base" = product).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for v in "$@"; do
  if [ "$v" = base ]; then unset WG_LIB_VARIANT; else export WG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/ab/k3_$v.json 2> gpurun_out/ab/k3_$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "STOP: $v rc=$rc"; tail -5 gpurun_out/ab/k3_$v.err; exit $rc; fi
  echo "$v $(grep -o '"kernel_ms": {[^}]*}' gpurun_out/ab/k3_$v.json)"
done
