#!/bin/bash
# Timing-only A/B of K1 variant libraries (no PMC pass): ab_k1_quick.sh <variant|base>...
# EMIT=separate times K1 without its RGBA tail.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for v in "$@"; do
  if [ "$v" = base ]; then unset WG_LIB_VARIANT; else export WG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --emit ${EMIT:-fused} > gpurun_out/ab/q_$v.json 2> gpurun_out/ab/q_$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "STOP: $v rc=$rc"; tail -5 gpurun_out/ab/q_$v.err; exit $rc; fi
  echo "$v emit=${EMIT:-fused} $(grep -o '"kernel_ms": {[^}]*}' gpurun_out/ab/q_$v.json)"
done
