#!/bin/bash
# K1 stall / instruction-fetch counters on c3 for library variants: pmc_k1_fetch.sh <variant|base>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then unset WG_LIB_VARIANT; else export WG_LIB_VARIANT=$v; fi
  TAG=fetch_$v WL=c3 STEPS=2 \
    PMC1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
    PMC2="SQ_BUSY_CYCLES SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM" \
    bash scripts/profile.sh > gpurun_out/pmc_fetch_$v.log 2>&1 || { echo "STOP $v"; tail -5 gpurun_out/pmc_fetch_$v.log; exit 1; }
  echo "== $v"; python3 scripts/pmc_summary.py gpurun_out/prof_fetch_$v | grep "recon" | awk '{print $4, $7}'
done
# SQC instruction-cache counters, if this rocprofv3 knows them (own pass, hard 60 s limit)
unset WG_LIB_VARIANT
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d gpurun_out/prof_sqc -o sqc --output-format csv -- python3 bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_sqc.log 2>&1
echo "sqc rc=$?"; tail -3 gpurun_out/prof_sqc.log
python3 scripts/pmc_summary.py gpurun_out/prof_sqc | grep recon | awk '{print $4, $7}'
exit 0
