#!/bin/bash
# PMC comparison of K3 library variants on c5: pmc_ab.sh <variant|base>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  if [ "$v" = base ]; then unset WG_LIB_VARIANT; else export WG_LIB_VARIANT=$v; fi
  TAG=ab_$v WL=c5 STEPS=2 \
    PMC1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES" \
    PMC2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_BUSY_CYCLES" \
    PMC3="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR" \
    PMC4="TCP_PENDING_STALL_CYCLES SQ_VMEM_TA_CMD_FIFO_FULL" \
    bash scripts/profile.sh > gpurun_out/pmc_ab_$v.log 2>&1 || { echo "STOP $v"; tail -5 gpurun_out/pmc_ab_$v.log; exit 1; }
  echo "== $v"; python3 scripts/pmc_summary.py gpurun_out/prof_ab_$v | grep "vp8l" | awk '{print $4, $7}'
done
