#!/bin/bash
# HBM/L2 traffic counters for one workload, one small counter set per rocprofv3 pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass): pmc_mem.sh <tag> <workload> [variant]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ -n "$3" ]; then export WG_LIB_VARIANT=$3; fi
TAG=$1 WL=$2 STEPS=1 \
  PMC1="FETCH_SIZE" PMC2="WRITE_SIZE" \
  PMC3="TCC_HIT TCC_MISS" PMC4="TCC_EA0_WRREQ TCC_EA0_WRREQ_64B" \
  PMC5="TCC_EA0_RDREQ TCC_EA0_RDREQ_128B" \
  bash scripts/profile.sh
python3 scripts/pmc_summary.py gpurun_out/prof_$1
