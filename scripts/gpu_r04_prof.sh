#!/bin/bash
# Round-4 profiles: c3s trace + HBM traffic + SQ instruction counters; c3 and c5 trace + SQ
# counters (VALU utilisation, VALU issue).  Each rocprofv3 pass under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU"
TAG=${TAG:-r04}_c3s WL=c3s PMC1="FETCH_SIZE" PMC2="WRITE_SIZE" PMC3="$SQ" bash scripts/profile.sh || exit $?
TAG=${TAG:-r04}_c3 WL=c3 PMC1="$SQ" bash scripts/profile.sh || exit $?
TAG=${TAG:-r04}_c5 WL=c5 PMC1="$SQ" bash scripts/profile.sh || exit $?
for w in c3s c3 c5; do python3 scripts/pmc_summary.py gpurun_out/prof_${TAG:-r04}_$w > gpurun_out/prof_${TAG:-r04}_$w/pmc_summary.txt; done
