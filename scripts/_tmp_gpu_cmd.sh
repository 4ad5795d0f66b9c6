#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/k7_stats.py 32 > gpurun_out/k7_stats.log 2>&1 || { echo k7 failed; tail gpurun_out/k7_stats.log; exit 1; }
cat gpurun_out/k7_stats.log
TAILN=6 SKIP_TESTS= bash scripts/gpu_r03.sh
