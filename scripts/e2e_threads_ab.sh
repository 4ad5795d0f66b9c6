#!/bin/bash
# Same-box A/B of the end-to-end decode (c3, automatic chunking): entropy-stage threads 16 / 15 /
# 14 (the job's CPU quota is 16; the device thread and the runtime's own threads share it), and
# the pipeline's chunks on the split K1 (default) vs the one-workgroup K1 (WG_K1_SPLIT=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-e2e_ab}; mkdir -p $OUT
for cfg in "16 -1" "15 -1" "14 -1" "16 0"; do
  set -- $cfg
  if [ "$2" = "-1" ]; then unset WG_K1_SPLIT; else export WG_K1_SPLIT=$2; fi
  OMP_NUM_THREADS=$1 timeout -k 10 300 python -u scripts/e2e_ab.py ${WL:-c3} 0 > $OUT/t$1_s$2.log 2>&1 || { tail -5 $OUT/t$1_s$2.log; exit 1; }
  echo "threads $1 split ${2/-1/auto}:"; grep round $OUT/t$1_s$2.log
done
