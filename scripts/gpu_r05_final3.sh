#!/bin/bash
# Round-5 final check 3 (after the last K7 changes): the whole GPU suite + smoke, every workload's
# bench line, the c3a / c5 soaks, and the c3a / c5 profiles (trace + PMC passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05final3} bash scripts/gpu_r05_final.sh || exit $?
OUT=gpurun_out/${TAG:-r05final3}
timeout -k 10 300 python -u scripts/soak_fused.py 30 c3a_4k > $OUT/soak_c3a.log 2>&1 || { tail $OUT/soak_c3a.log; exit 1; }
tail -1 $OUT/soak_c3a.log
timeout -k 10 300 python -u scripts/soak_fused.py 60 c5_ll2048 > $OUT/soak_c5.log 2>&1 || { tail $OUT/soak_c5.log; exit 1; }
tail -1 $OUT/soak_c5.log
echo FINAL3_DONE
