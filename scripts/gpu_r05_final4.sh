#!/bin/bash
# Round-5 final check 4 (after K7 on the side stream, alpha-first batches and K4's DPP scans): the
# whole GPU suite + smoke and every workload's bench line (scripts/gpu_r05_final.sh); then, with
# PART2=1, the c3a / c5 / c3 soaks and the c3a / anim profiles (trace + PMC passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05final4}
if [ -z "$PART2" ]; then
  TAG=${TAG:-r05final4} bash scripts/gpu_r05_final.sh || exit $?
  echo FINAL4_DONE
  exit 0
fi
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/soak_fused.py 30 c3a_4k > $OUT/soak_c3a.log 2>&1 || { tail $OUT/soak_c3a.log; exit 1; }
tail -1 $OUT/soak_c3a.log
timeout -k 10 300 python -u scripts/soak_fused.py 40 c5_ll2048 > $OUT/soak_c5.log 2>&1 || { tail $OUT/soak_c5.log; exit 1; }
tail -1 $OUT/soak_c5.log
timeout -k 10 300 python -u scripts/soak_fused.py 30 c3_4k > $OUT/soak_c3.log 2>&1 || { tail $OUT/soak_c3.log; exit 1; }
tail -1 $OUT/soak_c3.log
TAG=r05fp6 WLS="c3a anim" bash scripts/gpu_r04_final_prof.sh || exit $?
echo FINAL4B_DONE
