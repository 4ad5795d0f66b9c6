#!/bin/bash
# Round-6 soaks on the final code: full 256-frame batches re-run many times, a sample of frames
# hashed against libwebp after every run (scripts/soak_fused.py): c3 / c3s (K1's fused tail) and
# c3ag / c3av (K7's alpha bytes, K4's wavefront and 64-byte segments).  Stops at the first failure.
# SOAKS="c3a_4k 30 c3ag_4k 30" picks others (name and runs, in pairs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06soak}
mkdir -p $OUT
set -- ${SOAKS:-c3_4k 30 c3s_4k 30 c3ag_4k 30 c3av_4k 20}
while [ $# -ge 2 ]; do
  name=$1 runs=$2
  shift 2
  timeout -k 10 300 python -u scripts/soak_fused.py $runs $name > $OUT/soak_$name.log 2>&1 || { tail $OUT/soak_$name.log; exit 1; }
  tail -1 $OUT/soak_$name.log
done
echo SOAK_DONE
