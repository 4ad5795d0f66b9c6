#!/bin/bash
# Round-4 soaks of the final code: full batches run repeatedly, 16 frames' RGBA per run hashed
# against libwebp 1.6.0 (c3 and c3s through K1's new tail, c5 through the new K7 slot table).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-soak4}; mkdir -p $OUT
export TMPDIR=/tmp
for spec in "c3_4k ${N3:-60}" "c3s_4k ${N3S:-40}" "c5_ll2048 ${N5:-100}"; do
  set -- $spec
  timeout -k 10 400 python -u scripts/soak_fused.py $2 $1 > $OUT/soak_$1.log 2>&1 || { tail -5 $OUT/soak_$1.log; exit 1; }
  echo "$1: $(tail -1 $OUT/soak_$1.log)"
done
