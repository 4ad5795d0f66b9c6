#!/bin/bash
# K1's split kernel with balanced slabs: parts (WG_K1_SPLIT) x reconstructing waves per part
# (WG_K1_RECON_WAVES, the slab size in quads) on the anim workload and small c3 batches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-k1split}; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in ${CFGS:-auto 2:9 3:6 3:8 4:5}; do
    for wb in ${WBS:-anim:64 c3:1 c3:16}; do
      wl=${wb%%:*}; bt=${wb#*:}
      env=""; [ $cfg != auto ] && env="WG_K1_SPLIT=${cfg%%:*} WG_K1_RECON_WAVES=${cfg#*:}"
      env $env timeout -k 10 300 python bench.py --workload $wl --batch $bt --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --emit separate \
        > $OUT/${wl}_${bt}_${cfg/:/x}_$rep.log 2>&1 || { tail $OUT/${wl}_${bt}_${cfg/:/x}_$rep.log; exit 1; }
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in d['kernel_ms'].items()})" \
        $OUT/${wl}_${bt}_${cfg/:/x}_$rep.log $cfg $wb
    done
  done
done
echo K1SPLIT_DONE
