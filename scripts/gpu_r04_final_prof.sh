#!/bin/bash
# Round-4 final profiles of c3 / c3s / c5: kernel-trace stats, HBM traffic (FETCH_SIZE and
# WRITE_SIZE in their own passes) and the SQ instruction counters, each rocprofv3 pass under
# its own time limit; then profiles/pmc_traffic.json and per-workload PMC summaries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU"
T=${TAG:-r04f}
for w in ${WLS:-c3 c3s c5}; do
  TAG=${T}_$w WL=$w PMC1="FETCH_SIZE" PMC2="WRITE_SIZE" PMC3="$SQ" bash scripts/profile.sh || exit $?
  python3 scripts/pmc_summary.py gpurun_out/prof_${T}_$w > gpurun_out/prof_${T}_$w/pmc_summary.txt
done
args=""
for w in ${WLS:-c3 c3s c5}; do
  case $w in c3) n=c3_4k_deblock_x256;; c3s) n=c3s_4k_deblock_x256;; c5) n=c5_ll2048_x256;; c2) n=c2_1080p_x256;;
    c3a) n=c3a_4k_alpha_x256;; c3rgb565) n=c3_4k_rgb565_x256;; anim) n=anim_1080p_x64;; esac
  args="$args $n gpurun_out/prof_${T}_$w"
done
python3 scripts/make_pmc_traffic.py $args > gpurun_out/pmc_traffic_${T}.log 2>&1 || { tail gpurun_out/pmc_traffic_${T}.log; exit 1; }
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_${T}.json
