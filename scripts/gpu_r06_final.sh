#!/bin/bash
# Round-6 final check (stops at the first failure):
#   PART=A  the whole GPU suite + smoke, then every workload's bench line (c3 with the driver's own
#           flags: end-to-end and CPU legs; the others --steps 10 --warmup 3)
#   PART=B  rocprofv3 per workload ($WLS): kernel trace + stats with warm-up (--steps 12 --warmup 3:
#           the committed average is the steady state, scripts/trace_steady.py), then FETCH_SIZE,
#           WRITE_SIZE and the SQ counters in passes of their own, and profiles/pmc_traffic.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06final}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
wlname() {
  case $1 in c3) echo c3_4k_deblock_x256;; c3s) echo c3s_4k_deblock_x256;; c5) echo c5_ll2048_x256;;
    c2) echo c2_1080p_x256;; c3a) echo c3a_4k_alpha_x256;; c3ag) echo c3ag_4k_alpha_gradient_x256;;
    c3av) echo c3av_4k_alpha_vertical_x256;; c3rgb565) echo c3_4k_rgb565_x256;; anim) echo anim_1080p_x64;; esac
}
if [ "${PART:-A}" = A ]; then
  if [ -z "$SKIP_TESTS" ]; then
    step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  fi
  for w in ${BENCH_WLS:-c3 c3s c5 c2 c3a c3ag c3av c3rgb565 anim}; do
    if [ $w = c3 ]; then
      step bench_c3 600 python bench.py --gpus 1 --steps 20 --warmup 5
    else
      step bench_$w 400 python bench.py --workload $w --steps 10 --warmup 3
    fi
    grep -h '^{' $OUT/bench_$w.log > $OUT/bench_$w.json
  done
  echo FINAL_A_DONE
  exit 0
fi
SQ="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU"
args=""
for w in ${WLS:-c3 c3s c5}; do
  P=gpurun_out/prof_${TAG:-r06final}_$w
  TAG=${TAG:-r06final}_$w WL=$w STEPS=12 WARMUP=3 bash scripts/profile.sh > $OUT/prof_$w.log 2>&1 || { tail $OUT/prof_$w.log; exit 1; }
  grep -h '^{' $P/trace.log > $P/bench_line.json
  python3 scripts/trace_steady.py $P 3 $P/bench_line.json > $P/steady.json && cat $P/steady.json | head -30
  TAG=${TAG:-r06final}_$w WL=$w STEPS=3 WARMUP=1 PMC_ONLY=1 PMC1="FETCH_SIZE" PMC2="WRITE_SIZE" PMC3="$SQ" \
    bash scripts/profile.sh > $OUT/pmc_$w.log 2>&1 || { tail $OUT/pmc_$w.log; exit 1; }
  python3 scripts/pmc_summary.py $P > $P/pmc_summary.txt
  args="$args $(wlname $w) $P"
done
python3 scripts/make_pmc_traffic.py $args > $OUT/pmc_traffic.log 2>&1 || { tail $OUT/pmc_traffic.log; exit 1; }
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
echo FINAL_B_DONE
