#!/bin/bash
# Copy a round-6 profile run (gpurun_out/prof_<tag>_<wl>) into profiles/r06/final_prof/<wl>/: the
# kernel-trace stats and trace, the steady-state summary against the same command's bench line,
# the PMC passes and their summary.
cd "$(dirname "$0")/.."
TAG=${1:-r06fp}
shift
for w in "$@"; do
  s=gpurun_out/prof_${TAG}_$w
  d=profiles/r06/final_prof/$w
  mkdir -p $d
  cp $s/trace/trace_kernel_stats.csv $d/kernel_stats.csv
  cp $s/trace/trace_kernel_trace.csv $d/kernel_trace.csv
  cp $s/steady.json $s/bench_line.json $s/pmc_summary.txt $d/
  for p in pmc1 pmc2 pmc3; do [ -f $s/$p/${p}_counter_collection.csv ] && cp $s/$p/${p}_counter_collection.csv $d/; done
done
