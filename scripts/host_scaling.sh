#!/bin/bash
# The host entropy stage (the end-to-end bound) on the GPU box's own CPUs: the CPUs
# this job may use and their SMT siblings, then the batch host stage (scripts/bench_host_parse.cpp,
# the product's flags) over the c3 frames at 1, 2, 4, 8, 12 and 16 threads -- how the per-frame
# time per thread grows with the thread count, and the rate that bounds end to end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-host_scaling}; mkdir -p $OUT
{
  echo "nproc $(nproc)"
  grep -E "Cpus_allowed_list" /proc/self/status
  lscpu | grep -E "Model name|Thread\(s\) per core|Core\(s\) per socket|Socket\(s\)|L3 cache|MHz" || true
  for c in $(python3 -c "import os; print(' '.join(map(str, sorted(os.sched_getaffinity(0)))))"); do
    echo "cpu$c siblings $(cat /sys/devices/system/cpu/cpu$c/topology/thread_siblings_list 2>/dev/null) core $(cat /sys/devices/system/cpu/cpu$c/topology/core_id 2>/dev/null) pkg $(cat /sys/devices/system/cpu/cpu$c/topology/physical_package_id 2>/dev/null)"
  done
  cat /sys/fs/cgroup/cpu.max 2>/dev/null | sed 's/^/cgroup cpu.max /'
} > $OUT/topology.txt 2>&1
B=$(mktemp -d)
g++ -O2 -march=x86-64-v3 -std=c++17 -Igo-webp_amd/csrc/host -Iinclude scripts/bench_host_parse.cpp \
    go-webp_amd/csrc/host/*.cpp -lpthread -o $B/parse || exit 1
for t in 1 2 4 8 12 16; do
  n=$((t * 16)); [ $n -lt 16 ] && n=16
  echo "$(timeout 200 $B/parse -t $t -n $n -r 3 tests/golden/bench/c3_4k_s*.webp | tail -1)"
done | tee $OUT/scaling.txt
rm -rf $B
