#!/bin/bash
# Same-box A/B of the host entropy stage's code generation: the batch host stage
# (scripts/bench_host_parse.cpp over the c3 frames) built -O2 (the product's flags) and
# -O2 -march=x86-64-v3 (BMI2 flag-free shifts, LZCNT), on 1 and 16 threads, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-host_ab}; mkdir -p $OUT
B=$(mktemp -d)
SRC="scripts/bench_host_parse.cpp go-webp_amd/csrc/host/*.cpp"
g++ -O2 -std=c++17 -Igo-webp_amd/csrc/host -Iinclude $SRC -lpthread -o $B/base || exit 1
g++ -O2 -march=x86-64-v3 -std=c++17 -Igo-webp_amd/csrc/host -Iinclude $SRC -lpthread -o $B/v3 || exit 1
for rep in 1 2 3; do
  for v in base v3; do
    echo "$v rep $rep: $(timeout 120 $B/$v -t 1 -n 16 -r 3 tests/golden/bench/c3_4k_s*.webp)"
    echo "$v rep $rep: $(timeout 120 $B/$v -t 16 -n 256 -r 3 tests/golden/bench/c3_4k_s*.webp)"
  done
done | tee $OUT/host_parse_ab.txt
rm -rf $B
