#!/bin/bash
# Same-box A/B of the host entropy stage's code generation (scripts/bench_host_parse.cpp over the
# c3 frames, 1 and 16 threads, alternating): -O2 -march=x86-64-v3 (the product), -O3, and -O2 with
# profile feedback (-fprofile-use) trained on c3 + c3s + c5 frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-host_ab2}; mkdir -p $OUT
B=$(mktemp -d)
SRC="scripts/bench_host_parse.cpp go-webp_amd/csrc/host/*.cpp"
F="-std=c++17 -march=x86-64-v3 -Igo-webp_amd/csrc/host -Iinclude"
G=tests/golden/bench
g++ -O2 $F $SRC -lpthread -o $B/base || exit 1
g++ -O3 $F $SRC -lpthread -o $B/o3 || exit 1
g++ -O2 $F -fprofile-generate -fprofile-dir=$B/prof $SRC -lpthread -o $B/gen || exit 1
$B/gen -t 1 -n 8 -r 1 $G/c3_4k_s*.webp > /dev/null && $B/gen -t 1 -n 8 -r 1 $G/c3s_4k_s*.webp > /dev/null && \
  $B/gen -t 1 -n 2 -r 1 $G/c5_ll2048_s0.webp $G/c5_ll2048_s1.webp > /dev/null || exit 1
g++ -O2 $F -fprofile-use -fprofile-dir=$B/prof -Wno-missing-profile $SRC -lpthread -o $B/pgo || exit 1
for rep in 1 2 3; do
  for v in base o3 pgo; do
    echo "$v rep $rep: $(timeout 120 $B/$v -t 1 -n 16 -r 3 $G/c3_4k_s*.webp)"
    echo "$v rep $rep: $(timeout 120 $B/$v -t 16 -n 256 -r 3 $G/c3_4k_s*.webp)"
    echo "$v rep $rep c3s: $(timeout 120 $B/$v -t 1 -n 8 -r 2 $G/c3s_4k_s*.webp)"
  done
done | tee $OUT/host_parse_ab2.txt
rm -rf $B
