#!/bin/bash
# Round-4 check A: the new GPU tests (pipeline, C4 layout, K7 cross-window case), then a c3 bench
# line with the pipelined end-to-end legs (no CPU baseline), and the transfer-rate probe.
set -o pipefail
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_pipeline.py tests/test_gpu_k7.py tests/test_gpu_multi.py tests/test_gpu_c4.py \
    > $OUT/pytest.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
timeout -k 10 200 python scripts/e2e_probe.py > $OUT/e2e_probe.txt 2>&1
