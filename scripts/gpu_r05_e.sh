#!/bin/bash
# Round-5 check E: the whole GPU suite (K7 run collapse, per-row-unit K6), bench lines of c3
# (end to end included), c5, c3a and c3rgb565 with their profiles, the end-to-end thread / split
# A/B and the latency table.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05e
export TMPDIR=/tmp
echo "=== pytest ($(date +%T))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05e/pytest_gpu.log 2>&1
rc=$?; echo "=== pytest rc=$rc"; tail -3 gpurun_out/r05e/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05e/pytest_gpu.log | head; exit $rc; }
TAG=r05e SKIP_TESTS=1 BENCH_WLS="${BENCH_WLS-c3 c5 c3a c3rgb565}" PROF="${PROF-c5 c3a c3rgb565}" bash scripts/gpu_r05_b.sh || exit $?
[ -n "$NO_AB" ] || TAG=r05e/e2e_ab bash scripts/e2e_threads_ab.sh || exit $?
TAG=r05e bash scripts/gpu_r05_c.sh || exit $?
echo CHECK_E_DONE
