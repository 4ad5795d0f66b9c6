#!/bin/bash
# Round-5 check D: the whole GPU suite (split K1 + next-row tests), then check B (next-row bench
# lines + profiles) and check C (latency table).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05d
export TMPDIR=/tmp
echo "=== pytest ($(date +%T))"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05d/pytest_gpu.log 2>&1
rc=$?; echo "=== pytest rc=$rc"; tail -3 gpurun_out/r05d/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05d/pytest_gpu.log | head; exit $rc; }
SKIP_TESTS=1 PROF="${PROF-c3a c3rgb565 anim}" bash scripts/gpu_r05_b.sh || exit $?
bash scripts/gpu_r05_c.sh || exit $?
