cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/k7_stats.py 32 > gpurun_out/k7_stats.log 2>&1; rc=$?
cat gpurun_out/k7_stats.log; exit $rc
