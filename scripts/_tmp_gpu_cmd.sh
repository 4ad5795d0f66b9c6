cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python scripts/k7_stats.py 32 > gpurun_out/k7_stats.log 2>&1; rc=$?; tail -9 gpurun_out/k7_stats.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old nodc" ROUNDS=2 WLS="c3" bash scripts/ab_lib.sh
