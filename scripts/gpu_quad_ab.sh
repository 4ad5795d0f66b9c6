cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
WG_LIB_VARIANT=quad timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/quad_pytest.log 2>&1
rc=$?; echo "pytest quad rc=$rc"; tail -15 gpurun_out/quad_pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_k1.sh base quad
