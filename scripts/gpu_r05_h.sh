#!/bin/bash
# Round-5 check H: the output-stage / parity / pipeline GPU tests (K2 per mode set), the c3 bench
# line (its YUV->RGBA stage alone), and the end-to-end A/B of the committed library against the
# working tree (the pipeline's last chunks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05h}; mkdir -p $OUT
export TMPDIR=/tmp
echo "=== pytest ($(date +%T))"
timeout -k 10 500 python -u -m pytest tests/test_gpu_modes.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_next_rows.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "=== pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/bench_c3.log 2>&1 || { tail $OUT/bench_c3.log; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline_yuv_to_rgba']; print('c3', d['value'], d['kernel_ms'], 'K2 stage', r['avg_launch_ms'], r['frac'])" $OUT/bench_c3.log
TAG=${TAG:-r05h}/e2e bash scripts/e2e_prev_ab.sh
echo CHECK_H_DONE
