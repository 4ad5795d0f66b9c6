mkdir -p gpurun_out
[ -n "$RW_SKIP_TEST" ] || WG_K1_RECON_WAVES=13 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "sha256 or all_fixtures" > gpurun_out/pt13.log 2>&1 || { tail -20 gpurun_out/pt13.log; exit 1; }
[ -n "$RW_SKIP_TEST" ] || tail -2 gpurun_out/pt13.log
for r in ${RW_LIST:-16 15 14 13 12 10}; do
  WG_K1_RECON_WAVES=$r timeout -k 10 200 python bench.py --workload ${WL:-c3} --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/rw$r.json 2>gpurun_out/rw$r.err || { tail -5 gpurun_out/rw$r.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/rw$r.json')); print('R=$r', j['ms_per_step'], j['kernel_ms'], j['value'])"
done
