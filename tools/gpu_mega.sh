# persistent CP engine: parity first (each step time-limited; stop at the first failure)
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mega.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mega_pytest.log 2>&1 || { tail -40 gpurun_out/mega_pytest.log; exit 1; }
tail -3 gpurun_out/mega_pytest.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
for cut in ${CUTS:-6 7}; do
  RAOCP_MEGA_CUT=$cut timeout -k 10 120 python tools/stamps_mega.py 2 > gpurun_out/st_$cut.txt 2>&1 || { tail -5 gpurun_out/st_$cut.txt; exit 1; }
  cat gpurun_out/st_$cut.txt
  RAOCP_MEGA_CUT=$cut RAOCP_VERBOSE=1 timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --no-cpu --no-hbm --op-reps 10 > gpurun_out/bm_$cut.json 2> gpurun_out/bm_$cut.err || { tail -5 gpurun_out/bm_$cut.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bm_$cut.json')); print('cut $cut', round(d['value'],1), 'it/s', round(d['device_ms_per_step']*1e3,2), 'us/it')"
done
