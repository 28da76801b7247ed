# dynamics-only engine: parity, then bench with / without it
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mega.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mega_pytest.log 2>&1 || { tail -40 gpurun_out/mega_pytest.log; exit 1; }
tail -3 gpurun_out/mega_pytest.log
for v in "RAOCP_DYN_ENGINE=0" "RAOCP_DYN_ENGINE=1" ${VARIANTS:-}; do
  env $v RAOCP_VERBOSE=1 timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --no-cpu --no-hbm --op-reps 10 > gpurun_out/bv.json 2> gpurun_out/bv.err || { echo "fail $v"; tail -5 gpurun_out/bv.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bv.json')); print('$v', round(d['value'],1), 'it/s', round(d['device_ms_per_step']*1e3,2), 'us/it')"
  grep engine gpurun_out/bv.err | head -2
done
