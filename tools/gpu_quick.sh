# quick GPU loop: parity tests (both dynamics paths) + stamps + bench variants (no profiler)
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
RAOCP_DYN_PER_STAGE=1 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu_ps.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_ps.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/stamps.py 2 || exit 1
for v in "" ${VARIANTS:-}; do
  env $v timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --no-cpu > gpurun_out/bv.json 2> gpurun_out/bv.err || { echo "fail $v"; tail -5 gpurun_out/bv.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bv.json')); print('$v', round(d['value'],1), 'it/s', round(d['device_ms_per_step']*1e3,1), 'us/it')"
done
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- python3 bench.py --steps 1000 --warmup 50 --no-cpu > gpurun_out/prof.log 2>&1; echo prof_rc=$?
fi
