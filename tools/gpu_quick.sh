# quick GPU loop: parity tests + stamps + bench + kernel stats
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/stamps.py 2 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- python3 bench.py --steps 2000 --warmup 50 --no-cpu > gpurun_out/prof.log 2>&1; echo prof_rc=$?
grep -o '"value": [0-9.]*' gpurun_out/prof.log
