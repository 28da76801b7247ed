# GPU round: parity tests (both dynamics paths), smoke, bench, rocprof kernel stats
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
RAOCP_DYN_PER_STAGE=1 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu_perstage.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_perstage.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- python3 bench.py --steps 2000 --warmup 50 --no-cpu > gpurun_out/prof.log 2>&1; echo prof_rc=$?
