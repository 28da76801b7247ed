# GPU round: parity tests (both dynamics paths), smoke, bench, rocprof kernel stats.
# Every GPU step has its own time limit; the first failure ends the script.
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
RAOCP_DYN_PER_STAGE=1 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu_perstage.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_perstage.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_perstage.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
# kernel statistics: eager launches (rocprofv3 --kernel-trace crashes replaying the CP graph);
# the per-kernel durations are the graph's, the gaps between them are not
RAOCP_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- python3 bench.py --steps 2000 --warmup 48 --no-cpu > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/prof.log; exit 1; }
tail -1 gpurun_out/prof.log
