# Round 3: k_cp3 with per-parent summed children (one L^T chain per family), parity and
# timings, the whole GPU suite, smoke, and the bench at the driver's K and the default.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dyn3.py tests/test_gpu_cp3.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/pytest_dyn3.log 2>&1 || { tail -60 gpurun_out/pytest_dyn3.log; exit 1; }
grep -E "passed|failed|drift" gpurun_out/pytest_dyn3.log | tail -8
timeout -k 10 900 python -u tools/cp3_time.py > gpurun_out/cp3_time.log 2>&1 || { cat gpurun_out/cp3_time.log; exit 1; }
cat gpurun_out/cp3_time.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20.json 2> gpurun_out/bench_k20.err || { tail -20 gpurun_out/bench_k20.err; exit 1; }
cut -c1-600 gpurun_out/bench_k20.json
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
