# The split sweep in one launch (k_dyn_one): timing against the two-launch split sweep and the
# tier launches, stamps, the dynamics tests, the whole GPU suite, smoke, CP timings, bench.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
RAOCP_DYN_VERBOSE=1 timeout -k 10 300 python -u tools/dyn_time.py 2 default RAOCP_DYN_ONE=0 RAOCP_DYN_SPLIT=0 > gpurun_out/dyn_time.log 2>&1 || { cat gpurun_out/dyn_time.log; exit 1; }
cat gpurun_out/dyn_time.log
timeout -k 10 120 python3 tools/stamps.py 2 > gpurun_out/stamps_c2.log 2>&1 || { tail -5 gpurun_out/stamps_c2.log; exit 1; }
cat gpurun_out/stamps_c2.log
timeout -k 10 600 python -u -m pytest -m gpu -x -q tests/test_gpu_dyn_fuse.py tests/test_gpu_dyn3.py tests/test_gpu_variants.py --timeout 120 --timeout-method thread > gpurun_out/pytest_dyn.log 2>&1 || { tail -60 gpurun_out/pytest_dyn.log; exit 1; }
tail -2 gpurun_out/pytest_dyn.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u tools/cp3_time.py 2 > gpurun_out/cp3_time.log 2>&1 || { cat gpurun_out/cp3_time.log; exit 1; }
cat gpurun_out/cp3_time.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20.json 2> gpurun_out/bench_k20.err || { tail -20 gpurun_out/bench_k20.err; exit 1; }
cut -c1-300 gpurun_out/bench_k20.json
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
