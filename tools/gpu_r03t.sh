# Split tiered sweep (k_dyn_up / k_dyn_down): timing, stamps, the dynamics tests, CP loop, bench.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
RAOCP_DYN_VERBOSE=1 timeout -k 10 300 python -u tools/dyn_time.py 2 default RAOCP_DYN_FOLD=1 RAOCP_DYN_SPLIT=0 RAOCP_DYN_FUSE=1 > gpurun_out/dyn_time.log 2>&1 || { cat gpurun_out/dyn_time.log; exit 1; }
cat gpurun_out/dyn_time.log
timeout -k 10 120 python3 tools/stamps.py 2 > gpurun_out/stamps_c2.log 2>&1 || { tail -5 gpurun_out/stamps_c2.log; exit 1; }
cat gpurun_out/stamps_c2.log
timeout -k 10 600 python -u -m pytest -m gpu -x -q tests/test_gpu_dyn_fuse.py tests/test_gpu_dyn3.py tests/test_gpu_variants.py --timeout 120 --timeout-method thread > gpurun_out/pytest_dyn.log 2>&1 || { tail -60 gpurun_out/pytest_dyn.log; exit 1; }
tail -2 gpurun_out/pytest_dyn.log
timeout -k 10 600 python -u tools/cp3_time.py 2 > gpurun_out/cp3_time.log 2>&1 || { cat gpurun_out/cp3_time.log; exit 1; }
cat gpurun_out/cp3_time.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20.json 2> gpurun_out/bench_k20.err || { tail -20 gpurun_out/bench_k20.err; exit 1; }
cut -c1-300 gpurun_out/bench_k20.json
