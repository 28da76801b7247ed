# Round 3: k_cp3 (KC row layout, slot prefetch, split small trees) and k_dy3 (slot-parallel
# small stages) parity and timings, then the whole GPU suite.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dyn3.py tests/test_gpu_cp3.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/pytest_dyn3.log 2>&1 || { tail -60 gpurun_out/pytest_dyn3.log; exit 1; }
grep -E "passed|failed|drift" gpurun_out/pytest_dyn3.log | tail -8
timeout -k 10 900 python -u tools/cp3_time.py > gpurun_out/cp3_time.log 2>&1 || { cat gpurun_out/cp3_time.log; exit 1; }
cat gpurun_out/cp3_time.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
