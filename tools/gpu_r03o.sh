# Tier prologues without the level-range barrier; k_dy3 wide stages at 1,024 lanes; k_cp3's
# weight image: the whole GPU suite, stamps, timings.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python3 tools/stamps.py 2 > gpurun_out/stamps_c2.log 2>&1 || { tail -5 gpurun_out/stamps_c2.log; exit 1; }
cat gpurun_out/stamps_c2.log
timeout -k 10 900 python -u tools/cp3_time.py 2 4 5 > gpurun_out/cp3_time.log 2>&1 || { cat gpurun_out/cp3_time.log; exit 1; }
cat gpurun_out/cp3_time.log
