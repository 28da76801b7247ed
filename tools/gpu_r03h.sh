# fp32 mixed weight tables (k_cpd / k_cpp<float>) and the dynamics launch list, then the
# round-3 profiles (tools/gpu_r03g.sh).
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32.py tests/test_gpu_dyn3.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/pytest_fp32.log 2>&1 || { tail -60 gpurun_out/pytest_fp32.log; exit 1; }
grep -E "passed|failed|drift|mixed|v1 vs" gpurun_out/pytest_fp32.log | tail -8
bash tools/gpu_r03g.sh
