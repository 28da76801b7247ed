# Fused tiered dynamics sweep: stamps, the fused tests, timing.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/stamps.py 2 > gpurun_out/stamps_c2.log 2>&1 || { tail -5 gpurun_out/stamps_c2.log; exit 1; }
cat gpurun_out/stamps_c2.log
RAOCP_DYN_FUSE=0 timeout -k 10 120 python3 tools/stamps.py 2 > gpurun_out/stamps_c2_tiers.log 2>&1 || { tail -5 gpurun_out/stamps_c2_tiers.log; exit 1; }
cat gpurun_out/stamps_c2_tiers.log
timeout -k 10 600 python -u -m pytest -m gpu -x -q tests/test_gpu_dyn_fuse.py tests/test_gpu_dyn3.py tests/test_gpu_variants.py --timeout 120 --timeout-method thread > gpurun_out/pytest_dyn.log 2>&1 || { tail -60 gpurun_out/pytest_dyn.log; exit 1; }
tail -2 gpurun_out/pytest_dyn.log
