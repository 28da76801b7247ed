# The dynamics tests (split / one / fused sweeps against the tier launches and the oracle).
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
RAOCP_TEST_DYN_ONE=1 timeout -k 10 600 python -u -m pytest -m gpu -x -q tests/test_gpu_dyn_fuse.py tests/test_gpu_dyn3.py tests/test_gpu_variants.py --timeout 120 --timeout-method thread > gpurun_out/pytest_dyn.log 2>&1 || { tail -60 gpurun_out/pytest_dyn.log; exit 1; }
tail -2 gpurun_out/pytest_dyn.log
