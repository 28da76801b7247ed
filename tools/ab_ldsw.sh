# k_ell3 / k_ellt3 with the weight fragments in LDS (RAOCP_ELL3_LDSW=1) against registers:
# operator parity with LDS weights, then L / L^T launch times at configs 2 / 4 / 5 over grids.
export TMPDIR=/tmp
RAOCP_ELL3_LDSW=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_fp32.py -x -q --timeout 240 --timeout-method thread -k "ell or operators or fp32" > gpurun_out/pytest_ldsw.log 2>&1 || { tail -30 gpurun_out/pytest_ldsw.log; exit 1; }
tail -2 gpurun_out/pytest_ldsw.log
for v in "RAOCP_ELL3_LDSW=0" "RAOCP_ELL3_LDSW=1" "RAOCP_ELL3_LDSW=1 RAOCP_ELL3_GRID=1024 RAOCP_ELLT3_GRID=1024" "RAOCP_ELL3_LDSW=1 RAOCP_ELL3_GRID=2048 RAOCP_ELLT3_GRID=2048" "RAOCP_ELL3_LDSW=1 RAOCP_ELL3_GRID=8192 RAOCP_ELLT3_GRID=8192"; do
  echo "[$v]"
  env $v timeout -k 10 120 python3 tools/l_sweep.py 2 || exit 1
  env $v timeout -k 10 120 python3 tools/l_sweep.py 4 || exit 1
  env $v timeout -k 10 200 python3 tools/l_sweep.py 5 float32 || exit 1
done
