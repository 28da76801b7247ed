# k_ellt3 (streaming L^T) parity and launch times against k_ell_t, fp64 configs 2 / 4 and fp32
# config 5, with a grid sweep (RAOCP_ELLT3_GRID blocks of 256 lanes).
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_fp32.py -x -q --timeout 240 --timeout-method thread -k "ell or operators or fp32" > gpurun_out/pytest_ellt3.log 2>&1 || { tail -30 gpurun_out/pytest_ellt3.log; exit 1; }
tail -2 gpurun_out/pytest_ellt3.log
for v in "RAOCP_ELLT3=0" "RAOCP_ELLT3=1" "RAOCP_ELLT3_GRID=1024" "RAOCP_ELLT3_GRID=2048" "RAOCP_ELLT3_GRID=8192"; do
  echo "[$v]"
  env $v timeout -k 10 120 python3 tools/l_sweep.py 2 || exit 1
  env $v timeout -k 10 120 python3 tools/l_sweep.py 4 || exit 1
  env $v timeout -k 10 200 python3 tools/l_sweep.py 5 float32 || exit 1
done
