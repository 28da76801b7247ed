# k_ell3 / k_ellt3 with the epilogue operands loaded before the prefetch (and eta14 / eta7 from
# the A registers, computed box offsets): operator parity, then L / L^T times over grids.
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_fp32.py -x -q --timeout 240 --timeout-method thread -k "ell or operators or fp32 or trace" > gpurun_out/pytest_order.log 2>&1 || { tail -30 gpurun_out/pytest_order.log; exit 1; }
tail -2 gpurun_out/pytest_order.log
for v in "RAOCP_ELL3=1" "RAOCP_ELL3_GRID=1024 RAOCP_ELLT3_GRID=1024" "RAOCP_ELL3_GRID=2048 RAOCP_ELLT3_GRID=2048" "RAOCP_ELL3_GRID=4096 RAOCP_ELLT3_GRID=4096"; do
  echo "[$v]"
  env $v timeout -k 10 120 python3 tools/l_sweep.py 2 || exit 1
  env $v timeout -k 10 120 python3 tools/l_sweep.py 4 || exit 1
  env $v timeout -k 10 200 python3 tools/l_sweep.py 5 float32 || exit 1
done
