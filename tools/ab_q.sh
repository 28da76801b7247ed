# k_ellt3 with the parents-per-lane count QM a template parameter: operator parity, then
# L / L^T times at configs 2 / 4 / 5 over the L^T grid.
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_fp32.py -x -q --timeout 240 --timeout-method thread -k "ell or operators or fp32" > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -2 gpurun_out/pytest_q.log
for v in "RAOCP_ELLT3=1" "RAOCP_ELLT3_GRID=2048" "RAOCP_ELLT3_GRID=4096"; do
  echo "[$v]"
  env $v timeout -k 10 120 python3 tools/l_sweep.py 2 || exit 1
  env $v timeout -k 10 120 python3 tools/l_sweep.py 4 || exit 1
  env $v timeout -k 10 200 python3 tools/l_sweep.py 5 float32 || exit 1
done
