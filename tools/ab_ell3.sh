# k_ell3 with 16-B row loads / tile stores: parity (fp64 + fp32 L tests), L sweeps, and
# the dynamics with tables by vector loads (RAOCP_DYN_REGTAB=1)
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py -x -q --timeout 240 --timeout-method thread -k "ell or operators or fp32" > gpurun_out/pytest_ell3.log 2>&1 || { tail -30 gpurun_out/pytest_ell3.log; exit 1; }
tail -2 gpurun_out/pytest_ell3.log
timeout -k 10 120 python3 tools/l_sweep.py 2 || exit 1
timeout -k 10 120 python3 tools/l_sweep.py 4 || exit 1
timeout -k 10 200 python3 tools/l_sweep.py 5 float32 || exit 1
for v in "" "RAOCP_DYN_REGTAB=1"; do
  echo -n "c2 [$v] "
  env $v timeout -k 10 120 python3 tools/prof_cp.py 2 480 2>&1 | tail -1 || exit 1
  env $v timeout -k 10 120 python3 tools/stamps.py 2 2>&1 | tail -5 || exit 1
done
