# streaming L / L^T with 256-row flat tasks: operator parity, then L / L^T times at configs 2 / 4 / 5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_fp32.py -x -q --timeout 240 --timeout-method thread -k "ell or operators or fp32" > gpurun_out/pytest_flat.log 2>&1 || { tail -30 gpurun_out/pytest_flat.log; exit 1; }
tail -2 gpurun_out/pytest_flat.log
timeout -k 10 120 python3 tools/l_sweep.py 2 || exit 1
timeout -k 10 120 python3 tools/l_sweep.py 4 || exit 1
timeout -k 10 200 python3 tools/l_sweep.py 5 float32 || exit 1
