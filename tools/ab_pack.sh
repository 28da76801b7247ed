# k_cpd / k_cpp packed staging: parity, then CP us/it and block-0 stamps with and without
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_pack.log 2>&1 || { tail -30 gpurun_out/pytest_pack.log; exit 1; }
tail -2 gpurun_out/pytest_pack.log
for v in "" "RAOCP_CP_PACK=0" "" "RAOCP_CP_PACK=0"; do
  echo -n "c2 [$v] "
  env $v timeout -k 10 120 python3 tools/prof_cp.py 2 960 2>&1 | tail -1 || exit 1
done
for v in "" "RAOCP_CP_PACK=0"; do
  echo -n "c4 [$v] "
  env $v RAOCP_CP_V1=1 timeout -k 10 120 python3 tools/prof_cp.py 4 240 2>&1 | tail -1 || exit 1
done
for v in "" "RAOCP_CP_PACK=0"; do
  echo -n "stamps_cpp [$v] "
  env $v timeout -k 10 120 python3 tools/stamps_cpp.py 2>&1 | tail -1 || exit 1
done
