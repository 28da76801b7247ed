# compact staging (StgTable) in all CP / L kernels: parity (fp64 + fp32), then timings
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_pack.log 2>&1 || { tail -30 gpurun_out/pytest_pack.log; exit 1; }
tail -2 gpurun_out/pytest_pack.log
for cfg in 2 3 4; do
  for v in "" "RAOCP_CP_PACK=0"; do
    echo -n "c$cfg [$v] "
    env $v timeout -k 10 120 python3 tools/prof_cp.py $cfg 240 2>&1 | tail -1 || exit 1
  done
done
for v in "" "RAOCP_CP_PACK=0"; do
  echo -n "c5 fp32 [$v] "
  env $v timeout -k 10 200 python3 tools/prof_cp.py 5 48 2>&1 | tail -1 || exit 1
done
for v in "RAOCP_CP_FB=4" "RAOCP_CP_FB=2" "RAOCP_CP_FB=4 RAOCP_CP_LB=8" "RAOCP_CP_LB=8" "RAOCP_CP_FB=16"; do
  echo -n "c2 [$v] "
  env $v timeout -k 10 120 python3 tools/prof_cp.py 2 480 2>&1 | tail -1 || exit 1
done
