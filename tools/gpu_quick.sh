# quick GPU pass: parity tests (optionally a -k filter in $K), then CP timings at configs 2 and 4
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_quick.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_quick.log | tail -30; tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
for cfg in 2 4 3; do
  timeout -k 10 120 python3 tools/prof_cp.py $cfg 480 || exit 1
  RAOCP_CP_V1=1 timeout -k 10 120 python3 tools/prof_cp.py $cfg 480 || exit 1
done
