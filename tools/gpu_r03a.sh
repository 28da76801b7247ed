# Round 3, first box: MFMA rates (f64 / f32 16x16x4), rocprofv3 kernel statistics of the
# config-4 (fp64) and config-5 (fp32) CP loops (eager launches).
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench7 > gpurun_out/ubench7.log 2>&1 || { cat gpurun_out/ubench7.log; exit 1; }
cat gpurun_out/ubench7.log
RAOCP_EAGER=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_c4 -o prof --output-format csv -- python3 tools/prof_cp.py 4 48 > gpurun_out/r03_c4.log 2>&1 || { tail -5 gpurun_out/r03_c4.log; exit 1; }
tail -1 gpurun_out/r03_c4.log
RAOCP_EAGER=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_c5 -o prof --output-format csv -- python3 tools/prof_cp.py 5 12 > gpurun_out/r03_c5.log 2>&1 || { tail -5 gpurun_out/r03_c5.log; exit 1; }
tail -1 gpurun_out/r03_c5.log
