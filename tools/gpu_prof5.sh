export TMPDIR=/tmp
mkdir -p gpurun_out
RAOCP_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o prof --output-format csv -- python3 tools/prof_cp.py 5 24 float32 > gpurun_out/prof_c5.log 2>&1 || { tail -5 gpurun_out/prof_c5.log; exit 1; }
grep config gpurun_out/prof_c5.log
