# rocprofv3 kernel statistics of the CP iteration at config 2 and config 4 (eager launches)
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in 2 4; do
  RAOCP_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$cfg -o prof --output-format csv -- python3 tools/prof_cp.py $cfg 240 > gpurun_out/prof_c$cfg.log 2>&1 || { echo "rocprof c$cfg failed"; tail -5 gpurun_out/prof_c$cfg.log; exit 1; }
  grep "config" gpurun_out/prof_c$cfg.log
done
