# Round-3 profiles: rocprofv3 kernel statistics of the bench (eager launches: the kernel
# trace cannot see inside a replayed graph), the FETCH_SIZE / WRITE_SIZE passes (one counter
# per pass), in-kernel stamps of the tiered dynamics at configs 2 and 4, the ASan driver.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
BARGS="--steps 96 --warmup 24 --no-cpu --no-shard --op-reps 200 --fp32-steps 12"
RAOCP_EAGER=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof -o prof --output-format csv -- python3 bench.py $BARGS > gpurun_out/r03_prof.log 2>&1 || { echo "rocprof stats failed"; tail -5 gpurun_out/r03_prof.log; exit 1; }
echo stats_done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmc2_$ctr -o pmc --output-format csv -- python3 bench.py $BARGS > gpurun_out/pmc2_$ctr.log 2>&1 || { echo "pmc pass $ctr failed"; tail -5 gpurun_out/pmc2_$ctr.log; exit 1; }
done
echo pmc_done
RAOCP_DYN_VERBOSE=1 timeout -k 10 120 python3 tools/stamps.py 2 > gpurun_out/stamps_c2.log 2>&1 || { tail -5 gpurun_out/stamps_c2.log; exit 1; }
RAOCP_DYN_VERBOSE=1 timeout -k 10 180 python3 tools/stamps.py 4 > gpurun_out/stamps_c4.log 2>&1 || { tail -5 gpurun_out/stamps_c4.log; exit 1; }
cat gpurun_out/stamps_c2.log gpurun_out/stamps_c4.log
LSAN_OPTIONS=suppressions=tests/asan/lsan.supp timeout -k 10 120 ./build/asan_abi gpu > gpurun_out/asan_gpu.log 2>&1; echo "asan gpu rc=$?"; tail -2 gpurun_out/asan_gpu.log
