# Round-3 profiles of the split sweep build: rocprofv3 statistics of the bench (eager
# launches), FETCH_SIZE / WRITE_SIZE passes, config-2 stamps, the GPU ASan driver.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/r03_prof gpurun_out/pmc2_FETCH_SIZE gpurun_out/pmc2_WRITE_SIZE
BARGS="--steps 96 --warmup 24 --no-cpu --no-shard --op-reps 200 --fp32-steps 12"
RAOCP_EAGER=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof -o prof --output-format csv -- python3 bench.py $BARGS > gpurun_out/r03_prof.log 2>&1 || { echo "rocprof stats failed"; tail -5 gpurun_out/r03_prof.log; exit 1; }
echo stats_done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmc2_$ctr -o pmc --output-format csv -- python3 bench.py $BARGS > gpurun_out/pmc2_$ctr.log 2>&1 || { echo "pmc pass $ctr failed"; tail -5 gpurun_out/pmc2_$ctr.log; exit 1; }
done
echo pmc_done
LSAN_OPTIONS=suppressions=tests/asan/lsan.supp timeout -k 10 120 ./build/asan_abi gpu > gpurun_out/asan_gpu.log 2>&1; echo "asan gpu rc=$?"; tail -2 gpurun_out/asan_gpu.log
