# Round-2 deliverables on the GPU box: tests, smoke, bench (driver K and default), the
# rocprofv3 kernel statistics of the bench (eager launches: the kernel trace cannot see
# inside a replayed graph) and the FETCH_SIZE / WRITE_SIZE passes (one counter per pass).
export TMPDIR=/tmp
bash tools/gpu_check.sh || exit 1
RAOCP_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_prof -o prof --output-format csv -- python3 bench.py --steps 96 --warmup 24 --no-cpu --no-shard --op-reps 200 > gpurun_out/r02_prof.log 2>&1 || { echo "rocprof stats failed"; tail -5 gpurun_out/r02_prof.log; exit 1; }
echo stats_done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmc2_$ctr -o pmc --output-format csv -- python3 bench.py --steps 96 --warmup 24 --no-cpu --no-shard --op-reps 200 > gpurun_out/pmc2_$ctr.log 2>&1 || { echo "pmc pass $ctr failed"; exit 1; }
done
echo pmc_done
timeout -k 10 120 python3 tools/stamps.py 2 > gpurun_out/stamps_c2.log 2>&1 || exit 1
LSAN_OPTIONS=suppressions=tests/asan/lsan.supp timeout -k 10 120 ./build/asan_abi gpu > gpurun_out/asan_gpu.log 2>&1; echo "asan gpu rc=$?"; tail -2 gpurun_out/asan_gpu.log
