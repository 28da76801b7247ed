# Round deliverables on the GPU box: tests, smoke, bench, rocprof kernel stats, and the
# FETCH_SIZE / WRITE_SIZE passes behind roofline.traffic (one counter per pass).
export TMPDIR=/tmp
bash tools/gpu_check.sh || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmc2_$ctr -o pmc --output-format csv -- python3 bench.py --steps 96 --warmup 24 --no-cpu --op-reps 200 > gpurun_out/pmc2_$ctr.log 2>&1 || { echo "pmc pass $ctr failed"; exit 1; }
done
echo pmc_done
