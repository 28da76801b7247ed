# PMC counters for the CP kernels at the bench config (separate passes; no tracing domains)
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"; do
  tag=$(echo $ctrs | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/pmc_$tag -o pmc --output-format csv -- python3 bench.py --steps 200 --warmup 10 --no-cpu --op-reps 200 > gpurun_out/pmc_$tag.log 2>&1 || { echo "pmc pass $tag failed"; exit 1; }
done
echo pmc_done
