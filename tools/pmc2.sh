# PMC passes for the CP kernels (separate passes; kernel-trace only, no tracing domains)
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT" "TA_BUSY_avr TA_ADDR_STALLED_BY_TD_CYCLES_sum GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/pmc2_$i -o pmc --output-format csv -- python3 bench.py --steps 96 --warmup 24 --no-cpu --op-reps 50 > gpurun_out/pmc2_$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo pmc_done
