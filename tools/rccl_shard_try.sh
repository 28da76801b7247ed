# Try the RCCL shard transport with 2 ranks sharing the box's one GPU (RCCL may refuse
# duplicate devices; the multi-GPU run is the driver's).
export TMPDIR=/tmp
NCCL_DEBUG=INFO RAOCP_DEVICE=0 RAOCP_VERBOSE=1 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --mode shard --steps 240 --warmup 24 --no-cpu --op-reps 50 \
  > gpurun_out/rccl_try.log 2>&1; echo "rc=$?"
grep -v "^\s*$" gpurun_out/rccl_try.log | tail -25
