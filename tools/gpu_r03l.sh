# Shards on the fused k_cp3 (two launches around X1), k_dy3 LDS-fit check: shard / cp3 /
# fp32 parity first, then the whole GPU suite, smoke, and the bench at K = 20 and the default.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_cp3.py tests/test_gpu_fp32.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_shard.log 2>&1 || { tail -60 gpurun_out/pytest_shard.log; exit 1; }
grep -E "passed|failed|drift|RCCL" gpurun_out/pytest_shard.log | tail -12
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_asan_abi.py::test_asan_abi_full_lifecycle > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20.json 2> gpurun_out/bench_k20.err || { tail -20 gpurun_out/bench_k20.err; exit 1; }
cut -c1-400 gpurun_out/bench_k20.json
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
