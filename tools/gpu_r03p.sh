# After reverting the 1,024-lane wide stages: timings, plan experiments at config 2, the whole
# GPU suite, smoke and the bench at K = 20 and the default.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/dyn_time.py 2 default RAOCP_DYN_CUT=8 RAOCP_DYN_CUT=7 > gpurun_out/dyn_time.log 2>&1 || { cat gpurun_out/dyn_time.log; exit 1; }
timeout -k 10 600 python -u tools/dyn_time.py 5 default >> gpurun_out/dyn_time.log 2>&1 || { cat gpurun_out/dyn_time.log; exit 1; }
cat gpurun_out/dyn_time.log
timeout -k 10 900 python -u tools/cp3_time.py 2 4 5 > gpurun_out/cp3_time.log 2>&1 || { cat gpurun_out/cp3_time.log; exit 1; }
cat gpurun_out/cp3_time.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_k20.json 2> gpurun_out/bench_k20.err || { tail -20 gpurun_out/bench_k20.err; exit 1; }
cut -c1-300 gpurun_out/bench_k20.json
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
