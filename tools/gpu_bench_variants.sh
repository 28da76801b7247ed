# bench variants (no profiler): default plan, forced cuts, per-stage dynamics
export TMPDIR=/tmp
for v in "" "RAOCP_DYN_CUT=5" "RAOCP_DYN_CUT=7" "RAOCP_DYN_CUT=8" "RAOCP_DYN_PER_STAGE=1"; do
  env $v timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --no-cpu > gpurun_out/bv.json 2> gpurun_out/bv.err || { echo "fail $v"; cat gpurun_out/bv.err | tail -5; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bv.json')); print('$v', round(d['value'],1), 'it/s', round(d['device_ms_per_step']*1e3,1), 'us/it')"
done
