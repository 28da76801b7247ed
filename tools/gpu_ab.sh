# A/B variants of the bench (parity first): VARIANTS="A=1 B=0,C=2"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -1 gpurun_out/parity.log
for v in ${VARIANTS}; do
  env ${v//,/ } timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-cpu --op-reps 500 > gpurun_out/b.json 2> gpurun_out/b.err || { echo "fail $v"; tail -5 gpurun_out/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b.json')); r=d['roofline']; h=d['l_sweep_hbm']; print('$v it/s', round(d['value'],1), '| c2 L', round(r['us_per_launch'],2), 'us', round(r['frac'],3), '| c2 LT', round(d['l_transpose']['us_per_launch'],2), '| c4 L', round(h['L']['us_per_launch'],2), round(h['L']['frac'],3), '| c4 LT', round(h['L_transpose']['us_per_launch'],2), round(h['L_transpose']['frac'],3))"
done
