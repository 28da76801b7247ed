# L / L^T: parity at configs 2-4 and timing sweep of the nodes-per-block setting
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 -k "ell or adjoint or operators or trace or c2" > gpurun_out/pt_ell.log 2>&1 || { tail -40 gpurun_out/pt_ell.log; exit 1; }
tail -2 gpurun_out/pt_ell.log
for thr in ${ELL_THRS:-512}; do
for per in ${ELL_PERS:-32}; do
RAOCP_ELL_THREADS=$thr RAOCP_ELL_NODES=$per timeout -k 10 300 python - <<'PY' || exit 1
import sys, os
sys.path.insert(0, 'raocp-toolbox_amd')
import raocp.core as core
from raocp.problems import build_problem, recipe_config
import bench
for cfg in (2, 3, 4):
    r = recipe_config(cfg)
    tree, prob = build_problem(r)
    c = core.Cache(prob)
    bP, bD = bench.algorithmic_bytes(c)
    ml = c.native.op_bench(0, 500); mt = c.native.op_bench(1, 500)
    print(f"thr={os.environ['RAOCP_ELL_THREADS']} per={os.environ['RAOCP_ELL_NODES']} cfg{cfg} n={c.packed.n} bytes {(bP+bD)/1e6:.2f} MB  L {ml*1e3:.2f} us {(bP+bD)/ml/1e6:.0f} GB/s   LT {mt*1e3:.2f} us {(bP+bD)/mt/1e6:.0f} GB/s")
PY
done
done
