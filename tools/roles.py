"""Time each CP kernel (and each block role of it) alone with HIP events (op_bench)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raocp-toolbox_amd"))
import raocp.core as core
from raocp.problems import build_problem, recipe_config
r = recipe_config(int(sys.argv[1]) if len(sys.argv) > 1 else 2)
tree, prob = build_problem(r)
cache = core.Cache(prob)
names = ["ell", "ell_t", "cp_dual", "cp_dual child", "cp_dual nonleaf", "cp_dual leaf", "cp_primal",
         "cp_primal nonleaf", "cp_primal leaf", "dynamics (all launches)", "cp_check"]
for op, nm in enumerate(names):
    ms = cache.native.op_bench(op, 500)
    print(f"{nm:26s} {ms * 1e3:8.2f} us")
