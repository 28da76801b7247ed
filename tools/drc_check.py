"""Quick k_drc check (GPU): the fused CP loop against the pair k_dr + k_cp6 (RAOCP_DRC=0) and the
oracle at config 2, printing the per-entry differences; then the per-launch device times.
python tools/drc_check.py [K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import raocp.core as core  # noqa: E402
from raocp.problems import build_problem, recipe_config  # noqa: E402
from helpers import rel_err, trace_rel_err  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 30
r = recipe_config(2)
tree, prob = build_problem(r)
on = core.Cache(prob)
os.environ["RAOCP_DRC"] = "0"
off = core.Cache(prob)
del os.environ["RAOCP_DRC"]
alpha = 0.999 / on.native.step_size()
out = []
for c in (on, off):
    st, err, derr = c.native.cp_run(r["x0"], K, 0.0, alpha)
    out.append((st, err, derr, c.get_primal_flat(), c.get_dual_flat()))
a, b = out
print("status", a[0], b[0], "shapes", a[1].shape, b[1].shape)
print("trace err", trace_rel_err(a[1], b[1]), "delta", trace_rel_err(a[2], b[2]))
print("primal", rel_err(a[3], b[3]), "dual", rel_err(a[4], b[4]))
d = np.abs(a[3] - b[3])
print("worst primal entries", np.argsort(-d)[:8], d[np.argsort(-d)[:8]])
d = np.abs(a[4] - b[4])
print("worst dual entries", np.argsort(-d)[:8], d[np.argsort(-d)[:8]])
print("first rows", a[1][:3], b[1][:3])
from oracle.raocp_oracle import OracleProblem  # noqa: E402
st_o, err_o, derr_o, z_o, e_o, _ = OracleProblem(prob).chock(r["x0"], K, 0.0, alpha=alpha)
print("vs oracle: trace", trace_rel_err(a[1], err_o), "primal", rel_err(a[3], z_o), "dual", rel_err(a[4], e_o))
for op in (9, 10, 11):
    print("op", op, on.native.kernel_info(op) if op != 11 else "k_drc", f"{1e3 * on.native.op_bench(op, 400):.2f} us")
ms = on.native.cp_bench(r["x0"], 480, alpha)
print(f"loop k_drc {1e3 * ms / 480:.2f} us/it")
ms = off.native.cp_bench(r["x0"], 480, alpha)
print(f"loop pair  {1e3 * ms / 480:.2f} us/it")
