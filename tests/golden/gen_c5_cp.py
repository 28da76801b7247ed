"""Oracle fixture for the config-5 CP checks of tests/test_gpu_fp32.py (c5_cp.npz).

The oracle (oracle/raocp_oracle.py, pinned to the reference by tests/test_oracle_golden.py)
runs the reference's CP loop (solver.py:97-171, tol = 0) on SURVEY.md 8(d) config 5
(recipe_config(5): 349,525 nodes, nx = 64, nu = 16) at 18 s per iteration on 8 cores — too
slow for a GPU test — so its results are stored here: the step size (ARPACK on L'L,
solver.py:104-118), the residual traces of 10 and of 20 iterations (chock with max_iters 9
and 19: the reference runs max_iters + 1), and at both points the L2 / inf norms of the
primal and dual iterates and their entries at 20,000 seeded random positions each.
usage: python tests/golden/gen_c5_cp.py [out.npz]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
from oracle.raocp_oracle import OracleProblem  # noqa: E402
from raocp.problems import build_problem, recipe_config  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "c5_cp.npz")
r = recipe_config(5)
tree, prob = build_problem(r)
orc = OracleProblem(prob)
t0 = time.time()
lam, alpha = orc.step_size()
print(f"lambda {lam:.17g} ({time.time() - t0:.0f} s)", flush=True)
rng = np.random.default_rng(0)
ip = np.sort(rng.choice(orc.P, 20000, replace=False))
idl = np.sort(rng.choice(orc.D, 20000, replace=False))
res = {"alpha": np.float64(alpha), "lam": np.float64(lam), "x0": np.asarray(r["x0"], float), "ip": ip, "id": idl}
p = d = None
errs, derrs = [], []
for K in (10, 20):
    t0 = time.time()
    st, err, derr, p, d, _ = orc.chock(r["x0"], 9, 0.0, alpha=alpha, p0=p, d0=d)
    errs.append(err)
    derrs.append(derr)
    pre = f"k{K}/"
    res[pre + "err"] = np.concatenate(errs)
    res[pre + "derr"] = np.concatenate(derrs)
    res[pre + "z_sample"], res[pre + "eta_sample"] = p[ip], d[idl]
    res[pre + "z_norms"] = np.array([np.linalg.norm(p), np.max(np.abs(p))])
    res[pre + "eta_norms"] = np.array([np.linalg.norm(d), np.max(np.abs(d))])
    print(f"{K} iterations ({time.time() - t0:.0f} s): last residuals {err[-1]}", flush=True)
np.savez_compressed(out, **res)
print("wrote", out)
