"""k_cp4 against k_cp3 on config 2 (and variants): largest differences of the CP outputs.
python tools/cp4_diff.py [iters]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "raocp-toolbox_amd"))
import raocp.core as core  # noqa: E402
from raocp.problems import build_problem, recipe_config  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
for case in ("boxed", "nobox", "leafbox"):
    r = recipe_config(2)
    if case != "boxed":
        r["nl_min"] = r["nl_max"] = None
        if case == "nobox":
            r["l_min"] = r["l_max"] = None
    tree, prob = build_problem(r)
    c4 = core.Cache(prob)
    os.environ["RAOCP_CP4"] = "0"
    c3 = core.Cache(prob)
    del os.environ["RAOCP_CP4"]
    print(case, c4.native.kernel_info(10), "|", c3.native.kernel_info(10))
    alpha = 0.999 / c4.native.step_size()
    for k in (1, 2, iters):
        outs = []
        for c in (c4, c3):
            st, err, derr = c.native.cp_run(r["x0"], k, 0.0, alpha)
            outs.append((err, derr, c.get_primal_flat(), c.get_dual_flat()))
        d = [float(np.max(np.abs(u - v))) for u, v in zip(*outs)]
        z4, z3 = outs[0][2], outs[1][2]
        y4, y3 = outs[0][3], outs[1][3]
        iz = int(np.argmax(np.abs(z4 - z3)))
        iy = int(np.argmax(np.abs(y4 - y3)))
        print(f"  iters {k}: err {d[0]:.3e} derr {d[1]:.3e} primal {d[2]:.3e} @ {iz} dual {d[3]:.3e} @ {iy}"
              f"  n_primal_diff {int(np.sum(z4 != z3))} n_dual_diff {int(np.sum(y4 != y3))}")
