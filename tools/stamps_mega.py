"""Diagnostics: in-kernel timeline of the persistent CP engine (RAOCP_STAMP_KERNEL=m):
stamps of workgroup 0 (top) and workgroup 1 (a subtree) over 8 iterations, in ns from start.
Top per iteration: [UP arrived, deferred done, back done, fwd done, DOWN published, dual, primal];
subtree: [back done, UP published, DOWN arrived, fwd done, dual, primal]."""
import sys, os
os.environ["RAOCP_STAMP_KERNEL"] = "m"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raocp-toolbox_amd"))
import numpy as np
import raocp.core as core
from raocp.problems import build_problem, recipe_config
r = recipe_config(int(sys.argv[1]) if len(sys.argv) > 1 else 2)
tree, prob = build_problem(r)
cache = core.Cache(prob)
print("engine", cache.native.engine_info())
for rep in range(3):
    st = cache.native.debug_dyn_stamps(128).astype(np.int64)
t0 = min(st[0], st[64])
for w, name in ((0, "top"), (1, "subtree")):
    row = st[64 * w: 64 * w + 64]
    n = np.count_nonzero(row)
    print(name, "start", (row[0] - t0) * 10, "ns; deltas (ns):", (np.diff(row[:n]) * 10).tolist())
