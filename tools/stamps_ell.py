"""Diagnostics: block 0 timeline of k_ell (RAOCP_STAMP_KERNEL=l) at a given config."""
import sys, os
os.environ["RAOCP_STAMP_KERNEL"] = "l"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raocp-toolbox_amd"))
import numpy as np
import raocp.core as core
from raocp.problems import build_problem, recipe_config
for cfg in (2, 4):
    r = recipe_config(cfg)
    tree, prob = build_problem(r)
    cache = core.Cache(prob)
    cache.native.op_bench(0, 10)
    for rep in range(5):
        st = cache.native.debug_dyn_stamps(64).astype(np.int64)
    print(f"cfg{cfg} k_ell block 0 stamps (ns from start):", [(k, int((st[k] - st[0]) * 10)) for k in range(16) if st[k]])
