"""Diagnostics: per-phase timing of k_dyn_top from in-kernel stamps (100 MHz clock)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raocp-toolbox_amd"))
import numpy as np
import raocp.core as core
from raocp.problems import build_problem, recipe_config
r = recipe_config(int(sys.argv[1]) if len(sys.argv) > 1 else 2)
tree, prob = build_problem(r)
cache = core.Cache(prob)
cache.cache_initial_state(r["x0"])
cache.set_primal_flat(np.random.default_rng(0).standard_normal(cache.primal_size))
for rep in range(3):
    st = cache.native.debug_dyn_stamps(64).astype(np.int64)
nz = st[st > 0]
d = np.diff(st[:np.count_nonzero(st)]) * 10  # ns
print("stamps (ns deltas):", d.tolist(), "total us", (nz[-1] - nz[0]) / 100)
