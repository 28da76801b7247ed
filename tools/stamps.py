"""Diagnostics: per-phase timing of the dynamics kernels from in-kernel stamps (100 MHz
clock, workgroup 0 of every launch; launch order: backward tiers deepest first, the top,
forward tiers)."""
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
for rep in range(5):
    st = cache.native.debug_dyn_stamps(64 * 64).astype(np.int64).reshape(64, 64)
t0 = st[0, 0] if st[0, 0] else st[st[:, 0] != 0][0, 0]
for k in range(64):
    row = st[k]
    n = np.count_nonzero(row)
    if n == 0:
        continue
    d = (np.diff(row[:n]) * 10).tolist()
    print(f"launch {k}: starts at {(row[0] - t0) * 10} ns, total {(row[n - 1] - row[0]) * 10} ns, deltas {d}")
