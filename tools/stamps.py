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
for rep in range(5):
    st = cache.native.debug_dyn_stamps(64).astype(np.int64)
k = np.count_nonzero(st)
s = (k - 4) // 3
main = st[:2 + 3 * s]
d = np.diff(main) * 10  # ns
pro = (st[2 + 3 * s:4 + 3 * s] - st[0]) * 10
print(f"top kernel (cut s={s}): prologue {d[0]} ns (segments built at {pro[0]}, gather done at {pro[1]})")
print("  backward (phase A, phase B) per stage s-1..0:", [(int(d[1 + 2 * i]), int(d[2 + 2 * i])) for i in range(s)])
print("  forward per stage 0..s-1:", [int(v) for v in d[1 + 2 * s:]])
print("  total us", (main[-1] - main[0]) / 100)
