"""Diagnostics (diagnostic build of the dynamics unit, RAOCP_HIP_LIB=build/var/diag.so): the
per-level stamps of the first subtree of every tier (raocp_dynr.hip stamp / stamp_flush) for
the sweep alone (k_dr, the projection op) and inside the fused launch (k_drc), side by side,
in ns from each launch's earliest stamp: [start, prologue / children's q landed, every backward
level, backward done, root's x landed, every forward level, forward done, ...] and the end.
usage: python tools/dr_levels.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raocp-toolbox_amd"))
import numpy as np  # noqa: E402
import raocp.core as core  # noqa: E402
from raocp.problems import build_problem, recipe_config  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
r = recipe_config(2)
cache = core.Cache(build_problem(r)[1])
cache.cache_initial_state(r["x0"])
cache.set_primal_flat(np.random.default_rng(0).standard_normal(cache.primal_size))
for which in ("", "f"):
    os.environ["RAOCP_STAMP_KERNEL"] = which
    name = "k_drc" if which else "k_dr "
    for rep in range(reps):
        st = cache.native.debug_dyn_stamps(4096).astype(np.int64)
        if rep < reps - 2:
            continue
        blk = st[0:128].reshape(4, 32)
        live = blk[:, :30][blk[:, :30] != 0]
        t0 = live.min()
        for k in range(3):
            v = blk[k][:30][blk[k][:30] != 0]
            print(f"{name} rep {rep} tier {k}: " + " ".join(f"{(x - t0) * 10:6d}" for x in v) +
                  f" | end {(blk[k][30] - t0) * 10:6d}", flush=True)
