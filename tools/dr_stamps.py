"""Diagnostics: in-kernel stamps of the regular-tree sweep k_dr (raocp_dynr.hip). For the first
subtree of every tier the kernel stamps [start, (prologue landed: RAOCP_DR_FAULT bit 1),
(children's q rows landed), the start of every backward level, backward sweep done, (root's
x row landed), the start of every forward level, forward sweep done, written out] and the end,
printed in ns from the launch's earliest stamp (100 MHz clock), and the shader clock over the
workgroup's span (s_memtime cycles / ns).
usage: python tools/dr_stamps.py [config] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raocp-toolbox_amd"))
import numpy as np  # noqa: E402
import raocp.core as core  # noqa: E402
from raocp.problems import build_problem, recipe_config  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
r = recipe_config(cfg)
tree, prob = build_problem(r)
cache = core.Cache(prob)
print(cache.native.kernel_info(9), flush=True)
cache.cache_initial_state(r["x0"])
cache.set_primal_flat(np.random.default_rng(0).standard_normal(cache.primal_size))
for rep in range(reps):
    st = cache.native.debug_dyn_stamps(4096).astype(np.int64)
    if rep < reps - 3:
        continue
    blk = st[0:128].reshape(4, 32)
    live = blk[:, :31][blk[:, :31] != 0]
    if live.size == 0:
        continue
    t0 = live.min()
    for k in range(4):
        v = blk[k][:30][blk[k][:30] != 0]
        if v.size:
            span = (blk[k][30] - v[0]) * 10
            ghz = blk[k][31] / span if span > 0 else 0.0
            print(f"rep {rep} tier {k}: " + " ".join(f"{(x - t0) * 10:6d}" for x in v) +
                  f" | end {(blk[k][30] - t0) * 10:6d}  clock {ghz:.2f} GHz", flush=True)
