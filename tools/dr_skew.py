"""Diagnostics (diagnostic builds): the spread of k_dr's workgroups. Every workgroup stamps its
start, the end of its backward sweep and its end (raocp_dynr.hip wg_stamp); printed per tier as
min / median / max in ns from the launch's earliest stamp, and the backward-done times of the
children of the first subtree of each tier above the deepest.
usage: python tools/dr_skew.py [config] [reps]"""
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
# the default plan of config 2: tiers [8,12) x256 (blocks 0..255), [4,8) x16, [0,4) x1
tiers = [("deep", 0, 256), ("mid", 256, 16), ("top", 272, 1)]
for rep in range(reps):
    st = cache.native.debug_dyn_stamps(4096).astype(np.int64)
    if rep < reps - 3:
        continue
    w = st[1024:1024 + 4 * 273].reshape(273, 4)[:, :3]
    t0 = w[w > 0].min()
    w = (w - t0) * 10
    for name, b0, n in tiers:
        blk = w[b0:b0 + n]
        d = ", ".join(f"{q} {np.min(blk[:, i]):6d} / {int(np.median(blk[:, i])):6d} / {np.max(blk[:, i]):6d}"
                      for i, q in enumerate(("start", "bwd", "end")))
        print(f"rep {rep} {name:4s}: {d}", flush=True)
    print(f"rep {rep} bwd done of deep 0..15: " + " ".join(f"{x:5d}" for x in w[0:16, 1]), flush=True)
    # by XCD (block b on XCD b mod 8 under the round-robin dispatch): median start and backward done of the deep tier
    print(f"rep {rep} deep by b mod 8 (median start / bwd): " + "  ".join(
        f"{x}: {int(np.median(w[x:256:8, 0]))}/{int(np.median(w[x:256:8, 1]))}" for x in range(8)), flush=True)
    print(f"rep {rep} bwd done of deep by 16s (max): " +
          " ".join(f"{x:5d}" for x in w[0:256, 1].reshape(16, 16).max(axis=1)), flush=True)
