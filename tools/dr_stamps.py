"""Diagnostics: in-kernel stamps of the regular-tree sweep (raocp_dynr.hip). For the first
subtree of every tier, k_dr_up stamps [start, (children arrived), prologue landed, levels
done, published] and k_dr_down [start, (parent's flag seen), root x in LDS, levels done,
flag set]; printed in ns from the launch's earliest stamp (100 MHz clock).
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
    for name, base in (("up", 0), ("down", 64)):
        blk = st[base:base + 64].reshape(4, 16)
        live = blk[blk != 0]
        if live.size == 0:
            continue
        t0 = live.min()
        rows = []
        for k in range(4):
            v = blk[k][blk[k] != 0]
            if v.size:
                rows.append(f"tier {k}: " + " ".join(f"{(x - t0) * 10:6d}" for x in v))
        print(f"rep {rep} {name:4s} " + " | ".join(rows), flush=True)
