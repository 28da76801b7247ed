"""Diagnostics (a diagnostic build of the dynamics unit: VAR_UNIT=dynr tools/build_var.sh diag
-DRAOCP_DIAG, then RAOCP_HIP_LIB=build/var/diag.so): where the fused launch k_drc spends its time
at config 2. Every workgroup stamps its start, the end of its backward sweep, the end of its
forward sweep (the CP step's start) and its end (raocp_dynr.hip wg_stamp): printed per tier as
min / median / max in ns from the launch's earliest stamp. The first (deepest) and the last (top)
workgroup also stamp every wave's CP roles (cp_phase dstamp).
usage: RAOCP_STAMP_KERNEL=f python tools/drc_stamps.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raocp-toolbox_amd"))
import numpy as np  # noqa: E402
import raocp.core as core  # noqa: E402
from raocp.problems import build_problem, recipe_config  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
os.environ.setdefault("RAOCP_STAMP_KERNEL", "f")
r = recipe_config(2)
tree, prob = build_problem(r)
cache = core.Cache(prob)
print(cache.native.kernel_info(11), cache.native.kernel_info(9), flush=True)
tiers = [("deep", 0, 256), ("mid", 256, 16), ("top", 272, 1)]
for rep in range(reps):
    st = cache.native.debug_dyn_stamps(4096).astype(np.int64)
    if rep < reps - 2:
        continue
    w = st[1024:1024 + 4 * 273].reshape(273, 4)
    t0 = w[w > 0].min()
    w = np.where(w > 0, (w - t0) * 10, -1)
    for name, b0, n in tiers:
        blk = w[b0:b0 + n]
        d = ", ".join(f"{q} {np.min(blk[:, i]):6d} / {int(np.median(blk[:, i])):6d} / {np.max(blk[:, i]):6d}"
                      for i, q in ((0, "start"), (1, "bwd"), (3, "fwd"), (2, "end")))
        print(f"rep {rep} {name:4s}: {d}", flush=True)
    for which, base, b in (("deep wg 0", 3072, 0), ("top", 3136, 272)):
        s = st[base:base + 64].reshape(8, 8)
        s = np.where(s > 0, (s - t0) * 10, -1)
        print(f"rep {rep} {which} (fwd done {w[b, 3]}): per wave [start, role, barrier, role2, last role, "
              f"end, (slot waves: A2, SOC)] ns", flush=True)
        for wv in range(8):
            print(f"    wave {wv}: " + " ".join(f"{x:6d}" for x in s[wv, [0, 1, 2, 3, 5, 4, 6, 7]]), flush=True)
