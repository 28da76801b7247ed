"""Diagnostics: stamps of the fused CP kernel (k_cp4, raocp_cp4.hip) at config 2: one family
task (STAMP_WG = its index among the parent ranges' tasks, default 200) stamps [entry,
loads issued, leaf children done, phase 1 done, phase 2 done, phase 3 done, exit], and every
wave its [start, end]; printed in ns (100 MHz), the waves' spans relative to the earliest
start, the slowest waves with their first task.
usage: python tools/cp_stamps.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raocp-toolbox_amd"))
WG = os.environ.get("STAMP_WG", "200")
os.environ["RAOCP_STAMP_KERNEL"] = "c" + WG  # the stamped workgroup / task after the letter
import numpy as np  # noqa: E402
import raocp.core as core  # noqa: E402
from raocp.problems import build_problem, recipe_config  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
r = recipe_config(2)
cache = core.Cache(build_problem(r)[1])
print(cache.native.kernel_info(10), "task", WG, flush=True)
for rep in range(reps):
    st = cache.native.debug_dyn_stamps(4096).astype(np.int64)
    v = st[:16][st[:16] != 0]
    w = st[32:32 + 4000].reshape(-1, 2)
    w = w[w[:, 0] != 0]
    t0 = w[:, 0].min()
    s0, s1 = (w[:, 0] - t0) * 10, (w[:, 1] - t0) * 10
    order = np.argsort(-s1)[:6]
    print(f"rep {rep}: task " + " ".join(f"{(x - v[0]) * 10:6d}" for x in v) +
          f" | {len(w)} waves: start {s0.min()}..{s0.max()} ns, end {s1.min()}..{s1.max()} ns, median span "
          f"{int(np.median(s1 - s0))}; slowest waves (index: start-end) " +
          " ".join(f"{i}:{s0[i]}-{s1[i]}" for i in order), flush=True)
