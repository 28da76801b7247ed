"""Diagnostics (diagnostic build: make DIAG=1, or tools/build_var.sh with -DRAOCP_DIAG): stamps of
k_cp6 (raocp_cp5.hip) at config 2. The workgroup STAMP_WG (default 200: a tile of nonleaf
parents; 0..127 are leaf-parent tiles) stamps per wave [entry, prologue done, role done,
barrier, streams done, exit]; every workgroup its [entry, exit]. Printed in ns (100 MHz).
usage: RAOCP_HIP_LIB=build/var/diag.so python tools/cp6_stamps.py [reps]"""
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
print(cache.native.kernel_info(10), "workgroup", WG, flush=True)
for rep in range(reps):
    st = cache.native.debug_dyn_stamps(4200).astype(np.int64)
    w = st[64:64 + 4000].reshape(-1, 2)
    w = w[w[:, 0] != 0]
    t0 = w[:, 0].min()
    s0, s1 = (w[:, 0] - t0) * 10, (w[:, 1] - t0) * 10
    print(f"rep {rep}: {len(w)} workgroups: entry {s0.min()}..{s0.max()} ns, exit {s1.min()}..{s1.max()} ns, "
          f"median span {int(np.median(s1 - s0))} ns; slowest (block: entry-exit) " +
          " ".join(f"{i}:{s0[i]}-{s1[i]}" for i in np.argsort(-s1)[:5]), flush=True)
    for wv in range(4):
        v = st[8 * wv:8 * wv + 8]
        v = v[v != 0]
        if len(v):
            print(f"   wave {wv}: " + " ".join(f"{(x - t0) * 10:6d}" for x in v), flush=True)
