"""Run K CP iterations of one config (for rocprofv3 --kernel-trace --stats; set
RAOCP_EAGER=1 so the iteration's kernels launch one by one, the trace cannot replay the
graph). python tools/prof_cp.py <config> [K] [float64|float32] (config 5 defaults to fp32)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]

import raocp.core as core  # noqa: E402
from raocp.problems import build_problem, recipe_config  # noqa: E402

cfg = int(sys.argv[1])
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dt = sys.argv[3] if len(sys.argv) > 3 else ("float32" if cfg == 5 else "float64")
r = recipe_config(cfg)
t0 = time.time()
cache = core.Cache(build_problem(r)[1], dtype=dt)
t1 = time.time()
nat = cache.native
alpha = 0.999 / nat.step_size()
ms = nat.cp_bench(r["x0"], K, alpha)
print(f"config {cfg}: {cache.packed.n} nodes, setup {t1 - t0:.1f} s, {K} iterations {ms:.2f} ms "
      f"({1e3 * ms / K:.1f} us/it)", flush=True)
