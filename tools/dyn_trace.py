"""Eager dynamics projections for a rocprofv3 kernel trace (one launch per tier / stage, no
graph): python tools/dyn_trace.py <config> [reps]. RAOCP_DYN3=1 selects the per-stage
sweep. Prints the context's launch list (raocp_kernel_info)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
import numpy as np
import raocp.core as core
from raocp.problems import build_problem, recipe_config

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
r = recipe_config(cfg)
cache = core.Cache(build_problem(r)[1], dtype="float32" if cfg == 5 else "float64")
cache.cache_initial_state(r["x0"])
cache.native.set_primal(np.random.default_rng(0).standard_normal(cache.primal_size))
for _ in range(reps):
    cache.native.project_on_dynamics()
from raocp.core._native import device_synchronize
device_synchronize(cache.native.device)
print(cache.native.kernel_info(9), flush=True)
