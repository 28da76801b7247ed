"""L / L^T launch times (op_bench: graph of back-to-back launches, HIP events) at a config,
fp64 or fp32. python tools/l_sweep.py <config> [float32]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
import raocp.core as core  # noqa: E402
from raocp.problems import build_problem, recipe_config  # noqa: E402
from bench import active_sizes  # noqa: E402

cfg = int(sys.argv[1])
dt = sys.argv[2] if len(sys.argv) > 2 else "float64"
c = core.Cache(build_problem(recipe_config(cfg))[1], dtype=dt)
P, D = active_sizes(c)
w = 4 if dt == "float32" else 8
for op, name in ((0, "L"), (1, "L^T")):
    ms = c.native.op_bench(op, 200)
    print(f"config {cfg} {dt} {name}: {1e3 * ms:.2f} us, {w * (P + D) / (ms * 1e-3) / 1e9:.0f} GB/s "
          f"({w * (P + D) / 1e6:.1f} MB per launch)", flush=True)
