"""Standalone L / L^T at a config, as bench.py's l_sweep measures them (op_pair: HIP events
over a graph of back-to-back launches cycling over nsets buffer sets, beyond the 256 MiB
Infinity Cache for nsets * bytes > 256 MiB). python tools/l_sweep.py <config> [dtype] [nsets]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
import raocp.core as core  # noqa: E402
from raocp.problems import build_problem, recipe_config  # noqa: E402
from bench import op_pair  # noqa: E402

cfg = int(sys.argv[1])
dt = sys.argv[2] if len(sys.argv) > 2 else "float64"
nsets = int(sys.argv[3]) if len(sys.argv) > 3 else 1
c = core.Cache(build_problem(recipe_config(cfg))[1], dtype=dt)
res = op_pair(c.native, c, 4 if dt == "float32" else 8, 200, nsets)
for k in ("L", "L_transpose"):
    r = res[k]
    print(f"config {cfg} {dt} {k:12s} {r['kernel']:34s} {r['us_per_launch']:8.2f} us  frac {r['frac']:.3f}", flush=True)
print(json.dumps(res))
