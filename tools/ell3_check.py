"""k_ell3 (streaming wave tasks) vs the block kernels: parity vs the oracle and launch times.
python tools/ell3_check.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1:
    sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
    import numpy as np
    import raocp.core as core
    from raocp.problems import build_problem, recipe_config
    from oracle.raocp_oracle import OracleProblem
    from bench import active_sizes
    cfg, dt = int(sys.argv[1]), sys.argv[2]
    prob = build_problem(recipe_config(cfg))[1]
    c = core.Cache(prob, dtype=dt)
    P, D = active_sizes(c)
    w = 4 if dt == "float32" else 8
    zz = np.random.default_rng(5).standard_normal(c.primal_size)
    err = -1.0
    if cfg != 5:
        ref = OracleProblem(prob).ell(zz)
        err = float(np.max(np.abs(c.native.ell(zz) - ref)) / np.max(np.abs(ref)))
    ms = c.native.op_bench(0, 200)
    print(f"c{cfg} {dt} ELL3={os.environ.get('RAOCP_ELL3', '0')} grid={os.environ.get('RAOCP_ELL3_GRID', 'auto')}: "
          f"L {1e3 * ms:.2f} us {w * (P + D) / (ms * 1e-3) / 1e9:.0f} GB/s, rel err {err:.1e}", flush=True)
    sys.exit(0)
for cfg, dt in ((2, "float64"), (4, "float64"), (5, "float32")):
    for env in ({"RAOCP_ELL3": "0"}, {"RAOCP_ELL3": "1"}, {"RAOCP_ELL3": "1", "RAOCP_ELL3_GRID": "1024"},
                {"RAOCP_ELL3": "1", "RAOCP_ELL3_GRID": "4096"}, {"RAOCP_ELL3": "1", "RAOCP_ELL3_GRID": "16384"}):
        out = subprocess.run([sys.executable, __file__, str(cfg), dt], env=dict(os.environ, **env), capture_output=True,
                             text=True, timeout=300)
        print(out.stdout.strip(), out.stderr.strip()[-300:], flush=True)
