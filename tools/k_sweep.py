"""Fixed cost of a benchmark call: cp_bench at K iterations (config 2), the device time between
its events and the wall time of prepare-less calls, median of 7, graph-replayed and eager
(RAOCP_EAGER=1 in a child). python tools/k_sweep.py"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
    import numpy as np
    import raocp.core as core
    from raocp.core._native import device_synchronize
    from raocp.problems import build_problem, recipe_config
    r = recipe_config(2)
    c = core.Cache(build_problem(r)[1])
    nat = c.native
    alpha = 0.999 / nat.step_size()
    nat.cp_bench(r["x0"], 48, alpha)
    for K in (1, 2, 5, 10, 20, 24, 25, 48, 96, 480):
        dev, wall = [], []
        for _ in range(7):
            nat.cp_prepare(K, r["x0"], alpha)
            device_synchronize(nat.device)
            t0 = time.perf_counter()
            dev.append(nat.cp_bench(None, K, alpha))
            device_synchronize(nat.device)
            wall.append(time.perf_counter() - t0)
        d, w = 1e3 * float(np.median(dev)), 1e6 * float(np.median(wall))
        print(f"eager={os.environ.get('RAOCP_EAGER', '0')} K={K:4d} device {d:9.1f} us ({d / K:6.2f}/it) "
              f"wall {w:9.1f} us ({w / K:6.2f}/it)", flush=True)
    # the benchmark's order: a fresh graph for K = 20 after a 5-iteration warmup, one timed call
    for rep in range(5):
        nat.cp_bench(r["x0"], 5, alpha)
        nat.cp_prepare(20, r["x0"], alpha)
        device_synchronize(nat.device)
        t0 = time.perf_counter()
        d = nat.cp_bench(None, 20, alpha)
        device_synchronize(nat.device)
        w = time.perf_counter() - t0
        print(f"eager={os.environ.get('RAOCP_EAGER', '0')} fresh K=20 device {1e3 * d:9.1f} us wall {1e6 * w:9.1f} us",
              flush=True)
    sys.exit(0)
for eager in (os.environ.get("KS_EAGER", "0 1").split()):
    out = subprocess.run([sys.executable, __file__, "child"], env=dict(os.environ, RAOCP_EAGER=eager),
                         capture_output=True, text=True, timeout=300)
    print(out.stdout.strip() or out.stderr.strip()[-600:], flush=True)
