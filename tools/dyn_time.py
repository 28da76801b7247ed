"""Device time of one dynamics projection (op_bench 9, HIP events over graph-replayed
launches) under environment variants: python tools/dyn_time.py <config> VAR=V[,VAR=V] ...
(each variant a fresh process; "default" for none). DYN_DTYPE=float64 runs config 5 in fp64."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
    import raocp.core as core
    from raocp.problems import build_problem, recipe_config
    cfg = int(sys.argv[2])
    dt = os.environ.get("DYN_DTYPE") or ("float32" if cfg == 5 else "float64")
    c = core.Cache(build_problem(recipe_config(cfg))[1], dtype=dt)
    reps = {2: 200, 3: 50, 4: 50, 5: 20}[cfg]
    t = c.native.op_bench(9, reps)
    print(f"config {cfg} {dt} {sys.argv[3]:28s} dyn {1e3 * t:8.1f} us  {c.native.kernel_info(9)}", flush=True)
    sys.exit(0)
cfg = sys.argv[1]
for var in sys.argv[2:] or ["default"]:
    env = dict(os.environ)
    if var != "default":
        env.update(kv.split("=", 1) for kv in var.split(","))
    out = subprocess.run([sys.executable, __file__, "child", cfg, var], env=env, capture_output=True, text=True,
                         timeout=300)
    print(out.stdout.strip() or out.stderr.strip()[-400:], flush=True)
