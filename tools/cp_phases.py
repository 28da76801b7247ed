"""Timing diagnostics of the MFMA CP kernels: op_bench of k_cpd2 (op 2) and k_cpp2 (op 6)
with phases skipped (RAOCP_CP2_DBG bits: 1 child / x-u tiles, 2 parent rows / kernel
projection, 4 leaf tiles) and block shapes (RAOCP_CP2_W / _FB / _LB).
python tools/cp_phases.py <config>"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1] if len(sys.argv) > 1 else "4"
if len(sys.argv) > 2 and sys.argv[2] == "child":
    sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
    import raocp.core as core
    from raocp.problems import build_problem, recipe_config
    c = core.Cache(build_problem(recipe_config(int(cfg)))[1])
    print(f"cpd {1e3 * c.native.op_bench(2, 200):8.2f} us  cpp {1e3 * c.native.op_bench(6, 200):8.2f} us")
    sys.exit(0)
variants = [{}, {"RAOCP_CP2_DBG": "1"}, {"RAOCP_CP2_DBG": "2"}, {"RAOCP_CP2_DBG": "4"}, {"RAOCP_CP2_DBG": "7"},
            {"RAOCP_CP2_W": "4"}, {"RAOCP_CP2_W": "2"}, {"RAOCP_CP_V1": "1"}]
for v in variants:
    env = dict(os.environ, **v)
    out = subprocess.run([sys.executable, __file__, cfg, "child"], env=env, capture_output=True, text=True, timeout=120)
    print(f"c{cfg} {str(v):32s} {out.stdout.strip()} {out.stderr.strip()[-200:]}", flush=True)
