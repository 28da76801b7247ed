"""Timing probes of the fused launch k_drc at config 2 (a diagnostic build of the dynamics unit:
RAOCP_HIP_LIB=build/var/diag.so, tools/build_var.sh with VAR_UNIT=dynr -DRAOCP_DIAG). Each probe is
a fresh process with RAOCP_DR_FAULT set (raocp_dynr.h DrPlan::fault; the results are not valid,
the times are): 0 the launch as shipped, 64 no CP step, 128 no CP operand gather, 192 neither
(the sweep alone inside k_drc), 512 the CP step alone, 1024 no CP stores, 1536 the CP step alone
without stores; with 512: 64 no CP phase, 128 no gather (704: the weight DMA alone), 1664 the CP
phase alone without stores. Prints op_bench(11) (k_drc) and op_bench(9)
(k_dr) device times. usage: python tools/drc_probe.py [reps]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
    import raocp.core as core
    from raocp.problems import build_problem, recipe_config
    r = recipe_config(2)
    c = core.Cache(build_problem(r)[1])
    reps = int(sys.argv[2])
    t11 = c.native.op_bench(11, reps)
    t9 = c.native.op_bench(9, reps) if os.environ.get("RAOCP_DR_FAULT", "0") == "0" else 0.0
    print(f"fault {os.environ.get('RAOCP_DR_FAULT', '0'):>4s}  k_drc {1e3 * t11:7.2f} us  k_dr {1e3 * t9:7.2f} us", flush=True)
    sys.exit(0)
reps = sys.argv[1] if len(sys.argv) > 1 else "400"
for f in os.environ.get("PROBE_FAULTS", "0 64 128 192 512 576 640 704").split():
    env = dict(os.environ, RAOCP_DR_FAULT=f)
    out = subprocess.run([sys.executable, __file__, "child", reps], env=env, capture_output=True, text=True, timeout=120)
    print(out.stdout.strip() or out.stderr.strip()[-300:], flush=True)
