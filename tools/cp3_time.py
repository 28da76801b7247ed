"""Per-launch device time of the CP iteration's kernels after the dynamics sweep (op_bench 10:
k_cp4 / k_cp3, or k_cpd* + k_cpp* with RAOCP_CP3=0), the dynamics projection (op 9) and the CP loop
(cp_bench) at configs 2, 4 (fp64) and 5 (fp32). python tools/cp3_time.py [configs...]
(CP3T_QUICK=1: the default and RAOCP_DY3_TOP=0 / RAOCP_CP4_HELPER=0 only; CP3T_VARS="A=1,B=2|C=0":
the default and these environment variants only)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
    import raocp.core as core
    from raocp.problems import build_problem, recipe_config
    cfg = int(sys.argv[2])
    r = recipe_config(cfg)
    c = core.Cache(build_problem(r)[1], dtype="float32" if cfg == 5 else "float64")
    nat = c.native
    reps = {2: 400, 3: 100, 4: 100, 5: 20}[cfg]
    t10 = nat.op_bench(10, reps)
    t9 = nat.op_bench(9, max(1, reps // 2))
    t11 = nat.op_bench(11, reps) if nat.kernel_info(11) else 0.0  # the fused launch (k_drc)
    alpha = 0.999 / nat.step_size(rtol=1e-7 if cfg == 5 else 1e-14)
    K = {2: 480, 3: 120, 4: 120, 5: 24}[cfg]
    ms = nat.cp_bench(r["x0"], K, alpha)
    var = ",".join(f"{k[6:]}={v}" for k, v in sorted(os.environ.items()) if k.startswith("RAOCP_")) or "default"
    print(f"config {cfg} {var:12s} {nat.kernel_info(10):40s} {nat.kernel_info(9)[:34]:34s} "
          f"cp {1e3 * t10:8.1f} us  dyn {1e3 * t9:8.1f} us  fused {1e3 * t11:8.1f} us  loop {1e3 * ms / K:8.1f} us/it",
          flush=True)
    sys.exit(0)
cfgs = sys.argv[1:] or ["2", "4", "5"]
for cfg in cfgs:
    variants = [{}, {"RAOCP_CP3": "0"}, {"RAOCP_CP3_SPLIT": "1" if cfg != "2" else "0"}]
    variants.append({"RAOCP_DYN3": "1"} if cfg != "5" else {"RAOCP_DYN3": "0"})
    if cfg == "2":
        variants += [{"RAOCP_CP4": "0"}, {"RAOCP_DR": "0"}]
    else:
        variants.append({"RAOCP_DY3_TOP": "0"})
    if os.environ.get("CP3T_VARS"):
        variants = [{}] + [dict(kv.split("=") for kv in grp.split(",")) for grp in os.environ["CP3T_VARS"].split("|")]
    elif os.environ.get("CP3T_QUICK"):  # the default and the per-stage top launches only
        variants = [{}] + ([{"RAOCP_DY3_TOP": "0"}] if cfg != "2" else [{"RAOCP_CP4_HELPER": "0"}])
    for v in variants:
        env = dict(os.environ, **v)
        out = subprocess.run([sys.executable, __file__, "child", cfg], env=env, capture_output=True, text=True,
                             timeout=300)
        print(out.stdout.strip() or out.stderr.strip()[-400:], flush=True)
