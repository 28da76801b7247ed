"""The RCCL shard transport with ONE rank (R = 1 forced): the sharded iteration with its
RCCL all-gathers, graph-captured, must reproduce the unsharded solve exactly, on the
two-launch CP kernels (RAOCP_CP3=0) and on the fused k_cp3 (a shard's two k_cp3 launches
around X1). Run as its own process: torch must not be imported (see bench.py SocketGroup)."""
import os, sys
os.environ["RAOCP_SHARD_FORCE"] = "1"
# the unsharded reference runs the kernels a shard runs: the tier launches (not k_dr) and
# k_cp3 (not k_cp6 / k_cp4, the same arithmetic with a different FMA contraction)
os.environ["RAOCP_DR"] = "0"
os.environ["RAOCP_CP4"] = "0"
os.environ["RAOCP_CP6"] = "0"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raocp-toolbox_amd"))
import numpy as np
import raocp.core as core
from raocp.core._native import comm_unique_id
from raocp.problems import build_problem, recipe_config
r = recipe_config(2)
tree, prob = build_problem(r)
for cp3 in ("0", "1"):
    os.environ["RAOCP_CP3"] = cp3  # the same CP kernels unsharded and sharded
    base = core.Cache(prob)
    alpha = 0.999 / base.native.step_size()
    st0, e0, d0 = base.native.cp_run(r["x0"], 60, 0.0, alpha)
    sh = core.Cache(prob)
    sh.native.shard(0, 1)
    sh.native.comm_init(comm_unique_id(), 0, 1)
    st1, e1, d1 = sh.native.cp_run(r["x0"], 60, 0.0, alpha)
    assert st0 == st1 and np.array_equal(e0, e1) and np.array_equal(d0, d1), (np.max(np.abs(e0 - e1)))
    assert np.array_equal(base.get_primal_flat(), sh.get_primal_flat())
    ms0 = base.native.cp_bench(r["x0"], 480, alpha)
    ms1 = sh.native.cp_bench(r["x0"], 480, alpha)
    print(f"RCCL single-rank shard path OK ({base.native.kernel_info(10)}): traces bit-identical; "
          f"{480 / ms0 * 1e3:.0f} it/s unsharded, {480 / ms1 * 1e3:.0f} it/s through the shard exchange path")
# the shipped kernels at config 4 (BASELINE configs[3], the sharded bench leg's tree): k_cp5 and
# k_dy3 with its merged top, no pins on either side
for k in ("RAOCP_DR", "RAOCP_CP4", "RAOCP_CP6", "RAOCP_CP3"):
    os.environ.pop(k, None)
r = recipe_config(4)
tree, prob = build_problem(r)
base = core.Cache(prob)
alpha = 0.999 / base.native.step_size()
st0, e0, d0 = base.native.cp_run(r["x0"], 24, 0.0, alpha)
sh = core.Cache(prob)
sh.native.shard(0, 1)
sh.native.comm_init(comm_unique_id(), 0, 1)
assert sh.native.kernel_info(10).startswith("k_cp5_leaf"), sh.native.kernel_info(10)
st1, e1, d1 = sh.native.cp_run(r["x0"], 24, 0.0, alpha)
assert st0 == st1 and np.array_equal(e0, e1) and np.array_equal(d0, d1), (np.max(np.abs(e0 - e1)))
assert np.array_equal(base.get_primal_flat(), sh.get_primal_flat())
ms0 = base.native.cp_bench(r["x0"], 240, alpha)
ms1 = sh.native.cp_bench(r["x0"], 240, alpha)
print(f"RCCL single-rank shard path OK at config 4 ({sh.native.kernel_info(10)}; {sh.native.kernel_info(9)}): "
      f"traces bit-identical; {240 / ms0 * 1e3:.0f} it/s unsharded, {240 / ms1 * 1e3:.0f} it/s through the shard "
      f"exchange path")
