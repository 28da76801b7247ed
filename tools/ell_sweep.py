"""L / L^T timing sweep over the block shape (RAOCP_ELL_NODES x RAOCP_ELL_THREADS), one process.

The settings are read when a Cache (native context) is created, so each pair builds a fresh
context on the same problem. Prints the graph-timed us / launch and GB/s of algorithmic bytes.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raocp-toolbox_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import raocp.core as core
from raocp.problems import build_problem, recipe_config
import bench

cfgs = [int(c) for c in os.environ.get("CFGS", "4").split(",")]
pers = [int(v) for v in os.environ.get("PERS", "8,16,32,64,128").split(",")]
thrs = [int(v) for v in os.environ.get("THRS", "128,256,512").split(",")]
for cfg in cfgs:
    tree, prob = build_problem(recipe_config(cfg))
    for thr in thrs:
        for per in pers:
            os.environ["RAOCP_ELL_NODES"] = str(per)
            os.environ["RAOCP_ELL_THREADS"] = str(thr)
            c = core.Cache(prob)
            bP, bD = bench.algorithmic_bytes(c)
            ml = c.native.op_bench(0, 300)
            mt = c.native.op_bench(1, 300)
            print(f"cfg{cfg} thr={thr} per={per}  L {ml*1e3:6.2f} us {(bP+bD)/ml/1e6:5.0f} GB/s   "
                  f"LT {mt*1e3:6.2f} us {(bP+bD)/mt/1e6:5.0f} GB/s", flush=True)
            del c
