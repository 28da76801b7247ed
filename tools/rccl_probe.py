"""Probe: can this process's RCCL (dlopen'd by libraocp_hip.so) init a 1-rank communicator,
with and without torch imported? (diagnostics for the shard transport)"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raocp-toolbox_amd"))
import raocp.core as core
from raocp.core._native import comm_unique_id, load_library
from raocp.problems import build_problem, recipe_config
load_library()
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch  # noqa: F401
    import torch.distributed  # noqa: F401
r = recipe_config(2)
tree, prob = build_problem(r)
c = core.Cache(prob)
c.native.shard(0, 1)
uid = comm_unique_id()
c.native.rank, c.native.nranks = 0, 1
try:
    c.native._lib.raocp_shard_setup(c.native._h, 1, 0)
    import numpy as np, ctypes
    buf = np.frombuffer(uid, dtype=np.uint8).copy()
    rc = c.native._lib.raocp_comm_init(c.native._h, buf.ctypes.data_as(ctypes.c_void_p), 1, 0)
    print("comm_init rc", rc, c.native._lib.raocp_last_error())
except Exception as e:
    print("exception", e)
