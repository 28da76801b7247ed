"""Print the dynamics plan (tiers, LDS, fold) for BASELINE configs (RAOCP_DYN_VERBOSE)."""
import os
import sys
os.environ["RAOCP_DYN_VERBOSE"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "raocp-toolbox_amd"))
import raocp.core as core
from raocp.problems import build_problem, recipe_config
for cfg in [int(a) for a in sys.argv[1:]] or [2]:
    tree, prob = build_problem(recipe_config(cfg))
    print(f"config {cfg}:", flush=True)
    core.Cache(prob)
