"""GPU parity of the opt-in kernel variants (measured slower on MI355X than the defaults,
kept correct): the CP stopping test fused into k_cpp's last block (RAOCP_FUSE_CHECK=1);
and the default per-parent L^T tiles against the LDS-staged path
(RAOCP_ELLT_PARENT_TILES=0).

Tolerances as in test_gpu_parity.py.
"""
import os

import numpy as np
import pytest

import raocp.core as core
from raocp.problems import build_problem, recipe_config
from helpers import problem_from_golden, rel_err, trace_rel_err

pytestmark = pytest.mark.gpu


def _with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_fused_stopping_test_c2_vs_oracle():
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(2)
    tree, prob = build_problem(r)
    orc = OracleProblem(prob)
    cache = _with_env({"RAOCP_FUSE_CHECK": "1"}, lambda: core.Cache(prob))
    alpha = 0.999 / cache.native.step_size()
    st_o, err_o, derr_o, z_o, e_o, _ = orc.chock(r["x0"], 29, 0.0, alpha=alpha)
    for _ in range(2):  # the ticket is re-armed by the last block of every launch
        status, err, derr = cache.native.cp_run(r["x0"], 29, 0.0, alpha)
        assert status == st_o == 1 and err.shape == (30, 3)
        assert trace_rel_err(err, err_o) <= 1e-8
        assert trace_rel_err(derr, derr_o) <= 1e-8
        assert rel_err(cache.get_primal_flat(), z_o) <= 1e-10


def test_fused_stopping_test_main_py(golden):
    z = golden("main_trace")
    r, tree, prob = problem_from_golden(z, "main")
    solver = _with_env({"RAOCP_FUSE_CHECK": "1"}, lambda: core.Solver(problem_spec=prob))
    status = solver.chock(initial_state=r["x0"].reshape(-1, 1), max_iters=int(z["main/cp_max_iters"]),
                          tol=float(z["main/cp_tol"]), step_size=float(z["main/cp_alpha"]))
    assert status == 0 and solver.error_cache.shape == (937, 3)
    assert trace_rel_err(solver.error_cache, z["main/cp_error"]) <= 1e-8
    assert rel_err(solver.cache.get_primal_flat(), z["main/cp_z"]) <= 1e-9


@pytest.mark.parametrize("cfg", [2, 3, 4, "4-modes"])
def test_ell_t_parent_tiles_bit_identical_to_staged(cfg):
    """k_ell_t's per-parent MFMA tiles (regular blocks, default) against the LDS-staged
    product path (RAOCP_ELLT_PARENT_TILES=0): the children are summed in the same order, so
    the results are bit-identical; both match the oracle. Config 4-modes mixes weight tables
    (the staged path is taken there either way)."""
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(4 if cfg == "4-modes" else cfg)
    if cfg == "4-modes":
        r["Q"] = np.array([(1.0 + k) * q for k, q in enumerate(r["Q"])])
    tree, prob = build_problem(r)
    tiles = core.Cache(prob)
    staged = _with_env({"RAOCP_ELLT_PARENT_TILES": "0"}, lambda: core.Cache(prob))
    rng = np.random.default_rng(11)
    ee = rng.standard_normal(tiles.dual_size)
    a, b = tiles.native.ell_t(ee), staged.native.ell_t(ee)
    assert np.array_equal(a, b)
    assert rel_err(a, OracleProblem(prob).ell_t(ee)) <= 1e-12
