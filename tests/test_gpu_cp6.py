"""GPU parity of k_cp6 (raocp_cp5.hip): the fused CP iteration of k_cp3 (raocp_cp3.hip;
solver.py:27-95, cache.py:248-393) for the small C = 2 trees as one workgroup per 16-parent
family tile, its 2 C waves splitting the tile's roles (a child slot each for the parent
products, the SOC and the eta3..eta6 rows; the leaf children of leaf-parent tiles; the box
projection, the step of the primal and the kernel projection). The default of fp64 trees
with C = 2 at nx = 20, nu = 8 (config 2) whose nodes are all boxed or all unboxed;
RAOCP_CP6=0 keeps k_cp4.

Every entry's arithmetic is k_cp3's; the compiler contracts multiply-adds by code shape, so
k_cp6, k_cp4 and k_cp3 agree at rounding level: 1e-12 per residual trace entry and on the
iterate over 30 iterations (a graph batch boundary at 24 inside). Against the oracle: 1e-8 per
trace entry (BASELINE.json north_star), 1e-10 on the iterate. Shrinking the grid (every
workgroup looping over several tiles) changes no entry's arithmetic and the residual maxima
are order-free, so a one-workgroup grid reproduces the default grid bit for bit.
"""
import os

import numpy as np
import pytest

import raocp.core as core
from raocp.problems import build_problem, recipe_config, recipe_synthetic
from helpers import rel_err, trace_rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _pair_loop(monkeypatch):
    """These tests pin k_cp6 itself in the CP loop: RAOCP_DRC=0 keeps the pair k_dr + k_cp6
    where the fused launch k_drc would replace it (config 2; tests/test_gpu_drc.py)."""
    monkeypatch.setenv("RAOCP_DRC", "0")


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


def _recipe(case):
    if case in ("c2", "c2-nobox"):
        r = recipe_config(2)
        if case == "c2-nobox":
            r["nl_min"] = r["nl_max"] = r["l_min"] = r["l_max"] = None
        return r
    if case == "bin3":  # 15 nodes: one leaf-parent tile of 4, one nonleaf tile of 3
        return recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 3, 3, 20, 8, seed=11)
    if case == "bin7":  # 255 nodes: partial tiles at every level
        return recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 7, 7, 20, 8, seed=12)
    if case == "markov":  # 2 modes with their own dynamics, 1,023 nodes
        P = np.array([[.7, .3], [.2, .8]])
        return recipe_synthetic(P, np.array([.4, .6]), 9, 9, 20, 8, seed=13)
    if case == "a95":
        return recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 9, 9, 20, 8, seed=14, alpha_r=0.95)
    raise ValueError(case)


def _run(cache, x0, K, alpha, tol=0.0):
    st, err, derr = cache.native.cp_run(x0, K, tol, alpha)
    return st, err, derr, cache.get_primal_flat(), cache.get_dual_flat()


@pytest.mark.parametrize("case", ["c2", "c2-nobox", "bin3", "bin7", "markov", "a95"])
def test_cp6_matches_cp4_cp3_and_oracle(case):
    from oracle.raocp_oracle import OracleProblem
    r = _recipe(case)
    tree, prob = build_problem(r)
    c6 = core.Cache(prob)
    c4 = _with_env({"RAOCP_CP6": "0"}, lambda: core.Cache(prob))
    c3 = _with_env({"RAOCP_CP6": "0", "RAOCP_CP4": "0"}, lambda: core.Cache(prob))
    assert c6.native.kernel_info(10) == "k_cp6<double, 20, 8, 2>"
    assert c4.native.kernel_info(10) == "k_cp4<double, 20, 8>"
    assert c3.native.kernel_info(10).startswith("k_cp3<double, 20, 8")
    alpha = 0.999 / c6.native.step_size()
    K = 30
    a = _run(c6, r["x0"], K, alpha)
    for other in (c4, c3):
        b = _run(other, r["x0"], K, alpha)
        assert a[0] == b[0] == 1 and a[1].shape == b[1].shape == (K + 1, 3)
        assert trace_rel_err(a[1], b[1]) <= 1e-12 and trace_rel_err(a[2], b[2]) <= 1e-12
        assert rel_err(a[3], b[3]) <= 1e-12 and rel_err(a[4], b[4]) <= 1e-12
    st_o, err_o, derr_o, z_o, e_o, _ = OracleProblem(prob).chock(r["x0"], K, 0.0, alpha=alpha)
    assert st_o == 1
    assert trace_rel_err(a[1], err_o) <= 1e-8 and trace_rel_err(a[2], derr_o) <= 1e-8
    assert rel_err(a[3], z_o) <= 1e-10 and rel_err(a[4], e_o) <= 1e-10


def test_cp6_leafbox_falls_back_to_cp4():
    """Leaf boxes only (a second box pattern): k_cp6 is not compiled for it, k_cp4 runs."""
    r = recipe_config(2)
    r["nl_min"] = r["nl_max"] = None
    tree, prob = build_problem(r)
    assert core.Cache(prob).native.kernel_info(10) == "k_cp4<double, 20, 8>"


@pytest.mark.parametrize("case,grid", [("c2", "1"), ("c2", "7"), ("bin7", "1")])
def test_cp6_small_grids_bit_identical(case, grid):
    r = _recipe(case)
    tree, prob = build_problem(r)
    a = core.Cache(prob)
    b = _with_env({"RAOCP_CP6_GRID": grid}, lambda: core.Cache(prob))
    alpha = 0.999 / a.native.step_size()
    ra = _run(a, r["x0"], 14, alpha)
    rb = _run(b, r["x0"], 14, alpha)
    for u, v in zip(ra, rb):
        assert np.array_equal(u, v)


def test_cp6_early_stop_matches_cp4():
    """tol = the 42nd residual of k_cp4's loop (clear of rounding): both stop at the same
    iteration of a graph batch with the same history."""
    r = recipe_config(2)
    tree, prob = build_problem(r)
    c6 = core.Cache(prob)
    c4 = _with_env({"RAOCP_CP6": "0"}, lambda: core.Cache(prob))
    alpha = 0.999 / c6.native.step_size()
    _, err, _ = c4.native.cp_run(r["x0"], 60, 0.0, alpha)
    tol = float(err[41].max()) * (1 + 1e-9)
    a = _run(c6, r["x0"], 60, alpha, tol)
    b = _run(c4, r["x0"], 60, alpha, tol)
    assert a[0] == b[0] == 0 and a[1].shape == b[1].shape and a[1].shape[0] <= 42
    assert trace_rel_err(a[1], b[1]) <= 1e-12 and rel_err(a[3], b[3]) <= 1e-12


def test_cp6_nan_in_box_raises():
    """A NaN reaching a box projection (Rectangle._constrain, rectangle.py:50-59) raises
    ValueError through k_cp6 as through the reference."""
    r = recipe_config(2)
    tree, prob = build_problem(r)
    cache = core.Cache(prob)
    assert cache.native.kernel_info(10).startswith("k_cp6")
    x0 = np.array(r["x0"], dtype=float)
    x0[3] = np.nan
    alpha = 0.999 / cache.native.step_size()
    with pytest.raises(ValueError):
        cache.native.cp_run(x0, 5, 0.0, alpha)
