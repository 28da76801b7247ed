"""GPU parity of the persistent CP engine (raocp_mega.hip: one launch per solve, the tree cut
at stage s into a top workgroup and one workgroup per stage-s subtree) against the oracle
and against the multi-launch path, for several cuts.

Tolerances as in test_gpu_parity.py: CP residual traces 1e-8 relative per entry
(BASELINE.json north_star), iterates 1e-10 relative.
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


@pytest.fixture(scope="module")
def c2_ref():
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(2)
    tree, prob = build_problem(r)
    orc = OracleProblem(prob)
    lam, _ = orc.step_size()
    alpha = 0.999 / lam
    st, err, derr, z, e, _ = orc.chock(r["x0"], 29, 0.0, alpha=alpha)
    return r, prob, alpha, (st, err, derr, z, e)


@pytest.mark.parametrize("cut", [0, 5, 6, 7])
def test_c2_engine_cuts_vs_oracle(c2_ref, cut):
    """cut 0: the engine off (graph-replayed launches, the default); others: forced cut stage."""
    r, prob, alpha, (st_o, err_o, derr_o, z_o, e_o) = c2_ref
    env = {"RAOCP_MEGA": "0"} if cut == 0 else {"RAOCP_MEGA": "1", "RAOCP_MEGA_CUT": cut}
    cache = _with_env(env, lambda: core.Cache(prob))
    assert cache.native.engine_cut() == cut
    status, err, derr = cache.native.cp_run(r["x0"], 29, 0.0, alpha)
    assert status == st_o == 1 and err.shape == (30, 3)
    assert trace_rel_err(err, err_o) <= 1e-8
    assert trace_rel_err(derr, derr_o) <= 1e-8
    assert rel_err(cache.get_primal_flat(), z_o) <= 1e-10
    assert rel_err(cache.get_dual_flat(), e_o) <= 1e-10


def test_engine_declines_a_cut_that_does_not_fit(c2_ref):
    """cut 3 leaves 1,023-node subtrees: their LDS plan does not fit, the context falls back
    to the multi-kernel iteration (and still solves)"""
    r, prob, alpha, (st_o, err_o, derr_o, z_o, e_o) = c2_ref
    cache = _with_env({"RAOCP_MEGA": "1", "RAOCP_MEGA_CUT": 3}, lambda: core.Cache(prob))
    assert cache.native.engine_cut() == 0
    status, err, derr = cache.native.cp_run(r["x0"], 29, 0.0, alpha)
    assert trace_rel_err(err, err_o) <= 1e-8


def test_engine_stops_on_tolerance_like_the_reference(golden):
    """main.py tree (Markov, uneven child counts) through the engine: 937 iterations,
    status 0; the stopping test taken one iteration late must not move the iterate."""
    z = golden("main_trace")
    r, tree, prob = problem_from_golden(z, "main")
    solver = _with_env({"RAOCP_MEGA": "1"}, lambda: core.Solver(problem_spec=prob))
    assert solver.cache.native.engine_cut() > 0
    status = solver.chock(initial_state=r["x0"].reshape(-1, 1), max_iters=int(z["main/cp_max_iters"]),
                          tol=float(z["main/cp_tol"]), step_size=float(z["main/cp_alpha"]))
    assert status == 0
    assert solver.error_cache.shape == (937, 3)
    assert trace_rel_err(solver.error_cache, z["main/cp_error"]) <= 1e-8
    assert rel_err(solver.cache.get_primal_flat(), z["main/cp_z"]) <= 1e-9
    assert rel_err(solver.cache.get_dual_flat(), z["main/cp_eta"]) <= 1e-9


def test_engine_repeated_runs_are_identical(c2_ref):
    """the hand-off words are re-armed per launch: two solves give the same bits"""
    r, prob, alpha, _ = c2_ref
    cache = _with_env({"RAOCP_MEGA": "1"}, lambda: core.Cache(prob))
    assert cache.native.engine_cut() > 0
    _, e1, _ = cache.native.cp_run(r["x0"], 9, 0.0, alpha)
    z1 = cache.get_primal_flat().copy()
    _, e2, _ = cache.native.cp_run(r["x0"], 9, 0.0, alpha)
    assert np.array_equal(e1, e2)
    assert np.array_equal(z1, cache.get_primal_flat())


@pytest.mark.parametrize("cut", [0, 6, 7])
def test_c2_dynamics_engine_vs_oracle(c2_ref, cut):
    """graph-replayed CP iteration whose dynamics projection is ONE launch of the
    dynamics-only engine (cut 0: the planner's choice)"""
    r, prob, alpha, (st_o, err_o, derr_o, z_o, e_o) = c2_ref
    env = {"RAOCP_DYN_ENGINE": "1"}
    if cut:
        env["RAOCP_DYN_ENGINE_CUT"] = cut
    cache = _with_env(env, lambda: core.Cache(prob))
    dc = cache.native.dyn_engine_cut()
    assert dc > 0 and (cut == 0 or dc == cut)
    for _ in range(2):  # the epoch-tagged flags carry over between solves
        status, err, derr = cache.native.cp_run(r["x0"], 29, 0.0, alpha)
        assert status == st_o == 1 and err.shape == (30, 3)
        assert trace_rel_err(err, err_o) <= 1e-8
        assert trace_rel_err(derr, derr_o) <= 1e-8
        assert rel_err(cache.get_primal_flat(), z_o) <= 1e-10
        assert rel_err(cache.get_dual_flat(), e_o) <= 1e-10


def test_dynamics_engine_main_py_trace(golden):
    z = golden("main_trace")
    r, tree, prob = problem_from_golden(z, "main")
    solver = _with_env({"RAOCP_DYN_ENGINE": "1"}, lambda: core.Solver(problem_spec=prob))
    assert solver.cache.native.dyn_engine_cut() > 0
    status = solver.chock(initial_state=r["x0"].reshape(-1, 1), max_iters=int(z["main/cp_max_iters"]),
                          tol=float(z["main/cp_tol"]), step_size=float(z["main/cp_alpha"]))
    assert status == 0 and solver.error_cache.shape == (937, 3)
    assert trace_rel_err(solver.error_cache, z["main/cp_error"]) <= 1e-8
    assert rel_err(solver.cache.get_primal_flat(), z["main/cp_z"]) <= 1e-9
