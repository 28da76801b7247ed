"""GPU parity of the regular-tree dynamics sweep k_dr (raocp_dynr.hip; cache.py:259-288): one
launch, one workgroup per subtree of every tier running its backward and forward sweeps, the
q rows up and the x rows down as tagged 8-byte granules, every node address computed from
(stage, subtree). The default of fp64 regular trees at nx = 20, nu = 8 (config 2);
RAOCP_DR=0 falls back to the tiered sweep (raocp_dynf.hip / raocp_dyn.hip).

Tolerances: the projection against the oracle within 1e-12 of the largest entry and exact
feasibility x_j = A_j x_i + B_j u_i to 1e-12; against the tiered sweep (the same algebra, a
different summation order) 1e-13 of the largest entry; the CP loop against the tiered sweep
1e-10 per trace entry and the oracle 1e-8 (BASELINE.json north_star); the projection after
1,000 back-to-back launches (the tag advanced inside the kernel) bit for bit; a forced hand-off timeout reported as an error within a fraction of a second.
"""
import os
import time

import numpy as np
import pytest

import raocp.core as core
from raocp.problems import build_problem, recipe_config, recipe_synthetic
from helpers import rel_err, trace_rel_err

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


def _recipe(cfg):
    if cfg == "quad":  # branching 4, 6 stages
        return recipe_synthetic(np.full((4, 4), .25), np.full(4, .25), 6, 6, 20, 8, seed=6)
    if cfg == "tri":  # branching 3 (split-k groups of 4 lanes, one idle slot)
        return recipe_synthetic(np.full((3, 3), 1 / 3), np.full(3, 1 / 3), 7, 7, 20, 8, seed=8)
    if cfg == "bin10":
        return recipe_synthetic(np.full((2, 2), .5), np.full(2, .5), 10, 10, 20, 8, seed=4)
    if cfg == "bin3":  # a shallow tree: one tier
        return recipe_synthetic(np.full((2, 2), .5), np.full(2, .5), 3, 3, 20, 8, seed=5)
    return recipe_config(int(cfg[1:]))


TIERS = {"RAOCP_DR": "0", "RAOCP_DYN_SPLIT": "0"}


def _project(cache, r, zz):
    cache.cache_initial_state(r["x0"])
    cache.native.set_primal(zz)
    cache.native.project_on_dynamics()
    return cache.native.get_primal()


# (tree, forced cut list): the planner's own plan and the resident plans of other depths
# (config 2: [0,6)+[6,12) runs the LMAX = 6 build, the rest the LMAX = 4 one)
CASES = [("c2", None), ("c2", "4,8"), ("c2", "6"), ("c2", "3,7"), ("quad", None), ("quad", "2"), ("quad", "3"),
         ("tri", None), ("tri", "3"), ("tri", "4"), ("bin10", None), ("bin10", "4,8"), ("bin10", "6"),
         ("bin10", "3,7"), ("bin3", None)]


@pytest.mark.parametrize("cfg,cuts", CASES)
def test_dr_projection_matches_oracle_and_tiers(cfg, cuts):
    from oracle.raocp_oracle import OracleProblem
    r = _recipe(cfg)
    tree, prob = build_problem(r)
    env = {"RAOCP_DR_CUTS": cuts} if cuts else {}
    dr = _with_env(env, lambda: core.Cache(prob))
    assert dr.native.kernel_info(9) == "k_dr<20, 8> x1"
    tiers = _with_env(TIERS, lambda: core.Cache(prob))
    assert "k_dr_" not in tiers.native.kernel_info(9)
    zz = np.random.default_rng(5).standard_normal(dr.primal_size)
    z1 = _project(dr, r, zz)
    z2 = _project(tiers, r, zz)
    assert rel_err(z1, z2) <= 1e-13
    orc = OracleProblem(prob)
    assert rel_err(z1, orc.project_on_dynamics(zz, r["x0"])) <= 1e-12
    X = z1[orc.X0:orc.U0].reshape(orc.n, orc.nx)
    U = z1[orc.U0:orc.Y0].reshape(orc.m, orc.nu)
    j = np.arange(1, orc.n)
    pred = np.einsum("jab,jb->ja", np.stack(orc.A)[orc.iA[j]], X[orc.anc[j]]) + \
        np.einsum("jab,jb->ja", np.stack(orc.B)[orc.iB[j]], U[orc.anc[j]])
    assert np.max(np.abs(X[j] - pred)) <= 1e-12 * max(1.0, np.max(np.abs(X)))
    assert np.array_equal(X[0], np.asarray(r["x0"], float))
    # everything outside (x, u) untouched
    assert np.array_equal(z1[orc.Y0:], zz[orc.Y0:])


def test_dr_invalid_cut_list_is_rejected():
    """A forced plan whose grid cannot be resident (config 2 cut at stage 2: a 10-level
    deepest tier) is refused at context creation, naming the switch."""
    tree, prob = build_problem(recipe_config(2))
    with pytest.raises(Exception, match="RAOCP_DR_CUTS"):
        _with_env({"RAOCP_DR_CUTS": "2"}, lambda: core.Cache(prob))


@pytest.mark.parametrize("drc", ["1", "0"])
def test_dr_cp_loop_matches_tiers_and_oracle(drc):
    """30 CP iterations (a full 24-iteration graph batch plus a remainder; the deferred
    stopping test rides on k_dr), tol = 0; the loop's launch k_drc (k_dr with the CP families
    fused) and the pair k_dr + k_cp6 (RAOCP_DRC=0)."""
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(2)
    tree, prob = build_problem(r)
    dr = _with_env({"RAOCP_DRC": drc}, lambda: core.Cache(prob))
    assert dr.native.kernel_info(11) == ("k_drc<20, 8, 2>" if drc == "1" else "")
    tiers = _with_env(TIERS, lambda: core.Cache(prob))
    assert dr.native.kernel_info(9).startswith("k_dr<")
    alpha = 0.999 / dr.native.step_size()
    out = []
    for cache in (dr, tiers):
        st, err, derr = cache.native.cp_run(r["x0"], 30, 0.0, alpha)
        out.append((st, err, derr, cache.get_primal_flat(), cache.get_dual_flat()))
    (s1, e1, d1, z1, y1), (s2, e2, d2, z2, y2) = out
    assert s1 == s2 == 1 and e1.shape == e2.shape == (31, 3)
    assert trace_rel_err(e1, e2) <= 1e-10 and trace_rel_err(d1, d2) <= 1e-10
    assert rel_err(z1, z2) <= 1e-11 and rel_err(y1, y2) <= 1e-11
    st_o, err_o, _, z_o, _, _ = OracleProblem(prob).chock(r["x0"], 30, 0.0, alpha=alpha)
    assert trace_rel_err(e1, err_o) <= 1e-8 and rel_err(z1, z_o) <= 1e-10


@pytest.mark.parametrize("drc", ["1", "0"])
@pytest.mark.parametrize("iters,stop", [(1, None), (24, None), (30, None), (60, True)])
def test_dr_deferred_stopping_test_matches_eager(iters, stop, drc):
    """The deferred stopping test (an extra workgroup of k_dr / k_drc) against k_cp_check
    after every iteration (RAOCP_DEFER_CHECK=0): bit for bit, early stops included."""
    r = recipe_config(2)
    tree, prob = build_problem(r)
    dfr = _with_env({"RAOCP_DRC": drc}, lambda: core.Cache(prob))
    eag = _with_env({"RAOCP_DEFER_CHECK": "0", "RAOCP_DRC": drc}, lambda: core.Cache(prob))
    assert dfr.native.kernel_info(9).startswith("k_dr<")
    alpha = 0.999 / dfr.native.step_size()
    tol = 0.0
    if stop:
        _, err, _ = eag.native.cp_run(r["x0"], iters, 0.0, alpha)
        tol = float(err[37].max())
    out = []
    for cache in (dfr, eag):
        status, err, derr = cache.native.cp_run(r["x0"], iters, tol, alpha)
        out.append((status, err, derr, cache.get_primal_flat(), cache.get_dual_flat()))
    for u, v in zip(out[0], out[1]):
        assert np.array_equal(u, v)
    if stop:
        assert out[0][0] == 0 and out[0][1].shape[0] <= 38


def test_dr_many_launches_then_projection():
    """1,000 back-to-back launches: the tag advances inside the kernel (the top stores it when
    every workgroup has read it); a projection afterwards is the same bit for bit."""
    r = recipe_config(2)
    tree, prob = build_problem(r)
    dr = core.Cache(prob)
    zz = np.random.default_rng(9).standard_normal(dr.primal_size)
    out = []
    for rep in range(2):
        out.append(_project(dr, r, zz))
        dr.native.op_bench(9, 1000)
    assert np.array_equal(out[0], out[1])


def test_dr_forced_timeout_is_reported_quickly():
    """RAOCP_DR_FAULT=1: the deepest tier's first subtree never publishes its q row, so its
    parent's wait times out (RAOCP_FUSE_TIMEOUT_MS=5), sets the error word and leaves, and the
    waits on that parent time out in turn; the projection raises within a fraction of a
    second, the host clears the words and the granules, and the next projection raises the
    same way (not a 1 s wait per tier)."""
    r = recipe_config(2)
    tree, prob = build_problem(r)
    bad = _with_env({"RAOCP_DR_FAULT": "1", "RAOCP_FUSE_TIMEOUT_MS": "5"}, lambda: core.Cache(prob))
    zz = np.random.default_rng(3).standard_normal(bad.primal_size)
    for _ in range(2):
        t0 = time.perf_counter()
        with pytest.raises(Exception, match="timed out"):
            _project(bad, r, zz)
        assert time.perf_counter() - t0 < 0.5
    # a healthy context on the same device is unaffected
    good = core.Cache(prob)
    assert rel_err(_project(good, r, zz), _project(_with_env(TIERS, lambda: core.Cache(prob)), r, zz)) <= 1e-13


def test_drc_forced_timeout_in_the_cp_loop_is_reported():
    """RAOCP_DR_FAULT=1 in the fused CP loop (k_drc): the hand-off wait times out, every later
    launch of the batch leaves at its start (the error word), and cp_run raises within a
    fraction of a second per batch; a healthy context afterwards runs normally."""
    r = recipe_config(2)
    tree, prob = build_problem(r)
    bad = _with_env({"RAOCP_DR_FAULT": "1", "RAOCP_FUSE_TIMEOUT_MS": "5"}, lambda: core.Cache(prob))
    assert bad.native.kernel_info(11) == "k_drc<20, 8, 2>"
    alpha = 0.999 / bad.native.step_size()
    t0 = time.perf_counter()
    with pytest.raises(Exception, match="timed out"):
        bad.native.cp_run(r["x0"], 10, 0.0, alpha)
    assert time.perf_counter() - t0 < 1.0
    good = core.Cache(prob)
    st, err, _ = good.native.cp_run(r["x0"], 10, 0.0, alpha)
    assert st == 1 and err.shape == (11, 3) and np.all(np.isfinite(err))
