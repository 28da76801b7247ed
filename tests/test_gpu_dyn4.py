"""GPU parity of k_dy4 (raocp_dyn4.hip): the dynamics projection (cache.py:259-288) of the
regular trees k_dy3 takes, in ONE launch of dataflow tile tasks (a backward tile waits for its
C child tiles' flags, the top task for every tile of the first wide stage, a forward tile for
its parents' tile). Opt-in (RAOCP_DY4=1) wherever the per-stage sweep k_dy3 applies (configs
4, 5; fp64 trees of >= 64k nodes and fp32 contexts with one branching factor): measured slower
than k_dy3's per-stage launches, kept as the tested one-launch form.

Tolerances: the projection against the oracle within 1e-12 of the largest entry (fp64; fp32
2e-5 against the fp64 oracle) and exact feasibility of its output; against k_dy3's per-stage
launches 1e-12 (the slot sums of k_dy3's wide stages accumulate in the MFMA registers, k_dy4
sums them through LDS in slot order); the CP loop against the oracle within 1e-8 per residual
trace entry. Task scheduling changes no arithmetic: other grids and other top cuts reproduce
the default bit for bit.
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


def _recipe(case):
    if case == "t32":  # C = 3 at 32 / 12 (config 4's sizes), 3,280 nodes
        return recipe_synthetic(np.full((3, 3), 1 / 3), np.full(3, 1 / 3), 7, 7, 32, 12, seed=4)
    if case == "q20":  # C = 4 at 20 / 8, 5,461 nodes
        return recipe_synthetic(np.full((4, 4), .25), np.full(4, .25), 6, 6, 20, 8, seed=6)
    if case == "b20":  # C = 2 at 20 / 8, 2,047 nodes
        return recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 10, 10, 20, 8, seed=8)
    if case == "q64":  # C = 4 at 64 / 16 (config 5's sizes), 1,365 nodes
        return recipe_synthetic(np.full((4, 4), .25), np.full(4, .25), 5, 5, 64, 16, seed=7)
    return recipe_config(int(case[1:]))


def _dtype(case):
    return "float32" if case in ("q64", "c5") else "float64"


def _cache(prob, dtype, env=None):
    # fp64 trees below 64k nodes keep the tiers by default: RAOCP_DYN3=1 selects the sweep;
    # RAOCP_DY4=1 its one-launch form (RAOCP_DY4=0: the per-stage launches)
    env = {"RAOCP_DYN3": "1", "RAOCP_DY4": "1", **(env or {})}
    return _with_env(env, lambda: core.Cache(prob, dtype=dtype))


def _project(cache, r, zz):
    cache.cache_initial_state(r["x0"])
    cache.native.set_primal(zz)
    cache.native.project_on_dynamics()
    return cache.native.get_primal()


@pytest.mark.parametrize("case", ["t32", "q20", "b20", "q64", "c4", "c5"])
def test_dy4_projection_vs_oracle_and_dy3(case):
    from oracle.raocp_oracle import OracleProblem
    r = _recipe(case)
    tree, prob = build_problem(r)
    dt = _dtype(case)
    a = _cache(prob, dt)
    b = _cache(prob, dt, {"RAOCP_DY4": "0"})
    assert a.native.kernel_info(9).startswith("k_dy4<")
    assert b.native.kernel_info(9).startswith("k_dy3_back<")
    orc = OracleProblem(prob)
    zz = np.random.default_rng(29).standard_normal(a.primal_size)
    z1 = _project(a, r, zz)
    z2 = _project(b, r, zz)
    tol = 2e-5 if dt == "float32" else 1e-12
    assert rel_err(z1, z2) <= (1e-6 if dt == "float32" else 1e-12)
    assert rel_err(z1, orc.project_on_dynamics(zz, r["x0"])) <= tol
    X = z1[orc.X0:orc.U0].reshape(orc.n, orc.nx)
    U = z1[orc.U0:orc.Y0].reshape(orc.m, orc.nu)
    j = np.arange(1, orc.n, max(1, orc.n // 400))
    pred = np.stack([orc.A[orc.iA[k]] @ X[orc.anc[k]] + orc.B[orc.iB[k]] @ U[orc.anc[k]] for k in j])
    assert np.max(np.abs(X[j] - pred)) <= (1e-5 if dt == "float32" else 1e-12) * max(1.0, np.max(np.abs(X)))
    assert np.allclose(X[0], np.asarray(r["x0"], float), rtol=0, atol=1e-6 if dt == "float32" else 0)


@pytest.mark.parametrize("case,env", [("t32", {"RAOCP_DY4_GRID": "1"}), ("t32", {"RAOCP_DY4_GRID": "7"}),
                                      ("t32", {"RAOCP_DY4_TS": "1"}), ("t32", {"RAOCP_DY4_TS": "5"}),
                                      ("c4", {"RAOCP_DY4_GRID": "37"}), ("q64", {"RAOCP_DY4_TS": "2"})],
                         ids=["grid1", "grid7", "top1", "top5", "c4-grid37", "q64-top2"])
def test_dy4_schedule_bit_identical(case, env):
    """Fewer workgroups (every workgroup walking many tasks) and other top cuts move tiles
    between workgroups only: the projection and a CP loop are bit-identical."""
    r = _recipe(case)
    tree, prob = build_problem(r)
    dt = _dtype(case)
    a = _cache(prob, dt)
    b = _cache(prob, dt, env)
    zz = np.random.default_rng(31).standard_normal(a.primal_size)
    assert np.array_equal(_project(a, r, zz), _project(b, r, zz))
    alpha = 0.999 / a.native.step_size(rtol=1e-7 if dt == "float32" else 1e-14)
    ra = a.native.cp_run(r["x0"], 8, 0.0, alpha)
    rb = b.native.cp_run(r["x0"], 8, 0.0, alpha)
    for u, v in zip(ra, rb):
        assert np.array_equal(u, v)
    assert np.array_equal(a.get_primal_flat(), b.get_primal_flat())


@pytest.mark.parametrize("case", ["t32", "c4"])
def test_dy4_cp_loop_vs_oracle(case):
    """The CP loop on k_dy4 (30 iterations: a graph batch boundary and the deferred stopping
    test riding on k_dy4's extra workgroup) against the oracle."""
    from oracle.raocp_oracle import OracleProblem
    r = _recipe(case)
    tree, prob = build_problem(r)
    a = _cache(prob, "float64")
    alpha = 0.999 / a.native.step_size()
    K = 30 if case == "t32" else 12
    st, err, derr = a.native.cp_run(r["x0"], K, 0.0, alpha)
    st_o, err_o, derr_o, z_o, e_o, _ = OracleProblem(prob).chock(r["x0"], K, 0.0, alpha=alpha)
    assert st == st_o == 1
    assert trace_rel_err(err, err_o) <= 1e-8 and trace_rel_err(derr, derr_o) <= 1e-8
    assert rel_err(a.get_primal_flat(), z_o) <= 1e-10


def test_dy4_deferred_stopping_test_matches_eager():
    r = _recipe("t32")
    tree, prob = build_problem(r)
    dfr = _cache(prob, "float64")
    eag = _cache(prob, "float64", {"RAOCP_DEFER_CHECK": "0"})
    alpha = 0.999 / dfr.native.step_size()
    _, err, _ = eag.native.cp_run(r["x0"], 40, 0.0, alpha)
    mx = err.max(axis=1)
    tol = float(np.sqrt(mx[0] * mx[1]))
    out = []
    for cache in (dfr, eag):
        st, err, derr = cache.native.cp_run(r["x0"], 40, tol, alpha)
        out.append((st, err, derr, cache.get_primal_flat()))
    for u, v in zip(out[0], out[1]):
        assert np.array_equal(u, v)


def test_dy4_forced_timeout_is_reported_quickly():
    """RAOCP_DY4_FAULT=1: the first deepest tile never releases its flag, so its parent's wait
    times out (RAOCP_FUSE_TIMEOUT_MS=50): the call fails with the state error within a second,
    and a new context runs normally afterwards."""
    r = _recipe("t32")
    tree, prob = build_problem(r)
    bad = _cache(prob, "float64", {"RAOCP_DY4_FAULT": "1", "RAOCP_FUSE_TIMEOUT_MS": "50"})
    zz = np.random.default_rng(3).standard_normal(bad.primal_size)
    bad.cache_initial_state(r["x0"])
    bad.native.set_primal(zz)
    t0 = time.time()
    with pytest.raises(Exception):
        bad.native.project_on_dynamics()
    assert time.time() - t0 < 2.0
    good = _cache(prob, "float64")
    from oracle.raocp_oracle import OracleProblem
    z1 = _project(good, r, zz)
    assert rel_err(z1, OracleProblem(prob).project_on_dynamics(zz, r["x0"])) <= 1e-12


@pytest.mark.parametrize("case,wide", [("t32", "2"), ("q64", "1"), ("c4", "1000")])
def test_dy4_wide_stage_form_vs_oracle(case, wide):
    """The task form of a stage (RAOCP_DY4_WIDE: 4 tiles per task with the slot sums in the
    MFMA registers from that many tiles up, else a tile per task with the slot sums through
    LDS) changes the summation order only: the projection equals the default form to 1e-12
    (fp32: 1e-6) and the oracle to 1e-12 (fp32: 2e-5)."""
    from oracle.raocp_oracle import OracleProblem
    r = _recipe(case)
    tree, prob = build_problem(r)
    dt = _dtype(case)
    a = _cache(prob, dt)
    b = _cache(prob, dt, {"RAOCP_DY4_WIDE": wide})
    zz = np.random.default_rng(37).standard_normal(a.primal_size)
    z1 = _project(a, r, zz)
    z2 = _project(b, r, zz)
    f32 = dt == "float32"
    assert rel_err(z1, z2) <= (1e-6 if f32 else 1e-12)
    assert rel_err(z2, OracleProblem(prob).project_on_dynamics(zz, r["x0"])) <= (2e-5 if f32 else 1e-12)
