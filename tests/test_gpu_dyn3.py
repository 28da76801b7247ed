"""GPU parity of the per-stage streaming dynamics sweep k_dy3_back / k_dy3_fwd
(raocp_dyn3.hip: one launch per stage and direction, the children's products accumulated
per parent in MFMA registers; cache.py:259-288). It is the default of fp32 contexts and of
fp64 trees of >= 64k nodes with one branching factor whose child slots keep their (A, B)
pair across a stage (configs 4, 5; config 2 in fp32), and an fp64 opt-in (RAOCP_DYN3=1) on
smaller trees next to the tiered kernels (RAOCP_DYN3=0 forces the tiers).

Tolerances: the projection against the oracle within 1e-12 of the largest entry (fp64) and
exact feasibility x_j = A_j x_i + B_j u_i of its output to 1e-12; the CP loop against the
tiered fp64 path within 1e-10 per trace entry (the same arithmetic, other summation order)
and the oracle within 1e-8; the deferred stopping test bit-identical to the eager one.
"""
import os

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
    if cfg == "chain":
        return recipe_synthetic(np.ones((1, 1)), np.ones(1), 30, 30, 20, 8, seed=3)
    if cfg == "quad":
        return recipe_synthetic(np.full((4, 4), .25), np.full(4, .25), 5, 5, 20, 8, seed=6)
    return recipe_config(int(cfg[1:]))


@pytest.mark.parametrize("cfg", ["c2", "c4", "chain", "quad"])
def test_dyn3_projection_vs_oracle(cfg):
    from oracle.raocp_oracle import OracleProblem
    r = _recipe(cfg)
    tree, prob = build_problem(r)
    cache = _with_env({"RAOCP_DYN3": "1"}, lambda: core.Cache(prob))
    assert cache.native.kernel_info(9).startswith("k_dy3_back<double")
    orc = OracleProblem(prob)
    rng = np.random.default_rng(23)
    zz = rng.standard_normal(cache.primal_size)
    cache.cache_initial_state(r["x0"])
    cache.native.set_primal(zz)
    cache.native.project_on_dynamics()
    z1 = cache.native.get_primal()
    assert rel_err(z1, orc.project_on_dynamics(zz, r["x0"])) <= 1e-12
    X = z1[orc.X0:orc.U0].reshape(orc.n, orc.nx)
    U = z1[orc.U0:orc.Y0].reshape(orc.m, orc.nu)
    j = np.arange(1, orc.n, 7)
    pred = np.stack([orc.A[orc.iA[k]] @ X[orc.anc[k]] + orc.B[orc.iB[k]] @ U[orc.anc[k]] for k in j])
    assert np.max(np.abs(X[j] - pred)) <= 1e-12 * max(1.0, np.max(np.abs(X)))
    assert np.array_equal(X[0], np.asarray(r["x0"], float))


@pytest.mark.parametrize("cfg", ["c2", "c4"])
def test_dyn3_cp_loop_matches_tiers_and_oracle(cfg):
    from oracle.raocp_oracle import OracleProblem
    r = _recipe(cfg)
    tree, prob = build_problem(r)
    d3 = _with_env({"RAOCP_DYN3": "1"}, lambda: core.Cache(prob))
    tiers = _with_env({"RAOCP_DYN3": "0"}, lambda: core.Cache(prob))
    assert not tiers.native.kernel_info(9).startswith("k_dy3")
    alpha = 0.999 / tiers.native.step_size()
    K = 12 if cfg == "c4" else 20
    out = []
    for cache in (d3, tiers):
        st, err, derr = cache.native.cp_run(r["x0"], K, 0.0, alpha)
        out.append((st, err, derr, cache.get_primal_flat(), cache.get_dual_flat()))
    (s1, e1, d1, z1, y1), (s2, e2, d2, z2, y2) = out
    assert s1 == s2 == 1 and e1.shape == e2.shape == (K + 1, 3)
    assert trace_rel_err(e1, e2) <= 1e-10 and trace_rel_err(d1, d2) <= 1e-10
    assert rel_err(z1, z2) <= 1e-11 and rel_err(y1, y2) <= 1e-11
    st_o, err_o, derr_o, z_o, e_o, _ = OracleProblem(prob).chock(r["x0"], K, 0.0, alpha=alpha)
    assert trace_rel_err(e1, err_o) <= 1e-8 and rel_err(z1, z_o) <= 1e-10


@pytest.mark.parametrize("iters,stop", [(1, None), (24, None), (30, None), (60, True)])
def test_dyn3_deferred_stopping_test_matches_eager(iters, stop):
    """The deferred stopping test rides on the first k_dy3_back launch of the next iteration;
    against k_cp_check after every iteration (RAOCP_DEFER_CHECK=0): bit for bit."""
    r = recipe_config(2)
    tree, prob = build_problem(r)
    dfr = _with_env({"RAOCP_DYN3": "1"}, lambda: core.Cache(prob))
    eag = _with_env({"RAOCP_DYN3": "1", "RAOCP_DEFER_CHECK": "0"}, lambda: core.Cache(prob))
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


def test_kernel_info_lists_the_projection_launches():
    """raocp_kernel_info(9) names every launch of one projection as "name xcount" terms
    (bench.py sums their PMC traffic): the regular-tree sweep (one k_dr) at config 2; with
    RAOCP_DR=0 the tier launches (2 tiers + the top: the split sweep's grid of 274
    workgroups is not co-resident there), the same with RAOCP_DYN_SPLIT=0, one k_dy3_back and
    one k_dy3_fwd per nonleaf stage with RAOCP_DYN3=1; the split sweep (k_dyn_up + k_dyn_down)
    on a co-resident tree of a size k_dr does not take (nx = 32, nu = 12, 3,280 nodes)."""
    import re
    r = recipe_config(2)
    prob = build_problem(r)[1]
    off = {"RAOCP_DR": "0"}
    t32 = build_problem(recipe_synthetic(np.full((3, 3), 1 / 3), np.full(3, 1 / 3), 7, 7, 32, 12, seed=7))[1]
    for env, want, pb in (({}, "dr", prob), (off, None, prob), ({**off, "RAOCP_DYN_SPLIT": "0"}, None, prob),
                          ({"RAOCP_DYN3": "1"}, "dy3", prob), ({}, "split", t32)):
        cache = _with_env(env, lambda: core.Cache(pb))
        terms = [re.fullmatch(r"(k_\w+<[^>]*>) x(\d+)", t) for t in cache.native.kernel_info(9).split(" + ")]
        assert all(terms), cache.native.kernel_info(9)
        cnt = {m.group(1).split("<")[0]: int(m.group(2)) for m in terms}
        if want == "dy3":  # the 8 top stages (<= 8 tiles each) in one workgroup per direction
            assert cnt == {"k_dy3_back": 4, "k_dy3_top_back": 1, "k_dy3_top_fwd": 1, "k_dy3_fwd": 4}
        elif want == "dr":
            assert cnt == {"k_dr": 1}
        elif want == "split":
            assert cnt == {"k_dyn_up": 1, "k_dyn_down": 1}
        else:
            assert cnt["k_dyn_top"] == 1 and cnt["k_dyn_bottom_back"] == cnt["k_dyn_bottom_fwd"] >= 1


@pytest.mark.parametrize("cfg,dtype", [(4, "float64"), (2, "float64"), (5, "float32")])
def test_top_stages_in_one_workgroup_bit_identical(cfg, dtype):
    """k_dy3_top_back / k_dy3_top_fwd (the top stages back to back in one workgroup, the
    child-slot tables kept in LDS across stages) sum the child slots in the order of the
    slot-parallel per-stage launches they replace (RAOCP_DY3_TOP=0): the projection and a
    12-iteration CP loop are bit-identical (stage 3 of configs 4 and 5 takes two rounds)."""
    r = recipe_config(cfg)
    prob = build_problem(r)[1]
    env = {"RAOCP_DYN3": "1"} if cfg == 2 else {}
    top = _with_env(env, lambda: core.Cache(prob, dtype=dtype))
    per = _with_env({**env, "RAOCP_DY3_TOP": "0"}, lambda: core.Cache(prob, dtype=dtype))
    assert "k_dy3_top_back" in top.native.kernel_info(9) and "k_dy3_top" not in per.native.kernel_info(9)
    zz = np.random.default_rng(21).standard_normal(top.primal_size)
    out = []
    for cache in (top, per):
        cache.cache_initial_state(r["x0"])
        cache.native.set_primal(zz)
        cache.native.project_on_dynamics()
        out.append(cache.native.get_primal())
    assert np.array_equal(out[0], out[1])
    alpha = 0.999 / top.native.step_size(rtol=1e-7 if dtype == "float32" else 1e-14)
    runs = []
    for cache in (top, per):
        st, err, derr = cache.native.cp_run(r["x0"], 12, 0.0, alpha)
        runs.append((st, err, derr, cache.get_primal_flat()))
    for u, v in zip(runs[0], runs[1]):
        assert np.array_equal(u, v)
