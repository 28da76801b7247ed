"""GPU parity of k_drc (raocp_dynr.hip): the regular-tree dynamics sweep k_dr
(cache.py:259-288) with each subtree workgroup's CP families fused behind its forward sweep
(k_cp6's entry arithmetic; solver.py:27-95, cache.py:248-393), one launch per CP iteration.
The default of the config-2 loop (binary fp64 trees at nx = 20, nu = 8 whose dynamics plan has
4 levels in every tier and whose nodes are all boxed or all unboxed); RAOCP_DRC=0 keeps the
pair k_dr + k_cp6.

The fused launch runs the same entry arithmetic as k_cp6 on the same inputs (the projected
x+, u+ read from LDS instead of global memory), so the two loops agree at rounding level:
1e-12 per residual trace entry and on the iterate over 30 iterations (a graph batch boundary at
24 inside). Against the oracle: 1e-8 per trace entry (BASELINE.json north_star), 1e-10 on the
iterate. The stopping test of iteration k runs in launch k + 1 beside that iteration's CP step,
so the residual rows alternate between two sets and a NaN in a box raises the flag of its own
iteration's parity: status, iteration count, history and final iterate are those of the
eager test (checked against RAOCP_DEFER_CHECK=0 and eager launches, bit for bit).
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


# (recipe, forced tier cuts or None)
def _case(case):
    if case in ("c2", "c2-nobox"):
        r = recipe_config(2)
        if case == "c2-nobox":
            r["nl_min"] = r["nl_max"] = r["l_min"] = r["l_max"] = None
        return r, None
    if case == "bin8":  # 511 nodes, two tiers [0,4) + [4,8)
        return recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 8, 8, 20, 8, seed=21), "4"
    if case == "bin4":  # 31 nodes, the top alone (no hand-offs)
        return recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 4, 4, 20, 8, seed=22), ""
    if case == "markov8":  # 2 modes with their own dynamics, 511 nodes
        P = np.array([[.7, .3], [.2, .8]])
        return recipe_synthetic(P, np.array([.4, .6]), 8, 8, 20, 8, seed=23), "4"
    if case == "a95":  # AVaR alpha 0.95, 8,191 nodes
        return recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 12, 12, 20, 8, seed=24, alpha_r=0.95), None
    raise ValueError(case)


def _caches(case, extra_off=None):
    r, cuts = _case(case)
    tree, prob = build_problem(r)
    env = {} if cuts is None else {"RAOCP_DR_CUTS": cuts}
    on = _with_env(env, lambda: core.Cache(prob))
    off = _with_env(dict(env, RAOCP_DRC="0", **(extra_off or {})), lambda: core.Cache(prob))
    return r, prob, on, off


def _run(cache, x0, K, alpha, tol=0.0, warm=False):
    st, err, derr = cache.native.cp_run(x0, K, tol, alpha, warm=warm)
    return st, err, derr, cache.get_primal_flat(), cache.get_dual_flat()


def _close(a, b, tol=1e-12):
    assert a[0] == b[0] and a[1].shape == b[1].shape
    assert trace_rel_err(a[1], b[1]) <= tol and trace_rel_err(a[2], b[2]) <= tol
    assert rel_err(a[3], b[3]) <= tol and rel_err(a[4], b[4]) <= tol


@pytest.mark.parametrize("case", ["c2", "c2-nobox", "bin8", "bin4", "markov8", "a95"])
def test_drc_matches_dr_cp6_and_oracle(case):
    from oracle.raocp_oracle import OracleProblem
    r, prob, on, off = _caches(case)
    assert on.native.kernel_info(11) == "k_drc<20, 8, 2>"
    assert off.native.kernel_info(11) == ""
    assert off.native.kernel_info(10) == "k_cp6<double, 20, 8, 2>"
    alpha = 0.999 / on.native.step_size()
    K = 30
    a = _run(on, r["x0"], K, alpha)
    b = _run(off, r["x0"], K, alpha)
    assert a[0] == 1 and a[1].shape == (K + 1, 3)
    _close(a, b)
    st_o, err_o, derr_o, z_o, e_o, _ = OracleProblem(prob).chock(r["x0"], K, 0.0, alpha=alpha)
    assert st_o == 1
    assert trace_rel_err(a[1], err_o) <= 1e-8 and trace_rel_err(a[2], derr_o) <= 1e-8
    assert rel_err(a[3], z_o) <= 1e-10 and rel_err(a[4], e_o) <= 1e-10


def test_drc_off_where_a_tier_is_not_four_levels():
    """A plan with a tier of another depth (N = 9) keeps k_dr + k_cp6."""
    r = recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 9, 9, 20, 8, seed=25)
    tree, prob = build_problem(r)
    c = core.Cache(prob)
    assert c.native.kernel_info(11) == ""
    assert c.native.kernel_info(10) == "k_cp6<double, 20, 8, 2>"


@pytest.mark.parametrize("k_stop", [5, 23, 24, 25, 41])
def test_drc_early_stop_matches_pair(k_stop):
    """tol = a residual of the pair's loop (clear of rounding): both stop at the same iteration
    (inside a graph batch, at its last iteration and at the next batch's first) with the same
    history and iterate."""
    r, prob, on, off = _caches("c2")
    alpha = 0.999 / on.native.step_size()
    _, err, _ = off.native.cp_run(r["x0"], 60, 0.0, alpha)
    # the first iteration whose max residual is below tol is k_stop, provided the trace decreases there
    tol = float(err[k_stop].max()) * (1 + 1e-9)
    first = int(np.argmax(err.max(axis=1) <= tol))
    a = _run(on, r["x0"], 60, alpha, tol)
    b = _run(off, r["x0"], 60, alpha, tol)
    assert a[0] == b[0] == 0 and a[1].shape == b[1].shape == (first + 1, 3)
    _close(a, b)


@pytest.mark.parametrize("env", [{"RAOCP_DEFER_CHECK": "0"}, {"RAOCP_EAGER": "1"}])
def test_drc_launch_forms_bit_identical(env):
    """The stopping test after every launch (no deferral) and eager launches (no graphs) run the
    same kernels on the same buffers: bit-identical to the default graph-replayed loop, also
    for an early stop inside a batch."""
    r, prob, on, _ = _caches("c2")
    other = _with_env(env, lambda: core.Cache(prob))
    assert other.native.kernel_info(11) == "k_drc<20, 8, 2>"
    alpha = 0.999 / on.native.step_size()
    _, err, _ = on.native.cp_run(r["x0"], 40, 0.0, alpha)
    for tol in (0.0, float(err[17].max()) * (1 + 1e-9)):
        a = _run(on, r["x0"], 40, alpha, tol)
        b = _run(other, r["x0"], 40, alpha, tol)
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


def test_drc_warm_start_matches_pair():
    """Two chock calls on one solver (the second continues from the first's iterate,
    solver.py:124-131 with cache.py:58-66): the fused loop equals the pair's."""
    r, prob, on, off = _caches("c2")
    alpha = 0.999 / on.native.step_size()
    x1 = np.asarray(r["x0"], dtype=float) / 2
    for c in (on, off):
        c.native.cp_run(r["x0"], 20, 0.0, alpha)
    a = _run(on, x1, 13, alpha, warm=True)
    b = _run(off, x1, 13, alpha, warm=True)
    _close(a, b)


@pytest.mark.parametrize("K", [0, 1, 2])
def test_drc_short_runs_match_pair(K):
    """max_iters 0 / 1 / 2: one to three iterations, the 1-D history of a single iteration."""
    r, prob, on, off = _caches("c2")
    alpha = 0.999 / on.native.step_size()
    a = _run(on, r["x0"], K, alpha)
    b = _run(off, r["x0"], K, alpha)
    _close(a, b)


def test_drc_nan_in_box_raises():
    """A NaN reaching a box projection (Rectangle._constrain, rectangle.py:50-59) raises
    ValueError through the fused launch as through the reference."""
    r, prob, on, _ = _caches("c2")
    x0 = np.array(r["x0"], dtype=float)
    x0[3] = np.nan
    alpha = 0.999 / on.native.step_size()
    with pytest.raises(ValueError):
        on.native.cp_run(x0, 5, 0.0, alpha)
    # the context stays usable: a clean run afterwards equals a fresh one's
    a = _run(on, r["x0"], 8, alpha)
    fresh = _caches("c2")[2]
    b = _run(fresh, r["x0"], 8, alpha)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


def test_drc_bench_loop_matches_cp_run():
    """The benchmark's exact-K graphs (24-iteration batches and a remainder) leave the iterate
    the stopping-test loop leaves after the same K iterations."""
    r, prob, on, _ = _caches("c2")
    alpha = 0.999 / on.native.step_size()
    K = 50
    on.native.cp_bench(r["x0"], K, alpha)
    z_b = on.get_primal_flat()
    st, err, _ = on.native.cp_run(r["x0"], K - 1, 0.0, alpha)
    assert st == 1 and err.shape[0] == K
    assert np.array_equal(z_b, on.get_primal_flat())


def test_drc_two_contexts_in_threads():
    """One active context per device: k_drc needs its whole grid resident, so the entry points
    that launch it hold a per-device lock (raocp_capi.hip SweepLock). Two threads solving on two
    contexts of one device at once finish, each with the result of a solve alone."""
    import threading
    r, prob, on, _ = _caches("c2")
    other = core.Cache(prob)
    alpha = 0.999 / on.native.step_size()
    ref = _run(on, r["x0"], 40, alpha)
    res, errs = {}, []

    def work(name, cache):
        try:
            for _ in range(3):
                res[name] = _run(cache, r["x0"], 40, alpha)
        except Exception as e:  # reported by the main thread
            errs.append(e)

    th = [threading.Thread(target=work, args=(k, c)) for k, c in (("a", on), ("b", other))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs and not any(t.is_alive() for t in th)
    for name in ("a", "b"):
        for u, v in zip(res[name], ref):
            assert np.array_equal(u, v)
