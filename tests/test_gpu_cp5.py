"""GPU parity of k_cp5 (raocp_cp5.hip): the fused CP iteration of k_cp3 (raocp_cp3.hip;
solver.py:27-95, cache.py:248-393) for the large uniform trees as two software-pipelined
launches -- k_cp5_leaf (eta2 and s of every nonleaf node; the leaf tiles: eta11..eta14, x_l
and s_l of the half step before the kernel projection), then k_cp5_fams (the family tiles, a
workgroup of C waves per tile, reading eta2+ and the children's s from the first launch). The default of configs 3 (fp64,
20 / 8, C = 4), 4 (fp64, 32 / 12, C = 3) and 5 (fp32, 64 / 16, C = 4) with all nodes boxed
or none; RAOCP_CP5=0 keeps k_cp3.

The arithmetic of every entry is k_cp3's; the L^T accumulators start from the box terms
(k_cp3 adds the leaf's eta14 after its sqrtPf' product) and the compiler contracts
multiply-adds by code shape, so the two kernels agree at rounding level: fp64 1e-12 per
residual trace entry and on the iterate, fp32 1e-4 per trace entry and 1e-5 on the iterate
(the fp32 drift bound of test_gpu_cp3.py). Against the oracle: 1e-8 per trace entry
(BASELINE.json north_star), 1e-10 on the iterate. The grid-stride loops (several tiles per
wave, the next tile's operands loaded during the current one's arithmetic) are checked by shrinking
the grids: the residual maxima are order-free and every entry's arithmetic is the tile's, so
a one-workgroup grid reproduces the default grid bit for bit.
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


def _recipe(case):
    """Small trees of the compiled (nx, nu, C) combinations (the oracle runs them in
    seconds) and the benchmark configs."""
    if case in ("q20", "q20-nobox"):  # C = 4 at 20 / 8 (config 3's sizes), 5,461 nodes
        r = recipe_synthetic(np.full((4, 4), .25), np.full(4, .25), 6, 6, 20, 8, seed=6)
        if case == "q20-nobox":
            r["nl_min"] = r["nl_max"] = r["l_min"] = r["l_max"] = None
        return r
    if case == "m20":  # Markov 4 modes at 20 / 8 (per-mode dynamics, one cost table)
        rng = np.random.default_rng(5)
        P = rng.random((4, 4)) + 0.1
        P /= P.sum(axis=1, keepdims=True)
        return recipe_synthetic(P, np.full(4, .25), 5, 5, 20, 8, seed=2)
    if case in ("t32", "t32-nobox"):  # C = 3 at 32 / 12 (config 4's sizes), 3,280 nodes
        r = recipe_synthetic(np.full((3, 3), 1 / 3), np.full(3, 1 / 3), 7, 7, 32, 12, seed=4)
        if case == "t32-nobox":
            r["nl_min"] = r["nl_max"] = r["l_min"] = r["l_max"] = None
        return r
    if case == "t32-a95":
        r = recipe_synthetic(np.full((3, 3), 1 / 3), np.full(3, 1 / 3), 6, 6, 32, 12, seed=9, alpha_r=0.95)
        return r
    if case == "q64":  # C = 4 at 64 / 16 (config 5's sizes), 1,365 nodes
        return recipe_synthetic(np.full((4, 4), .25), np.full(4, .25), 5, 5, 64, 16, seed=7)
    return recipe_config(int(case[1:]))


def _pair(prob, dtype=None, env=None):
    env = env or {}
    mk = (lambda: core.Cache(prob, dtype=dtype)) if dtype else (lambda: core.Cache(prob))
    c5 = _with_env(env, mk)
    c3 = _with_env({**env, "RAOCP_CP5": "0"}, mk)
    return c5, c3


def _run(cache, x0, K, alpha, tol=0.0):
    st, err, derr = cache.native.cp_run(x0, K, tol, alpha)
    return st, err, derr, cache.get_primal_flat(), cache.get_dual_flat()


@pytest.mark.parametrize("case", ["q20", "m20", "t32", "t32-nobox", "t32-a95"])
def test_cp5_matches_cp3_and_oracle_fp64(case):
    from oracle.raocp_oracle import OracleProblem
    r = _recipe(case)
    tree, prob = build_problem(r)
    c5, c3 = _pair(prob)
    assert c5.native.kernel_info(10).startswith("k_cp5_leaf<double")
    assert c3.native.kernel_info(10).startswith("k_cp3<double")
    alpha = 0.999 / c5.native.step_size()
    K = 30  # a graph batch boundary (24) inside
    a = _run(c5, r["x0"], K, alpha)
    b = _run(c3, r["x0"], K, alpha)
    assert a[0] == b[0] == 1 and a[1].shape == (K + 1, 3)
    assert trace_rel_err(a[1], b[1]) <= 1e-12 and trace_rel_err(a[2], b[2]) <= 1e-12
    assert rel_err(a[3], b[3]) <= 1e-12 and rel_err(a[4], b[4]) <= 1e-12
    st_o, err_o, derr_o, z_o, e_o, _ = OracleProblem(prob).chock(r["x0"], K, 0.0, alpha=alpha)
    assert st_o == 1
    assert trace_rel_err(a[1], err_o) <= 1e-8 and trace_rel_err(a[2], derr_o) <= 1e-8
    assert rel_err(a[3], z_o) <= 1e-10 and rel_err(a[4], e_o) <= 1e-10


def test_cp5_fp32_small_tree_vs_fp64_oracle():
    """C = 4 at 64 / 16 in fp32 (config 5's kernels on a 1,365-node tree): 20 iterations
    against the fp64 oracle (fp32 drift bound) and against k_cp3<float>."""
    from oracle.raocp_oracle import OracleProblem
    r = _recipe("q64")
    tree, prob = build_problem(r)
    c5, c3 = _pair(prob, "float32")
    assert c5.native.kernel_info(10).startswith("k_cp5_leaf<float, 64, 4>")
    alpha = 0.999 / c5.native.step_size(rtol=1e-7)
    K = 20
    a = _run(c5, r["x0"], K, alpha)
    b = _run(c3, r["x0"], K, alpha)
    assert a[0] == b[0] == 1
    assert trace_rel_err(a[1], b[1]) <= 1e-4 and trace_rel_err(a[2], b[2]) <= 1e-4
    assert rel_err(a[3], b[3]) <= 1e-5 and rel_err(a[4], b[4]) <= 1e-5
    st_o, err_o, derr_o, z_o, e_o, _ = OracleProblem(prob).chock(r["x0"], K, 0.0, alpha=alpha)
    assert trace_rel_err(a[1], err_o) <= 2e-3 and trace_rel_err(a[2], derr_o) <= 2e-3
    assert rel_err(a[3], z_o) <= 2e-4 and rel_err(a[4], e_o) <= 2e-4


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_cp5_full_size_matches_cp3(cfg):
    """Configs 3 and 4 at full size (87k / 89k nodes): 12 iterations of k_cp5 against k_cp3
    (the oracle at these sizes: test_gpu_parity.py test_large_cp_trace_vs_oracle)."""
    r = _recipe(cfg)
    tree, prob = build_problem(r)
    c5, c3 = _pair(prob)
    assert c5.native.kernel_info(10).startswith("k_cp5_leaf<double")
    alpha = 0.999 / c5.native.step_size()
    K = 12
    a = _run(c5, r["x0"], K, alpha)
    b = _run(c3, r["x0"], K, alpha)
    assert a[0] == b[0] == 1
    assert trace_rel_err(a[1], b[1]) <= 1e-12 and trace_rel_err(a[2], b[2]) <= 1e-12
    assert rel_err(a[3], b[3]) <= 1e-12 and rel_err(a[4], b[4]) <= 1e-12


def test_cp5_config5_fp32_matches_cp3():
    r = _recipe("c5")
    tree, prob = build_problem(r)
    c5, c3 = _pair(prob, "float32")
    assert c5.native.kernel_info(10).startswith("k_cp5_leaf<float, 64, 4> x1 + k_cp5_fam")
    alpha = 0.999 / c5.native.step_size(rtol=1e-7)
    K = 8
    a = _run(c5, r["x0"], K, alpha)
    b = _run(c3, r["x0"], K, alpha)
    assert a[0] == b[0] == 1
    assert trace_rel_err(a[1], b[1]) <= 1e-4 and trace_rel_err(a[2], b[2]) <= 1e-4
    assert rel_err(a[3], b[3]) <= 1e-5 and rel_err(a[4], b[4]) <= 1e-5


@pytest.mark.parametrize("case,grids", [("t32", ("1", "1")), ("t32", ("3", "2")), ("q20", ("1", "5")),
                                        ("c4", ("7", "13"))], ids=["t32-1-1", "t32-3-2", "q20-1-5", "c4-7-13"])
def test_cp5_small_grids_bit_identical(case, grids):
    """Grids of a few workgroups (every wave looping over many leaf tiles, every workgroup
    over many family tiles with the next tile's slot rows prefetched) reproduce the default
    grids bit for bit."""
    r = _recipe(case)
    tree, prob = build_problem(r)
    a = core.Cache(prob)
    b = _with_env({"RAOCP_CP5_LGRID": grids[0], "RAOCP_CP5_FGRID": grids[1]}, lambda: core.Cache(prob))
    alpha = 0.999 / a.native.step_size()
    ra = _run(a, r["x0"], 14, alpha)
    rb = _run(b, r["x0"], 14, alpha)
    for u, v in zip(ra, rb):
        assert np.array_equal(u, v)


@pytest.mark.parametrize("case", ["t32", "q20"])
def test_cp5_early_stop_matches_cp3(case):
    """A tolerance between the first two residual maxima stops k_cp5 and k_cp3 at iteration 1
    with the same status and history (to rounding). On these trees the maximum is flat after
    it (the xi2 term of the leaf SOC's constant offsets dominates, as the oracle's trace
    shows), so a later stop is not reachable by any tolerance there; the unboxed trees' mid-batch
    stops: test_cp5_mid_batch_early_stop_matches_cp3."""
    r = _recipe(case)
    tree, prob = build_problem(r)
    c5, c3 = _pair(prob)
    alpha = 0.999 / c5.native.step_size()
    _, err, _ = c3.native.cp_run(r["x0"], 30, 0.0, alpha)
    mx = err.max(axis=1)
    assert mx[1] < mx[0] * (1 - 1e-3) and np.all(mx[2:] >= mx[1] * (1 - 1e-9))
    tol = float(np.sqrt(mx[0] * mx[1]))
    a = _run(c5, r["x0"], 30, alpha, tol)
    b = _run(c3, r["x0"], 30, alpha, tol)
    assert a[0] == b[0] == 0 and a[1].shape == b[1].shape == (2, 3)
    assert trace_rel_err(a[1], b[1]) <= 1e-12 and rel_err(a[3], b[3]) <= 1e-12


@pytest.mark.parametrize("case", ["t32-nobox", "q20-nobox"])
def test_cp5_mid_batch_early_stop_matches_cp3(case):
    """Unboxed trees, whose residual maxima keep falling (with ripples): the tolerance is the
    first new low of k_cp3's trace after the first graph batch (k > 24, not at a batch's first
    or last iteration) by a 1 % margin, so both loops first meet it at that iteration; k_cp5
    stops there inside its graph batch with k_cp3's status, history and iterate."""
    r = _recipe(case)
    tree, prob = build_problem(r)
    c5, c3 = _pair(prob)
    assert c5.native.kernel_info(10).startswith("k_cp5_leaf<double")
    alpha = 0.999 / c5.native.step_size()
    K = 72
    _, err, _ = c3.native.cp_run(r["x0"], K, 0.0, alpha)
    mx = err.max(axis=1)
    lows = [k for k in range(25, K) if k % 24 not in (0, 23) and mx[k] < 0.99 * mx[:k].min()]
    assert lows, "the trace makes no new low after the first batch"
    k = lows[0]
    tol = float(mx[k]) * (1 + 1e-9)
    a = _run(c5, r["x0"], K, alpha, tol)
    b = _run(c3, r["x0"], K, alpha, tol)
    assert a[0] == b[0] == 0 and a[1].shape == b[1].shape == (k + 1, 3)
    assert trace_rel_err(a[1], b[1]) <= 1e-12 and trace_rel_err(a[2], b[2]) <= 1e-12
    assert rel_err(a[3], b[3]) <= 1e-12 and rel_err(a[4], b[4]) <= 1e-12


def test_cp5_nan_in_box_raises():
    """A NaN reaching a box projection (Rectangle._constrain, rectangle.py:50-59) raises
    ValueError through k_cp5 as through the reference."""
    r = _recipe("t32")
    tree, prob = build_problem(r)
    cache = core.Cache(prob)
    assert cache.native.kernel_info(10).startswith("k_cp5")
    x0 = np.array(r["x0"], dtype=float)
    x0[3] = np.nan
    alpha = 0.999 / cache.native.step_size()
    with pytest.raises(ValueError):
        cache.native.cp_run(x0, 5, 0.0, alpha)


@pytest.mark.parametrize("case", ["q20", "t32", "c4", "q64"])
def test_cp5_leaf_forms_agree(case):
    """k_cp5_leaf's two forms (RAOCP_CP5_LPF: 1 = one wave per SIMD with the next tile's
    operands in registers, 0 = two waves per SIMD with one L^T stream at a time, its entries
    recomputed; fp64 default 0, fp32 default 1) differ in FMA contraction only: 1e-12 on the
    traces and the iterate (fp32: 1e-5)."""
    r = _recipe(case)
    tree, prob = build_problem(r)
    dt = "float32" if case == "q64" else None
    mk = (lambda: core.Cache(prob, dtype=dt)) if dt else (lambda: core.Cache(prob))
    a = _with_env({"RAOCP_CP5_LPF": "1"}, mk)
    b = _with_env({"RAOCP_CP5_LPF": "0"}, mk)
    # each context reads the switch at its creation (not once per process)
    assert a.native.kernel_info(12).startswith("leaf_pf=1")
    assert b.native.kernel_info(12).startswith("leaf_pf=0")
    alpha = 0.999 / a.native.step_size(rtol=1e-7 if dt else 1e-14)
    K = 14 if case == "c4" else 30
    ra = _run(a, r["x0"], K, alpha)
    rb = _run(b, r["x0"], K, alpha)
    tol = 1e-5 if dt else 1e-12
    assert ra[0] == rb[0] == 1
    assert trace_rel_err(ra[1], rb[1]) <= tol and trace_rel_err(ra[2], rb[2]) <= tol
    assert rel_err(ra[3], rb[3]) <= tol and rel_err(ra[4], rb[4]) <= tol
