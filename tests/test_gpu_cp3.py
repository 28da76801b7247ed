"""GPU parity of the fused CP iteration k_cp3 (raocp_cp3.hip: the dual step, prox g*, the
next primal half step with the AVaR kernel projection and all six residuals in ONE launch
after the dynamics sweep, xi2 kept in registers). It is the default on trees with one
branching factor and one sqrtQ / sqrtR / sqrtPf table at the benchmark sizes; RAOCP_CP3=0
selects the two-launch kernels (k_cpd* + k_cpp*, xi2 through HBM).

Both paths compute the reference's arithmetic (solver.py:27-95, cache.py:248-393) with the
sums of L / L^T in a different order, so they agree to rounding: residual traces within
1e-10 relative per entry and iterates within 1e-11 of their largest entry, and both match
the oracle within the suite's tolerances (traces 1e-8, iterates 1e-10).

fp32 (BASELINE configs[4] and the fp32 variants of configs 2 / 4): 30 CP iterations of an
fp32 context against the fp64 run of the same problem. The drift bound: each iteration's
products are fp32 dot products of <= 80 terms (a few ulp, 1.2e-7 each) and the CP map is
non-expansive, so the iterate error grows at most linearly in the iteration count: 30
iterations x ~3e-7 per iteration -> 1e-5 of the iterate scale; the residual maxima
(differences of iterates over alpha) carry that error relative to their own size, bounded
here by 1e-4 per trace entry (measured on MI355X: traces 2-3e-6, iterates 1e-7 - 1e-6).
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
    if cfg == "chain":  # C = 1
        return recipe_synthetic(np.ones((1, 1)), np.ones(1), 40, 40, 20, 8, seed=3)
    if cfg == "quad":  # C = 4 at nx = 20
        return recipe_synthetic(np.full((4, 4), .25), np.full(4, .25), 5, 5, 20, 8, seed=6)
    if cfg == "bin32":  # C = 2 at nx = 32
        return recipe_synthetic(np.full((2, 2), .5), np.full(2, .5), 9, 9, 32, 12, seed=4)
    if cfg in ("c2-nobox", "c2-leafbox"):
        r = recipe_config(2)
        r["nl_min"] = r["nl_max"] = None
        if cfg == "c2-nobox":
            r["l_min"] = r["l_max"] = None
        return r
    if cfg == "c2-a95":  # main.py's AVaR level at the benchmark size
        r = recipe_config(2)
        r["alpha_r"] = 0.95
        return r
    return recipe_config(int(cfg[1:]))


@pytest.mark.parametrize("cfg", ["c2", "c4", "chain", "quad", "bin32", "c2-nobox", "c2-leafbox", "c2-a95"])
def test_cp3_matches_two_kernel_path_and_oracle(cfg):
    from oracle.raocp_oracle import OracleProblem
    r = _recipe(cfg)
    tree, prob = build_problem(r)
    fused = core.Cache(prob)
    two = _with_env({"RAOCP_CP3": "0"}, lambda: core.Cache(prob))
    # the fused iteration: k_cp6 (a workgroup per family tile, config 2 boxed / unboxed), k_cp4
    # (tile-start loads, C = 2 at 20 / 8 otherwise), k_cp5 (leaf + family launches, configs 3 / 4
    # and C = 4 at 20 / 8) or k_cp3
    assert fused.native.kernel_info(10).startswith(("k_cp3<double", "k_cp4<double", "k_cp5_leaf<double", "k_cp6<double"))
    assert not two.native.kernel_info(10).startswith(("k_cp3", "k_cp4", "k_cp5", "k_cp6"))
    alpha = 0.999 / fused.native.step_size()
    K = 12 if cfg == "c4" else 20
    out = []
    for cache in (fused, two):
        st, err, derr = cache.native.cp_run(r["x0"], K, 0.0, alpha)
        out.append((st, err, derr, cache.get_primal_flat(), cache.get_dual_flat()))
    (s1, e1, d1, z1, y1), (s2, e2, d2, z2, y2) = out
    assert s1 == s2 == 1 and e1.shape == e2.shape == (K + 1, 3)
    assert trace_rel_err(e1, e2) <= 1e-10 and trace_rel_err(d1, d2) <= 1e-10
    assert rel_err(z1, z2) <= 1e-11 and rel_err(y1, y2) <= 1e-11
    st_o, err_o, derr_o, z_o, e_o, _ = OracleProblem(prob).chock(r["x0"], K, 0.0, alpha=alpha)
    assert trace_rel_err(e1, err_o) <= 1e-8 and trace_rel_err(d1, derr_o) <= 1e-8
    assert rel_err(z1, z_o) <= 1e-10 and rel_err(y1, e_o) <= 1e-10


def test_cp3_early_stop_and_batches():
    """A tolerance met mid-batch (graph batches of 24 iterations) stops the fused loop at the
    same iteration with the same history as the two-launch loop."""
    r = recipe_config(2)
    tree, prob = build_problem(r)
    fused = core.Cache(prob)
    two = _with_env({"RAOCP_CP3": "0"}, lambda: core.Cache(prob))
    alpha = 0.999 / fused.native.step_size()
    _, err, _ = two.native.cp_run(r["x0"], 60, 0.0, alpha)
    # a tolerance between two of the run's residual maxima, far (> 1e-6 relative) from every
    # one of them, so that the two paths (1e-10 apart) take the same stopping decisions
    mx = np.sort(err.max(axis=1))
    gaps = [(mx[q + 1] / mx[q], q) for q in range(10, 40) if mx[q + 1] > mx[q] * (1 + 1e-6)]
    q = max(gaps)[1]
    tol = float(np.sqrt(mx[q] * mx[q + 1]))
    s1, e1, _ = fused.native.cp_run(r["x0"], 60, tol, alpha)
    s2, e2, _ = two.native.cp_run(r["x0"], 60, tol, alpha)
    assert s1 == s2 == 0 and e1.shape == e2.shape and e1.shape[0] < 60
    assert trace_rel_err(e1, e2) <= 1e-10


@pytest.mark.parametrize("cfg", ["c2", "c4", "chain"])
def test_cp3_split_matches_fused(cfg):
    """The split task layout (RAOCP_CP3_SPLIT=1, default on small trees: leaves as tasks of
    their own, the family recomputing only their SOC scalars) against the fused family
    tiles: the same arithmetic per entry, so the runs agree to rounding (1e-10)."""
    r = _recipe(cfg)
    tree, prob = build_problem(r)
    a = _with_env({"RAOCP_CP3_SPLIT": "1", "RAOCP_CP5": "0", "RAOCP_CP6": "0"}, lambda: core.Cache(prob))
    b = _with_env({"RAOCP_CP3_SPLIT": "0", "RAOCP_CP5": "0", "RAOCP_CP6": "0"}, lambda: core.Cache(prob))
    alpha = 0.999 / a.native.step_size()
    K = 10 if cfg == "c4" else 20
    out = []
    for cache in (a, b):
        st, err, derr = cache.native.cp_run(r["x0"], K, 0.0, alpha)
        out.append((st, err, derr, cache.get_primal_flat(), cache.get_dual_flat()))
    (s1, e1, d1, z1, y1), (s2, e2, d2, z2, y2) = out
    assert s1 == s2 and trace_rel_err(e1, e2) <= 1e-10 and trace_rel_err(d1, d2) <= 1e-10
    assert rel_err(z1, z2) <= 1e-11 and rel_err(y1, y2) <= 1e-11


@pytest.mark.parametrize("cfg", ["c2", "c4", "c5", "c5-cp3"])
def test_cp3_fp32_drift_vs_fp64(cfg):
    """30 fp32 CP iterations (k_cp3<float, ...>; config 5: k_cp5<float> by default, k_cp3 with
    RAOCP_CP5=0) against the fp64 run of the same problem and step size (fp64: the k_cp3 /
    k_cpd2 + k_cpp2 path pinned to the oracle above)."""
    r = recipe_config(int(cfg[1]))
    tree, prob = build_problem(r)
    c32 = _with_env({"RAOCP_CP5": "0"} if cfg.endswith("cp3") else {}, lambda: core.Cache(prob, dtype="float32"))
    assert c32.native.kernel_info(10).startswith("k_cp5_leaf<float" if cfg == "c5" else "k_cp3<float")
    c64 = core.Cache(prob)
    alpha = 0.999 / c64.native.step_size()
    K = 29
    s32, e32, d32 = c32.native.cp_run(r["x0"], K, 0.0, alpha)
    s64, e64, d64 = c64.native.cp_run(r["x0"], K, 0.0, alpha)
    assert s32 == s64 == 1 and e32.shape == e64.shape == (K + 1, 3)
    te, td = trace_rel_err(e32, e64), trace_rel_err(d32, d64)
    zr = rel_err(c32.get_primal_flat(), c64.get_primal_flat())
    er = rel_err(c32.get_dual_flat(), c64.get_dual_flat())
    print(f"fp32 drift {cfg}: traces {te:.2e} / {td:.2e}, iterate {zr:.2e} / {er:.2e}")
    assert te <= 1e-4 and td <= 1e-4
    assert zr <= 1e-5 and er <= 1e-5
