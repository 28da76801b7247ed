"""GPU parity of the split sweep k_dyn_up / k_dyn_down (raocp_dynf.hip; cache.py:259-288):
the tiered dynamics in two launches, one workgroup per subtree of every tier plus the top,
counters of arrivals up the tiers and epoch flags down. It is the fallback of regular trees
the regular-tree sweep (raocp_dynr.hip, test_gpu_dynr.py) does not take (other state and
input sizes: "t32" below, nx = 32, nu = 12, branching 3) where its grid is co-resident (not
config 2's 274 workgroups at 153 VGPRs: there the tier launches run), against the tier
launches (RAOCP_DYN_SPLIT=0).

The split sweep runs the tier kernels' level routines on the same operands; its top runs
on 512 lanes where k_dyn_top has 1,024, which changes the split-k summation order of the
top's dot products. So: against the tier launches 1e-13 of the largest entry (projection),
1e-10 per residual entry (CP trace); against itself after 1,000 back-to-back launches (the
counters and flags carry over between launches without a host reset) bit for bit; against
the oracle 1e-12 of the largest entry (projection), 1e-8 per residual entry (CP trace).
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
    if cfg == "quad":  # branching 4, tiers of 4-ary subtrees
        return recipe_synthetic(np.full((4, 4), .25), np.full(4, .25), 6, 6, 20, 8, seed=6)
    if cfg == "bin10":
        return recipe_synthetic(np.full((2, 2), .5), np.full(2, .5), 10, 10, 20, 8, seed=4)
    if cfg == "t32":  # branching 3, N = 7 (3,280 nodes), nx = 32, nu = 12: not a k_dr size
        return recipe_synthetic(np.full((3, 3), 1 / 3), np.full(3, 1 / 3), 7, 7, 32, 12, seed=7)
    return recipe_config(int(cfg[1:]))


SPLIT = {"RAOCP_DR": "0"}
TIERS = {"RAOCP_DYN_SPLIT": "0", "RAOCP_DR": "0"}
MODES = {"split": (SPLIT, "k_dyn_up")}


def _pair(prob, env=None, mode=SPLIT):
    env = env or {}
    sweep = _with_env({**env, **mode}, lambda: core.Cache(prob))
    tiers = _with_env({**env, **TIERS}, lambda: core.Cache(prob))
    return sweep, tiers


@pytest.mark.parametrize("env", [{}, {"RAOCP_DYN_FOLD": "0"}], ids=["default", "two_phase"])
@pytest.mark.parametrize("mode", ["split"])
@pytest.mark.parametrize("cfg", ["t32", "bin10"])
def test_split_projection_matches_tiers_and_oracle(cfg, mode, env):
    """default: one-phase backward levels (per-pair WT tables) in the sweep and in the tiers;
    two_phase: the two-phase levels (per-kind W, child products through LDS)."""
    from oracle.raocp_oracle import OracleProblem
    r = _recipe(cfg)
    tree, prob = build_problem(r)
    sweep, tiers = _pair(prob, env, MODES[mode][0])
    name = MODES[mode][1]
    assert sweep.native.kernel_info(9).startswith(name), sweep.native.kernel_info(9)
    assert not any(n in tiers.native.kernel_info(9) for _, n in MODES.values())
    zz = np.random.default_rng(5).standard_normal(sweep.primal_size)
    out = []
    for cache in (sweep, tiers):
        cache.cache_initial_state(r["x0"])
        cache.native.set_primal(zz)
        cache.native.project_on_dynamics()
        out.append(cache.native.get_primal())
    assert rel_err(out[0], out[1]) <= 1e-13
    assert rel_err(out[0], OracleProblem(prob).project_on_dynamics(zz, r["x0"])) <= 1e-12


@pytest.mark.parametrize("mode", ["split"])
def test_split_cp_loop_matches_tiers(mode):
    """30 CP iterations (one full 24-iteration graph batch plus a remainder), tol = 0."""
    from oracle.raocp_oracle import OracleProblem
    r = _recipe("t32")
    tree, prob = build_problem(r)
    sweep, tiers = _pair(prob, None, MODES[mode][0])
    assert sweep.native.kernel_info(9).startswith(MODES[mode][1])
    alpha = 0.999 / sweep.native.step_size()
    out = []
    for cache in (sweep, tiers):
        st, err, derr = cache.native.cp_run(r["x0"], 30, 0.0, alpha)
        out.append((st, err, derr, cache.get_primal_flat(), cache.get_dual_flat()))
    (s1, e1, d1, z1, y1), (s2, e2, d2, z2, y2) = out
    assert s1 == s2 == 1 and e1.shape == e2.shape == (31, 3)
    assert trace_rel_err(e1, e2) <= 1e-10 and trace_rel_err(d1, d2) <= 1e-10
    assert rel_err(z1, z2) <= 1e-11 and rel_err(y1, y2) <= 1e-11
    st_o, err_o, _, z_o, _, _ = OracleProblem(prob).chock(r["x0"], 30, 0.0, alpha=alpha)
    assert trace_rel_err(out[0][1], err_o) <= 1e-8 and rel_err(out[0][3], z_o) <= 1e-10


@pytest.mark.parametrize("mode", ["split"])
def test_split_many_launches_then_projection(mode):
    """1,000 back-to-back launches (graph-replayed, as in the CP loop): the tickets / counters
    are reset and the epoch advances inside the kernels; a projection afterwards is the same
    bit for bit."""
    r = _recipe("t32")
    tree, prob = build_problem(r)
    sweep = _with_env(MODES[mode][0], lambda: core.Cache(prob))
    assert sweep.native.kernel_info(9).startswith(MODES[mode][1])
    zz = np.random.default_rng(9).standard_normal(sweep.primal_size)
    out = []
    for rep in range(2):  # (op_bench initialises the CP control block with x0 = 0)
        sweep.cache_initial_state(r["x0"])
        sweep.native.set_primal(zz)
        sweep.native.project_on_dynamics()
        out.append(sweep.native.get_primal())
        sweep.native.op_bench(9, 1000)
    assert np.array_equal(out[0], out[1])
