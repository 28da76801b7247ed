"""CPU: the oracle (oracle/raocp_oracle.py) and the host tree factory pinned against the
reference's own outputs (tests/golden/*.npz, produced by tests/golden/gen_golden.py from
/root/reference).

These tests are what makes the oracle a trustworthy checker for the GPU parity tests:
every function the HIP path implements is pinned here against the reference on the
same inputs.
"""
import numpy as np
import pytest

from oracle.raocp_oracle import OracleProblem
import raocp.core as core
from helpers import problem_from_golden, rel_err, trace_rel_err

OPS = ["main", "ops2x2", "bin6", "c1n5"]
PROX = ["main", "bin6", "cache3", "c1n5"]
TRAJ = ["bin6", "c1n5", "ops2x2"]


def _oracle(z, name):
    r, tree, prob = problem_from_golden(z, name)
    return r, OracleProblem(prob)


# ---------------------------------------------------------------- scenario tree factory
def test_tree_factory_matches_reference_kats(golden):
    """scenario_tree.py:273-315 (MarkovChainScenarioTreeFactory.create), exact."""
    z = golden("tree_kat")
    for name in z["names"]:
        name = str(name)
        P, v = z[f"{name}/P"], z[f"{name}/v"]
        N, tau = int(z[f"{name}/N"]), int(z[f"{name}/tau"])
        tree = core.MarkovChainScenarioTreeFactory(P, v, N, tau).create()
        n, m = tree.num_nodes, tree.num_nonleaf_nodes
        assert n == z[f"{name}/tree_anc"].size, name
        assert m == int(z[f"{name}/tree_num_nonleaf"]), name
        anc = np.array([tree.ancestor_of(i) for i in range(n)])
        stg = np.array([tree.stage_of(i) for i in range(n)])
        val = np.array([tree.value_at_node(i) for i in range(n)])
        assert np.array_equal(anc, z[f"{name}/tree_anc"]), name
        assert np.array_equal(stg, z[f"{name}/tree_stage"]), name
        assert np.array_equal(val, z[f"{name}/tree_value"]), name
        # probabilities bit-identical, including the length-n+1 quirk when tau == N
        probs = np.asarray(tree._ScenarioTree__probability, dtype=float)
        assert np.array_equal(probs, z[f"{name}/tree_prob"]), name
        ch = np.concatenate([np.asarray(tree.children_of(i)) for i in range(m)]) if m else np.zeros(0)
        assert np.array_equal(ch, z[f"{name}/tree_children"]), name
        cond = np.concatenate([tree.conditional_probabilities_of_children(i) for i in range(m)])
        assert np.array_equal(cond, z[f"{name}/tree_cond_prob"]), name


# ---------------------------------------------------------------- L and L^T
@pytest.mark.parametrize("name", OPS)
def test_oracle_ell_matches_reference(golden, name):
    z = golden("ops_kat")
    r, orc = _oracle(z, name)
    assert orc.P == z[f"{name}/ops_z"].size and orc.D == z[f"{name}/ops_eta"].size
    assert rel_err(orc.ell(z[f"{name}/ops_z"]), z[f"{name}/ops_Lz"]) <= 1e-13
    assert rel_err(orc.ell_t(z[f"{name}/ops_eta"]), z[f"{name}/ops_LTeta"]) <= 1e-13
    # the block API rebinding only written slots (operators.py:19-94): template slots survive
    out_d = orc.ell(z[f"{name}/ops_z"], template=z[f"{name}/ops_tmpl_dual"])
    assert rel_err(out_d, z[f"{name}/ops_ell_out"]) <= 1e-13
    out_p = orc.ell_t(z[f"{name}/ops_eta"], template=z[f"{name}/ops_tmpl_primal"])
    assert rel_err(out_p, z[f"{name}/ops_ellT_out"]) <= 1e-13


@pytest.mark.parametrize("name", OPS)
def test_oracle_adjoint(golden, name):
    """tests/test_operators.py adjointness: <L z, eta> == <z, L^T eta> on active entries."""
    z = golden("ops_kat")
    r, orc = _oracle(z, name)
    rng = np.random.default_rng(7)
    zz = rng.standard_normal(orc.P)
    zz[orc.T0] = 0.0   # tau_0 is never read by L and never written by L^T
    ee = rng.standard_normal(orc.D)
    lhs = float(orc.ell(zz) @ ee)
    rhs = float(zz @ orc.ell_t(ee))
    assert abs(lhs - rhs) <= 1e-10 * max(1.0, abs(lhs))


# ---------------------------------------------------------------- proximal steps
@pytest.mark.parametrize("name", PROX)
def test_oracle_offline_products(golden, name):
    """cache.py:207-233: P, K, Abar per node from the per-class memo equal the reference's."""
    z = golden("prox_kat")
    r, orc = _oracle(z, name)
    P, K, Abar = orc.offline_per_node()
    m = orc.m
    assert rel_err(P, z[f"{name}/off_P"]) <= 1e-12
    assert rel_err(K[:m], z[f"{name}/off_K"]) <= 1e-12
    assert rel_err(Abar[1:], z[f"{name}/off_Abar"][1:]) <= 1e-12


@pytest.mark.parametrize("name", PROX)
def test_oracle_prox_f_steps(golden, name):
    z = golden("prox_kat")
    r, orc = _oracle(z, name)
    orc.offline()
    alpha = float(z[f"{name}/prox_alpha"])
    zin = z[f"{name}/prox_z"]
    x0 = r["x0"]
    assert rel_err(orc.project_on_dynamics(zin, x0), z[f"{name}/prox_dyn"]) <= 1e-11
    assert rel_err(orc.project_on_kernel(zin), z[f"{name}/prox_kernel"]) <= 1e-12
    assert rel_err(orc.prox_f(zin, alpha, x0), z[f"{name}/prox_f"]) <= 1e-11


@pytest.mark.parametrize("name", PROX)
def test_oracle_prox_gconj_steps(golden, name):
    z = golden("prox_kat")
    r, orc = _oracle(z, name)
    alpha = float(z[f"{name}/prox_alpha"])
    ein = z[f"{name}/prox_eta"]
    assert rel_err(orc.modify_dual_add_halves(ein, alpha), z[f"{name}/prox_modify_halves"]) <= 1e-14
    assert rel_err(orc.project_on_constraints_nonleaf(ein), z[f"{name}/prox_proj_nonleaf"]) <= 1e-14
    assert rel_err(orc.project_on_constraints_leaf(ein), z[f"{name}/prox_proj_leaf"]) <= 1e-14
    assert rel_err(orc.prox_gconj(ein, alpha), z[f"{name}/prox_gconj"]) <= 1e-13


# ---------------------------------------------------------------- the CP loop
def test_oracle_main_trace(golden):
    """main.py end to end: the 937 x 3 residual trace of the reference (and of
    4-3-residuals.tex) with the reference's own ARPACK step size."""
    z = golden("main_trace")
    r, orc = _oracle(z, "main")
    orc.offline()
    lam, _ = orc.step_size()
    assert abs(lam - float(z["main/cp_lambda"])) <= 1e-10 * lam
    st, err, derr, zf, ef, _ = orc.chock(r["x0"], int(z["main/cp_max_iters"]), float(z["main/cp_tol"]),
                                          alpha=float(z["main/cp_alpha"]))
    assert st == int(z["main/cp_status"])
    assert trace_rel_err(err, z["main/cp_error"]) <= 1e-8
    assert trace_rel_err(derr, z["main/cp_delta_error"]) <= 1e-8
    assert rel_err(zf, z["main/cp_z"]) <= 1e-9
    assert rel_err(ef, z["main/cp_eta"]) <= 1e-9
    # the tex file carries the same trace at its printed precision
    tex = z["main/tex_trace"]
    assert tex.shape == err.shape
    assert np.max(np.abs(err - tex) / np.abs(tex)) <= 1e-6


@pytest.mark.parametrize("name", TRAJ)
def test_oracle_small_trajectories(golden, name):
    z = golden("traj_small")
    r, orc = _oracle(z, name)
    orc.offline()
    st, err, derr, zf, ef, _ = orc.chock(r["x0"], int(z[f"{name}/cp_max_iters"]), float(z[f"{name}/cp_tol"]),
                                          alpha=float(z[f"{name}/cp_alpha"]))
    assert st == int(z[f"{name}/cp_status"])
    assert trace_rel_err(err, z[f"{name}/cp_error"]) <= 1e-8
    assert trace_rel_err(derr, z[f"{name}/cp_delta_error"]) <= 1e-8
    assert rel_err(zf, z[f"{name}/cp_z"]) <= 1e-9
    assert rel_err(ef, z[f"{name}/cp_eta"]) <= 1e-9


def test_oracle_chock_status_contract(golden):
    """solver.py:163-166: 0 if it stopped before max_iters, else 1 (also when the
    tolerance is met exactly at k == max_iters)."""
    z = golden("main_trace")
    r, orc = _oracle(z, "main")
    orc.offline()
    alpha = float(z["main/cp_alpha"])
    n_it = z["main/cp_error"].shape[0]           # 937 rows: stopped at k = 936
    st, err, _, _, _, _ = orc.chock(r["x0"], n_it - 1, float(z["main/cp_tol"]), alpha=alpha)
    assert st == 1 and err.shape[0] == n_it
    st, err, _, _, _, _ = orc.chock(r["x0"], 0, 0.0, alpha=alpha)
    assert st == 1 and err.shape[0] == 1


def test_oracle_warm_start_matches_reference(golden):
    """Two chock calls on one reference Solver (tests/golden/gen_golden.py gen_warm): the
    second continues from the first one's cached primal / dual with x0 / 2 written into
    node 0's state (solver.py:97-102, cache.py:79-82). The oracle's p0 / d0 path reproduces
    both calls' traces and iterates."""
    z = golden("warm_start")
    r, tree, prob = problem_from_golden(z, "warm")
    orc = OracleProblem(prob)
    p0 = d0 = None
    for call in (0, 1):
        key = f"warm/call{call}/"
        st, err, derr, p0, d0, _ = orc.chock(z[key + "x0"], int(z[key + "max_iters"]), 0.0,
                                             alpha=float(z[key + "alpha"]), p0=p0, d0=d0)
        assert st == int(z[key + "status"])
        assert trace_rel_err(err, z[key + "error"]) <= 1e-9
        assert trace_rel_err(derr, z[key + "delta_error"]) <= 1e-9
        assert rel_err(p0, z[key + "z"]) <= 1e-10 and rel_err(d0, z[key + "eta"]) <= 1e-10
