"""Problem recipes for tests, smoke and bench (not part of the reference API).

A recipe is a dict of plain arrays: Markov chain (P, v, N, tau), per-mode
dynamics A/B, per-mode nonleaf costs Q/R, leaf cost Pf, AVaR alpha_r, boxes and
the initial state x0. `build_problem(recipe)` turns it into a `raocp.core.RAOCP`
through the public builder API (the same calls main.py:18-76 makes), so the
GPU path is exercised exactly as a reference user would drive it.

Recipes mirror main.py:11-80, the reference tests' fixtures
(tests/test_operators.py:20-66, tests/test_cache.py:19-76) and the synthetic
benchmark configs of SURVEY.md section 8(d) / BASELINE.json `configs`.
"""
import numpy as np

import raocp.core as core
import raocp.core.constraints.rectangle as rectangle
import raocp.core.dynamics as dynamics

__all__ = ["recipe_main", "recipe_ops2x2", "recipe_cache3", "recipe_synthetic", "recipe_bin6",
           "recipe_c1n5", "recipe_config", "build_problem", "recipe_from_npz"]


def recipe_main():
    """main.py:11-79 (config 1 as committed: 43 nodes, nx=3, nu=2)."""
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0.0], [0.0, 0.3, 0.7]])
    f = 0.1
    Aw = f * np.array([[1, 2, 1], [1, 1, 2], [2, 1, 1]])
    Bw = f * np.array([[1, 0], [1, 0], [0, 2]])
    return dict(P=p, v=np.array([0.1, 0.6, 0.3]), N=4, tau=3,
                A=np.array([0.5 * Aw, Aw, -0.5 * Aw]), B=np.array([-0.5 * Bw, Bw, 0.5 * Bw]),
                Q=np.array([.2 * f * np.eye(3)] * 3), R=np.array([.2 * f * np.eye(2)] * 3),
                Pf=f * .1 * np.eye(3), alpha_r=.95,
                nl_min=np.r_[-7 * np.ones(3), -.1 * np.ones(2)], nl_max=np.r_[7 * np.ones(3), .1 * np.ones(2)],
                l_min=-7 * np.ones(3), l_max=7 * np.ones(3), x0=np.array([5., -6., -1.]))


def recipe_ops2x2():
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0], [0, 0.3, 0.7]])
    I2 = np.eye(2)
    return dict(P=p, v=np.array([0.5, 0.4, 0.1]), N=4, tau=3, A=np.array([I2, 2 * I2, 3 * I2]),
                B=np.array([I2, 2 * I2, 3 * I2]), Q=np.array([10 * I2, 20 * I2, 30 * I2]),
                R=np.array([I2, 2 * I2, 3 * I2]), Pf=5 * I2, alpha_r=0.5,
                nl_min=None, nl_max=None, l_min=None, l_max=None, x0=np.array([1., -1.]))


def recipe_cache3():
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0], [0, 0.3, 0.7]])
    I3, I2 = np.eye(3), np.eye(2)
    return dict(P=p, v=np.array([0.5, 0.4, 0.1]), N=4, tau=3, A=np.array([I3, 2 * I3, 3 * I3]),
                B=np.array([I3, 2 * I3, 3 * I3]), Q=np.array([10 * I2, 20 * I2, 30 * I2]),
                R=np.array([I2, 2 * I2, 3 * I2]), Pf=5 * I2, alpha_r=0.5,
                nl_min=-2 * np.ones(6), nl_max=2 * np.ones(6), l_min=-0.5 * np.ones(3), l_max=0.5 * np.ones(3),
                x0=np.array([0.3, -0.2, 0.1]))


def recipe_synthetic(P, v, N, tau, nx, nu, seed=0, alpha_r=0.9):
    """rng = default_rng(seed); per mode A then B ~ 0.1 N(0,1); Q=R=0.1 I,
    Pf = 0.01 I; boxes +-1 on [x;u] (nonleaf) and x (leaf); x0 ~ N(0,1) drawn after A/B."""
    rng = np.random.default_rng(seed)
    M = P.shape[0]
    A = np.zeros((M, nx, nx))
    B = np.zeros((M, nx, nu))
    for k in range(M):
        A[k] = 0.1 * rng.standard_normal((nx, nx))
        B[k] = 0.1 * rng.standard_normal((nx, nu))
    x0 = rng.standard_normal(nx)
    return dict(P=P, v=v, N=N, tau=tau, A=A, B=B, Q=np.array([0.1 * np.eye(nx)] * M),
                R=np.array([0.1 * np.eye(nu)] * M), Pf=0.01 * np.eye(nx), alpha_r=alpha_r,
                nl_min=-np.ones(nx + nu), nl_max=np.ones(nx + nu), l_min=-np.ones(nx), l_max=np.ones(nx), x0=x0)


def recipe_bin6():
    return recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 6, 6, 20, 8, seed=0)


def recipe_c1n5():
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0.0], [0.0, 0.3, 0.7]])
    return recipe_synthetic(p, np.array([0.1, 0.6, 0.3]), 5, 3, 4, 2, seed=3, alpha_r=0.95)


def recipe_config(k, seed=0):
    """BASELINE.json configs[k]."""
    if k == 1:
        return recipe_main()
    if k == 2:  # i.i.d. binary tree, N = 12: 8,191 nodes, nx=20, nu=8
        return recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 12, 12, 20, 8, seed=seed)
    if k == 3:  # Markov, 4 modes, full support, N = 8: 87,381 nodes
        rng = np.random.default_rng(seed + 100)
        P = rng.random((4, 4)) + 0.1
        P /= P.sum(axis=1, keepdims=True)
        return recipe_synthetic(P, np.full(4, .25), 8, 8, 20, 8, seed=seed)
    if k == 4:  # branching 3, N = 10: 88,573 nodes, nx=32, nu=12
        return recipe_synthetic(np.full((3, 3), 1 / 3), np.full(3, 1 / 3), 10, 10, 32, 12, seed=seed)
    if k == 5:  # branching 4, N = 9: 349,525 nodes, nx=64, nu=16
        return recipe_synthetic(np.full((4, 4), .25), np.full(4, .25), 9, 9, 64, 16, seed=seed)
    raise ValueError(f"unknown config {k}")


def recipe_from_npz(z, name):
    """Read a recipe stored by tests/golden/gen_golden.py under prefix `name/`."""
    keys = ["P", "v", "N", "tau", "A", "B", "Q", "R", "Pf", "alpha_r", "nl_min", "nl_max", "l_min", "l_max", "x0"]
    r = {}
    for k in keys:
        key = f"{name}/{k}"
        r[k] = z[key] if key in z else None
    for k in ("N", "tau"):
        r[k] = int(r[k])
    r["alpha_r"] = float(r["alpha_r"])
    return r


def build_problem(r):
    """Recipe -> (tree, RAOCP) via the public builder (main.py:18-76)."""
    tree = core.MarkovChainScenarioTreeFactory(transition_prob=r["P"], initial_distribution=r["v"],
                                               num_stages=r["N"], stopping_time=r["tau"]).create()
    nl, lf = core.Nonleaf(), core.Leaf()
    M = r["A"].shape[0]
    dyn = [dynamics.Dynamics(r["A"][k], r["B"][k]) for k in range(M)]
    costs = [core.Quadratic(nl, r["Q"][k], r["R"][k]) for k in range(M)]
    prob = core.RAOCP(scenario_tree=tree) \
        .with_markovian_dynamics(dyn) \
        .with_markovian_nonleaf_costs(costs) \
        .with_all_leaf_costs(core.Quadratic(lf, r["Pf"])) \
        .with_all_risks(core.AVaR(r["alpha_r"]))
    if r.get("nl_min") is not None:
        prob = prob.with_all_nonleaf_constraints(
            rectangle.Rectangle(nl, np.asarray(r["nl_min"]).reshape(-1, 1), np.asarray(r["nl_max"]).reshape(-1, 1)))
    if r.get("l_min") is not None:
        prob = prob.with_all_leaf_constraints(
            rectangle.Rectangle(lf, np.asarray(r["l_min"]).reshape(-1, 1), np.asarray(r["l_max"]).reshape(-1, 1)))
    return tree, prob
