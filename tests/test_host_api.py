"""CPU: the host mirror of the reference's problem-builder API (raocp.core.*), checked
for the behaviour the reference's own unit tests pin (tests/test_costs.py,
test_risks.py, test_rectangle.py, test_base_constraint.py, test_no_constraint.py,
test_nodes.py, test_dynamics.py, test_cones.py, test_raocp.py, test_scenario_tree.py).
These classes are the input side of the hot path: the packer reads them.
"""
import numpy as np
import pytest
from scipy.linalg import sqrtm

import raocp.core as core
import raocp.core.costs as costs
import raocp.core.dynamics as dynamics
import raocp.core.nodes as nodes
import raocp.core.risks as risks
import raocp.core.raocp_spec as spec
import raocp.core.scenario_tree as tree_mod
import raocp.core.constraints.cones as cones
import raocp.core.constraints.rectangle as rectangle
import raocp.core.constraints.no_constraint as no_constraint
import raocp.core.constraints.base_constraint as base_constraint

NL, L = nodes.Nonleaf(), nodes.Leaf()


# ---------------------------------------------------------------- nodes / dynamics / costs
def test_nodes():
    assert NL.is_nonleaf and not NL.is_leaf
    assert L.is_leaf and not L.is_nonleaf


def test_dynamics_shapes():
    d = dynamics.Dynamics(np.eye(3), np.ones((3, 2)))
    assert d.state_dynamics.shape == (3, 3) and d.control_dynamics.shape == (3, 2)
    with pytest.raises(ValueError):
        dynamics.Dynamics(np.eye(3), np.ones((2, 2)))


def test_quadratic_costs():
    w = np.diag([1.0, 4.0, 9.0])
    c = costs.Quadratic(NL, w, np.eye(2))
    assert np.array_equal(c.state_weights, w)
    assert np.array_equal(c.sqrt_state_weights, sqrtm(w))
    assert np.array_equal(c.sqrt_control_weights, sqrtm(np.eye(2)))
    leaf = costs.Quadratic(L, 5 * np.eye(3))
    assert np.array_equal(leaf.sqrt_state_weights, sqrtm(5 * np.eye(3)))
    with pytest.raises(Exception):
        costs.Quadratic(NL, w)                       # nonleaf without control weights
    with pytest.raises(Exception):
        costs.Quadratic(L, w, np.eye(2))             # leaf with control weights
    with pytest.raises(Exception):
        costs.Quadratic(NL, np.ones((2, 3)), np.eye(2))
    with pytest.raises(Exception):
        costs.Quadratic(NL, w, np.ones((2, 3)))
    with pytest.raises(Exception):
        costs.Quadratic(L, np.ones((2, 3)))


# ---------------------------------------------------------------- risks
def test_avar():
    assert risks.AVaR.is_risk
    for a in (0.0, 1.0, 0.5):
        assert risks.AVaR(a).alpha == a
    for a in (-0.1, 1.1):
        with pytest.raises(ValueError):
            risks.AVaR(a)
    r = risks.AVaR(0.5)
    probs = np.array([0.2, 0.3, 0.5])
    r.probs = probs
    assert np.array_equal(r.probs, probs)
    c = probs.size
    assert r.matrix_e.shape == (2 * c + 1, c)
    assert r.matrix_f.shape == (2 * c + 1, 0)
    assert r.cone.dimension == 2 * c + 1
    assert r.vector_b.shape == (2 * c + 1, 1)
    # E = [alpha I; -I; 1'], b = [p; 0; 1] (risks.py:26-35 of the reference)
    assert np.array_equal(r.matrix_e[:c], 0.5 * np.eye(c))
    assert np.array_equal(r.matrix_e[c:2 * c], -np.eye(c))
    assert np.array_equal(r.vector_b.ravel(), np.concatenate([probs, np.zeros(c), [1.0]]))


# ---------------------------------------------------------------- constraints
def test_base_and_no_constraint():
    b = base_constraint.Constraint(NL)
    with pytest.raises(Exception):
        _ = b.is_active
    b.state_size = 3
    b.control_size = 2
    assert b.state_size == 3 and b.control_size == 2
    lb = base_constraint.Constraint(L)
    lb.state_size = 3
    assert lb.control_size == 0
    with pytest.raises(Exception):
        lb.control_size = 2
    assert not no_constraint.No(NL).is_active


def test_rectangle():
    lo, hi = -np.ones((5, 1)), 2 * np.ones((5, 1))
    r = rectangle.Rectangle(NL, lo, hi)
    assert r.is_active
    r.state_size = 3
    r.control_size = 2
    assert np.array_equal(r.state_matrix, np.vstack([np.eye(3), np.zeros((2, 3))]))
    assert np.array_equal(r.control_matrix, np.vstack([np.zeros((3, 2)), np.eye(2)]))
    v = np.array([[-3.0], [0.5], [5.0], [2.0], [-1.0]])
    p = r.project(v)
    assert np.array_equal(p.ravel(), [-1.0, 0.5, 2.0, 2.0, -1.0])
    with pytest.raises(Exception):
        r.project(np.ones((4, 1)))
    with pytest.raises(ValueError):
        r.project(np.array([[np.nan], [0], [0], [0], [0]]))
    with pytest.raises(Exception):
        rectangle.Rectangle(NL, np.ones(2), np.zeros(2))       # min > max
    with pytest.raises(Exception):
        rectangle.Rectangle(NL, np.ones(2), np.ones(3))        # sizes differ


# ---------------------------------------------------------------- cones (projection VI)
def _vi_ok(x, p, samples):
    x, p = x.ravel(), p.ravel()
    return all(np.inner(x - p, s - p) <= 1e-10 for s in samples)


def test_cone_projections_variational_inequality():
    rng = np.random.default_rng(0)
    d = 20
    for _ in range(20):
        x = 10 * rng.standard_normal((d, 1))
        assert _vi_ok(x, cones.Real().project(x), [rng.integers(-100, 100, d) for _ in range(20)])
        assert _vi_ok(x, cones.Zero().project(x), [np.zeros(d)])
        assert _vi_ok(x, cones.NonnegativeOrthant().project(x), [rng.integers(0, 100, d) for _ in range(20)])
        soc = []
        for _ in range(20):
            s = rng.standard_normal(d - 1)
            soc.append(np.hstack([s, np.linalg.norm(s) + abs(rng.standard_normal())]))
        assert _vi_ok(x, cones.SecondOrderCone().project(x), soc)
        # duals: R* = {0}, {0}* = R, the other two are self dual
        assert np.array_equal(cones.Real().project_onto_dual(x), np.zeros((d, 1)))
        assert np.array_equal(cones.Zero().project_onto_dual(x), x)
    with pytest.raises(ValueError):
        cones._check_dimension("Real", 5, np.ones(6))
    cart = cones.Cartesian([cones.Real(), cones.Zero(), cones.NonnegativeOrthant(), cones.SecondOrderCone()])
    x = rng.standard_normal((4 * d, 1))
    p = cart.project([x[:d], x[d:2 * d], x[2 * d:3 * d], x[3 * d:]])   # a list in, a list out
    assert np.array_equal(p[0], x[:d]) and np.array_equal(p[1], np.zeros((d, 1)))
    assert np.array_equal(p[2], np.maximum(x[2 * d:3 * d], 0))
    cart2 = cones.Cartesian([cones.Real(d), cones.Zero(d), cones.NonnegativeOrthant(d), cones.SecondOrderCone(d)]) \
        if cones.Real.__init__.__code__.co_argcount > 1 else None
    if cart2 is not None:   # one stacked vector in, one stacked vector out
        q = cart2.project([x])
        assert q.shape == (4 * d, 1) and np.array_equal(q[:d], x[:d])


def test_soc_three_cases():
    """cones.py:113-132: inside, polar, and the boundary case."""
    soc = cones.SecondOrderCone()
    inside = np.array([[0.3], [0.4], [1.0]])
    assert np.array_equal(soc.project(inside), inside)
    polar = np.array([[0.3], [0.4], [-1.0]])
    assert np.array_equal(soc.project(polar), np.zeros((3, 1)))
    x = np.array([[3.0], [4.0], [1.0]])
    p = soc.project(x).ravel()
    assert np.allclose(p, 3.0 * np.array([0.6, 0.8, 1.0]))


# ---------------------------------------------------------------- scenario tree
def test_scenario_tree_markov_kat():
    """tests/test_scenario_tree.py:11-50 of the reference."""
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0], [0, 0.3, 0.7]])
    v = np.array([0.5, 0.5, 0])
    t = core.MarkovChainScenarioTreeFactory(p, v, 4, 3).create()
    assert t.num_nonleaf_nodes == 20 and t.num_nodes == 32 and t.num_stages == 5
    assert [t.ancestor_of(i) for i in range(1, 11)] == [0, 0, 1, 1, 1, 2, 2, 3, 3, 3]
    assert t.ancestor_of(13) == 5 and all(t.ancestor_of(20 + i) == 8 + i for i in range(12))
    assert [len(t.children_of(i)) for i in (0, 1, 2, 5, 6)] == [2, 3, 2, 2, 3]
    assert all(len(t.children_of(i)) == 1 for i in range(8, 20))
    with pytest.raises(IndexError):
        t.children_of(20)
    with pytest.raises(ValueError):
        t.stage_of(-1)
    assert t.stage_of(0) == 0 and t.stage_of(31) == 4
    assert np.isclose(sum(t.probability_of_node(i) for i in t.nodes_at_stage(4)), 1.0)
    assert t.is_markovian


def test_scenario_tree_factory_checks():
    p = np.array([[0.5, 0.5], [0.5, 0.5]])
    with pytest.raises(ValueError):
        core.MarkovChainScenarioTreeFactory(p, np.array([0.5, 0.6]), 3, 2)
    with pytest.raises(ValueError):
        core.MarkovChainScenarioTreeFactory(np.array([[0.5, 0.6], [0.5, 0.5]]), np.array([0.5, 0.5]), 3, 2)
    with pytest.raises(ValueError):
        core.MarkovChainScenarioTreeFactory(p, np.array([0.5, 0.5]), 3, 4)   # tau > N


def test_scenario_tree_large_is_vectorised():
    """The factory builds the benchmark tree (8,191 nodes) quickly."""
    import time
    t0 = time.perf_counter()
    t = core.MarkovChainScenarioTreeFactory(np.full((2, 2), .5), np.array([.5, .5]), 12, 12).create()
    assert t.num_nodes == 8191 and t.num_nonleaf_nodes == 4095
    assert time.perf_counter() - t0 < 5.0


# ---------------------------------------------------------------- RAOCP builder
def _raocp():
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0], [0, 0.3, 0.7]])
    tree = core.MarkovChainScenarioTreeFactory(p, np.array([0.5, 0.4, 0.1]), 4, 3).create()
    dyn = [dynamics.Dynamics(k * np.eye(2), k * np.eye(2)) for k in (1, 2, 3)]
    nlc = [costs.Quadratic(NL, 10 * k * np.eye(2), k * np.eye(2)) for k in (1, 2, 3)]
    leaf = costs.Quadratic(L, 5 * np.eye(2))
    nl_rect = rectangle.Rectangle(NL, -2 * np.ones((4, 1)), 2 * np.ones((4, 1)))
    l_rect = rectangle.Rectangle(L, -.5 * np.ones((2, 1)), .5 * np.ones((2, 1)))
    prob = spec.RAOCP(scenario_tree=tree).with_markovian_dynamics(dyn).with_markovian_nonleaf_costs(nlc) \
        .with_all_leaf_costs(leaf).with_all_nonleaf_constraints(nl_rect).with_all_leaf_constraints(l_rect) \
        .with_all_risks(risks.AVaR(0.5))
    return tree, prob


def test_raocp_builder_lists():
    tree, prob = _raocp()
    n, m = tree.num_nodes, tree.num_nonleaf_nodes
    assert prob.list_of_dynamics[0] is None
    assert all(prob.list_of_dynamics[i] is not None for i in range(1, n))
    assert all(prob.list_of_nonleaf_costs[i] is not None for i in range(1, n))
    for i in range(n):
        assert (prob.list_of_leaf_costs[i] is None) == (i < m)
        assert (prob.list_of_leaf_constraints[i] is None) == (i < m)
    assert all(prob.list_of_nonleaf_constraints[i] is not None for i in range(m))
    assert all(prob.list_of_risks[i] is not None for i in range(m))
    # per-node risks carry the node's conditional probabilities
    for i in range(m):
        assert np.array_equal(prob.risk_at_node(i).probs, tree.conditional_probabilities_of_children(i))
    # Markovian dynamics follow the node's value
    for j in range(1, n):
        k = tree.value_at_node(j) + 1
        assert np.array_equal(prob.state_dynamics_at_node(j), k * np.eye(2))


def test_raocp_builder_failures():
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0], [0, 0.3, 0.7]])
    tree = core.MarkovChainScenarioTreeFactory(p, np.array([0.5, 0.4, 0.1]), 4, 3).create()
    with pytest.raises(ValueError):
        spec.RAOCP(scenario_tree=tree).with_markovian_dynamics(
            [dynamics.Dynamics(np.eye(2), np.eye(2)), dynamics.Dynamics(np.eye(3), np.eye(3)),
             dynamics.Dynamics(np.eye(2), np.eye(2))])
    with pytest.raises(Exception):
        spec.RAOCP(scenario_tree=tree).with_all_nonleaf_constraints(
            rectangle.Rectangle(NL, -np.ones((4, 1)), np.ones((4, 1))))
    with pytest.raises(Exception):
        spec.RAOCP(scenario_tree=tree).with_all_leaf_constraints(
            rectangle.Rectangle(L, -np.ones((2, 1)), np.ones((2, 1))))
