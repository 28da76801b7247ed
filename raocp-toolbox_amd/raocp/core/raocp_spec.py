# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Risk-averse optimal control problem builder (reference: raocp/core/raocp_spec.py:7-198).

Same fluent API. One deliberate difference: the reference deep-copies the
given cost/constraint/risk object into every node slot (raocp_spec.py:127,
138, 147, 161, 171, 182), which runs out of memory at 350k nodes (SURVEY.md
section 6). Here every node slot holds a *reference* to the shared object;
only AVaR risks are copied (shallowly) per nonleaf node because each carries
that node's conditional probabilities. Nothing in the solver mutates these
objects, so the numbers are unchanged; identity sharing is also what the
device packer uses to build its per-mode matrix tables (`raocp.core._pack`).
"""
import copy

import raocp.core.constraints as core_constraints
import raocp.core.scenario_tree as core_tree

__all__ = ["RAOCP"]


class RAOCP:
    def __init__(self, scenario_tree: core_tree.ScenarioTree):
        self.__tree = scenario_tree
        self.__num_nodes = scenario_tree.num_nodes
        self.__num_nonleaf_nodes = scenario_tree.num_nonleaf_nodes
        self.__num_possibilities = len(scenario_tree.children_of(0))
        n = self.__num_nodes
        self.__list_of_dynamics = [None] * n
        self.__list_of_nonleaf_costs = [None] * n
        self.__list_of_leaf_costs = [None] * n
        self.__list_of_nonleaf_constraints = [None] * n
        self.__list_of_leaf_constraints = [None] * n
        self.__list_of_risks = [None] * self.__num_nonleaf_nodes
        self._load_constraints()

    # ----- getters
    @property
    def tree(self):
        return self.__tree

    @property
    def list_of_dynamics(self):
        return self.__list_of_dynamics

    @property
    def list_of_nonleaf_costs(self):
        return self.__list_of_nonleaf_costs

    @property
    def list_of_leaf_costs(self):
        return self.__list_of_leaf_costs

    @property
    def list_of_nonleaf_constraints(self):
        return self.__list_of_nonleaf_constraints

    @property
    def list_of_leaf_constraints(self):
        return self.__list_of_leaf_constraints

    @property
    def list_of_risks(self):
        return self.__list_of_risks

    def state_dynamics_at_node(self, idx):
        return self.__list_of_dynamics[idx].state_dynamics

    def control_dynamics_at_node(self, idx):
        return self.__list_of_dynamics[idx].control_dynamics

    def nonleaf_cost_at_node(self, idx):
        return self.__list_of_nonleaf_costs[idx]

    def leaf_cost_at_node(self, idx):
        return self.__list_of_leaf_costs[idx]

    def nonleaf_constraint_at_node(self, idx):
        return self.__list_of_nonleaf_constraints[idx]

    def leaf_constraint_at_node(self, idx):
        return self.__list_of_leaf_constraints[idx]

    def risk_at_node(self, idx):
        return self.__list_of_risks[idx]

    # ----- checks
    def _is_dynamics_given(self):
        # the reference looks at node 1 only (raocp_spec.py:77-82)
        if len(self.__list_of_dynamics) < 2:
            return None
        return self.__list_of_dynamics[1] is not None

    def _check_dynamics_before_constraints(self):
        if not self._is_dynamics_given():
            raise Exception("Constraints provided before dynamics - dynamics must be provided first")

    def _load_constraints(self):
        m = self.__num_nonleaf_nodes
        for i in range(self.__num_nodes):
            if i < m:
                self.__list_of_nonleaf_constraints[i] = core_constraints.No()
            else:
                self.__list_of_leaf_constraints[i] = core_constraints.No()

    def _require_markovian(self, what):
        if not self.__tree.is_markovian:
            raise TypeError(f"{what} provided as Markovian, scenario tree provided is not Markovian")

    # ----- dynamics
    def with_markovian_dynamics(self, ordered_list_of_dynamics):
        first = ordered_list_of_dynamics[0]
        for dyn in ordered_list_of_dynamics:
            if dyn.state_dynamics.shape != first.state_dynamics.shape:
                raise ValueError("Markovian state dynamics matrices are different shapes")
            if dyn.control_dynamics.shape != first.control_dynamics.shape:
                raise ValueError("Markovian control dynamics matrices are different shapes")
        self._require_markovian("dynamics")
        values = self.__tree.values
        for i in range(1, self.__num_nodes):
            self.__list_of_dynamics[i] = ordered_list_of_dynamics[values[i]]
        return self

    # ----- costs
    def with_markovian_nonleaf_costs(self, ordered_list_of_costs):
        if not all(c.node_type.is_nonleaf for c in ordered_list_of_costs):
            raise Exception("Markovian costs provided are not nonleaf")
        self._require_markovian("costs")
        values = self.__tree.values
        # every node j >= 1 (leaves too): L weights the parent's (x, u) with node j's cost
        for i in range(1, self.__num_nodes):
            self.__list_of_nonleaf_costs[i] = ordered_list_of_costs[values[i]]
        return self

    def with_all_nonleaf_costs(self, cost):
        if not cost.node_type.is_nonleaf:
            raise Exception("Nonleaf cost provided is not nonleaf")
        for i in range(1, self.__num_nodes):
            self.__list_of_nonleaf_costs[i] = cost
        return self

    def with_all_leaf_costs(self, cost):
        if not cost.node_type.is_leaf:
            raise Exception("Leaf cost provided is not leaf")
        for i in range(self.__num_nonleaf_nodes, self.__num_nodes):
            self.__list_of_leaf_costs[i] = cost
        return self

    # ----- constraints
    def with_all_nonleaf_constraints(self, nonleaf_constraint):
        self._check_dynamics_before_constraints()
        if not nonleaf_constraint.node_type.is_nonleaf:
            raise Exception("Nonleaf constraint provided is not nonleaf")
        last = self.__list_of_dynamics[-1]
        nonleaf_constraint.state_size = last.state_dynamics.shape[1]
        nonleaf_constraint.control_size = last.control_dynamics.shape[1]
        for i in range(self.__num_nonleaf_nodes):
            self.__list_of_nonleaf_constraints[i] = nonleaf_constraint
        return self

    def with_all_leaf_constraints(self, leaf_constraint):
        self._check_dynamics_before_constraints()
        if not leaf_constraint.node_type.is_leaf:
            raise Exception("Leaf constraint provided is not leaf")
        leaf_constraint.state_size = self.__list_of_dynamics[-1].state_dynamics.shape[1]
        for i in range(self.__num_nonleaf_nodes, self.__num_nodes):
            self.__list_of_leaf_constraints[i] = leaf_constraint
        return self

    # ----- risks
    def with_all_risks(self, risk):
        if not risk.is_risk:
            raise Exception("Risk provided is not of risk type")
        tree = self.__tree
        for i in range(self.__num_nonleaf_nodes):
            node_risk = copy.copy(risk)
            node_risk.probs = tree.conditional_probabilities_of_children(i)
            self.__list_of_risks[i] = node_risk
        return self

    def __str__(self):
        return f"RAOCP\n+ Nodes: {self.__tree.num_nodes}\n" \
               f"+ {self.__list_of_nonleaf_costs[0]}\n" \
               f"+ {self.__list_of_risks[0]}"

    def __repr__(self):
        return f"RAOCP with {self.__tree.num_nodes} nodes, " \
               f"with root cost: {type(self.__list_of_nonleaf_costs[0]).__name__}, " \
               f"with root risk: {type(self.__list_of_risks[0]).__name__}."
