# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Scenario trees and the stopped-Markov-chain factory
(reference: raocp/core/scenario_tree.py:21-351).

The factory here is vectorised per stage (the reference appends node by node
with `np.concatenate`, O(n^2): 99.9 s at 350k nodes) but
produces bit-identical arrays: same BFS node order, same values, and each
probability is the same single product  prob[anc] * P[value[anc], value]
(scenario_tree.py:332-333), or a copy of the ancestor's after the stopping
time (scenario_tree.py:337-339), including the documented length quirk (one
extra entry when tau == N).

Invariants the GPU kernels rely on (checked in `raocp.core._pack`): stage is
non-decreasing in node id, the children of every node form a contiguous
ascending id range, and nonleaf nodes are exactly ids 0..m-1.
"""
import numpy as np

__all__ = ["ScenarioTree", "MarkovChainScenarioTreeFactory"]


def _check_probability_vector(p):
    if abs(sum(p) - 1) >= 1e-10:
        raise ValueError("probability vector does not sum up to 1")
    if any(pi <= -1e-16 for pi in p):
        raise ValueError("probability vector contains negative entries")
    return True


def _check_stopping_time(n, t):
    if t > n:
        raise ValueError("stopping time greater than number of stages")
    return True


class ScenarioTree:
    """Tree of scenarios: node i has ancestor `ancestors[i]` (-1 for the root), stage,
    probability and (for Markov trees) the value of the disturbance w."""

    def __init__(self, stages, ancestors, probability, w_values=None, is_markovian=False):
        self.__is_markovian = is_markovian
        self.__stages = stages
        self.__ancestors = ancestors
        self.__probability = probability
        self.__w_idx = w_values
        self.__children = None
        self.__data = None
        self.__update_children()
        self.__allocate_data()

    def __update_children(self):
        # children_of(i) == np.where(ancestors == i)[0] (scenario_tree.py:45-49), for all i at once
        m = int(self.num_nonleaf_nodes)
        anc = np.asarray(self.__ancestors)
        order = np.argsort(anc, kind="stable")
        keys = anc[order]
        lo = np.searchsorted(keys, np.arange(m), side="left")
        hi = np.searchsorted(keys, np.arange(m), side="right")
        self.__children = [order[lo[i]:hi[i]].astype(np.int64) for i in range(m)]

    def __allocate_data(self):
        self.__data = np.empty(shape=(self.num_nodes,), dtype=dict)

    def get_data_at_node(self, node_idx):
        return self.__data[node_idx]

    def set_data_at_node(self, node_idx, data_dict: dict):
        self.__data[node_idx] = data_dict

    @property
    def is_markovian(self):
        return self.__is_markovian

    @property
    def num_nonleaf_nodes(self):
        return np.sum(self.__stages < (self.num_stages - 1))

    @property
    def num_nodes(self):
        return len(self.__ancestors)

    @property
    def num_stages(self):
        """Number of stages including stage zero."""
        return self.__stages[-1] + 1

    def ancestor_of(self, node_idx):
        return self.__ancestors[node_idx]

    def children_of(self, node_idx):
        return self.__children[node_idx]

    def stage_of(self, node_idx):
        if node_idx < 0:
            raise ValueError("node_idx cannot be <0")
        return self.__stages[node_idx]

    def value_at_node(self, node_idx):
        return self.__w_idx[node_idx]

    def nodes_at_stage(self, stage_idx):
        return np.where(self.__stages == stage_idx)[0]

    def probability_of_node(self, node_idx):
        return self.__probability[node_idx]

    def siblings_of_node(self, node_idx):
        if node_idx == 0:
            return [0]
        return self.children_of(self.ancestor_of(node_idx))

    def conditional_probabilities_of_children(self, node_idx):
        prob_children = self.__probability[self.children_of(node_idx)]
        return prob_children / self.probability_of_node(node_idx)

    # ----- array views used by the device packer (not in the reference API)
    @property
    def ancestors(self):
        return np.asarray(self.__ancestors)

    @property
    def stages(self):
        return np.asarray(self.__stages)

    @property
    def probabilities(self):
        return np.asarray(self.__probability)

    @property
    def values(self):
        return None if self.__w_idx is None else np.asarray(self.__w_idx)

    def __str__(self):
        return f"Scenario Tree\n+ Nodes: {self.num_nodes}\n+ Stages: {self.num_stages}\n" \
               f"+ Scenarios: {len(self.nodes_at_stage(self.num_stages - 1))}\n" \
               f"+ Data: {self.__data is not None}"

    def __repr__(self):
        return f"Scenario tree with {self.num_nodes} nodes, {self.num_stages} stages " \
               f"and {len(self.nodes_at_stage(self.num_stages - 1))} scenarios"

    def bulls_eye_plot(self, dot_size=5, radius=300, filename=None):
        """Bull's eye picture of the tree (reference scenario_tree.py:217-240). Needs a
        display and tkinter; `turtle` is imported lazily so the rest of the package
        works headless."""
        import turtle
        screen = turtle.Screen()
        screen.tracer(0)
        pen = turtle.Turtle(visible=False)
        pen.speed(0)
        n_st = int(self.num_stages)
        arcs = np.zeros(self.num_nodes)

        def circle(r):
            pen.penup(); pen.home(); pen.goto(0, -r); pen.pendown(); pen.circle(r)

        def at(r, arc):
            return r * np.cos(np.deg2rad(arc)), r * np.sin(np.deg2rad(arc))

        pen.pencolor('gray'); circle(radius)
        leaves = self.nodes_at_stage(n_st - 1)
        for k, node in enumerate(leaves):
            arcs[node] = k * 360 / len(leaves)
            pen.penup(); pen.goto(at(radius, arcs[node])); pen.pendown()
            pen.pencolor('black'); pen.dot(dot_size); pen.pencolor('gray')
        step = radius / (n_st - 1)
        for st in range(n_st - 2, -1, -1):
            outer, radius = radius, radius - step
            pen.pencolor('gray'); circle(radius)
            for node in self.nodes_at_stage(st):
                arcs[node] = np.mean(arcs[self.children_of(node)])
                pen.penup(); pen.goto(at(radius, arcs[node])); pen.pendown()
                pen.pencolor('black'); pen.dot(dot_size)
                for ch in self.children_of(node):
                    here = pen.pos(); pen.goto(at(outer, arcs[ch])); pen.goto(here)
                pen.pencolor('gray')
        screen.update()
        if filename is not None:
            screen.getcanvas().postscript(file=filename)
        screen.mainloop()


class MarkovChainScenarioTreeFactory:
    """Scenario tree of a Markov chain with transition matrix P and initial distribution v,
    branching up to the stopping time tau and then carried forward with one child per node."""

    def __init__(self, transition_prob, initial_distribution, num_stages, stopping_time=None):
        self.__factory_type = "MarkovChain"
        if stopping_time is None:
            stopping_time = num_stages
        else:
            _check_stopping_time(num_stages, stopping_time)
        self.__transition_prob = transition_prob
        self.__initial_distribution = initial_distribution
        self.__num_stages = num_stages
        self.__stopping_time = stopping_time
        for row in transition_prob:
            _check_probability_vector(row)
        _check_probability_vector(initial_distribution)

    def __make_ancestors_values_stages(self):
        P = np.asarray(self.__transition_prob)
        v = np.asarray(self.__initial_distribution)
        first = np.flatnonzero(v)
        # support of each row of P, as CSR (cover(i) = flatnonzero(P[i, :]))
        covers = [np.flatnonzero(P[i, :]) for i in range(P.shape[0])]
        cover_len = np.array([len(c) for c in covers], dtype=np.int64)
        cover_off = np.concatenate(([0], np.cumsum(cover_len)))
        cover_flat = np.concatenate(covers).astype(np.int64) if len(covers) else np.zeros(0, np.int64)

        anc_parts = [np.array([-1], dtype=np.int64), np.zeros(len(first), dtype=np.int64)]
        val_parts = [np.array([-1], dtype=np.int64), first.astype(np.int64)]
        stg_parts = [np.array([0], dtype=np.int64), np.ones(len(first), dtype=np.int64)]
        cursor = 1
        level_vals = first.astype(np.int64)
        for stage_idx in range(1, self.__stopping_time):
            cnt = cover_len[level_vals]
            tot = int(cnt.sum())
            parents = np.repeat(np.arange(cursor, cursor + len(level_vals), dtype=np.int64), cnt)
            rank = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(cnt) - cnt, cnt)
            child_vals = cover_flat[np.repeat(cover_off[level_vals], cnt) + rank]
            anc_parts.append(parents)
            val_parts.append(child_vals)
            stg_parts.append(np.full(tot, 1 + stage_idx, dtype=np.int64))
            cursor += len(level_vals)
            level_vals = child_vals
        for stage_idx in range(self.__stopping_time, self.__num_stages):
            k = len(level_vals)
            anc_parts.append(np.arange(cursor, cursor + k, dtype=np.int64))
            val_parts.append(level_vals)
            stg_parts.append(np.full(k, 1 + stage_idx, dtype=np.int64))
            cursor += k
        return np.concatenate(anc_parts), np.concatenate(val_parts), np.concatenate(stg_parts)

    def __make_probability_values(self, ancestors, values, stages):
        P = np.asarray(self.__transition_prob)
        v = np.asarray(self.__initial_distribution)
        nz = np.flatnonzero(v)
        n = len(values)
        tau = self.__stopping_time
        head = np.zeros(len(nz) + 1)
        head[0] = 1
        head[1:] = v[nz]
        if len(nz) + 1 >= n:
            # degenerate tree (no node beyond stage 1): replay scenario_tree.py:327-339 literally
            probs = list(head)
            for j in range(0, n):
                probs.append(probs[ancestors[j]])
            return np.array(probs)
        probs = np.zeros(n)
        probs[:len(nz) + 1] = head
        st = stages
        for t in range(2, int(st[-1]) + 1):
            sel = np.flatnonzero(st == t)
            a = ancestors[sel]
            if t <= tau:
                probs[sel] = probs[a] * P[values[a], values[sel]]
            else:
                probs[sel] = probs[a]
        if not np.any(st == tau + 1):
            # the reference's loop never breaks: it re-appends the last node's ancestor probability
            probs = np.concatenate((probs, [probs[ancestors[n - 1]]]))
        return probs

    def create(self):
        ancestors, values, stages = self.__make_ancestors_values_stages()
        probs = self.__make_probability_values(ancestors, values, stages)
        return ScenarioTree(stages, ancestors, probs, values, is_markovian=True)
