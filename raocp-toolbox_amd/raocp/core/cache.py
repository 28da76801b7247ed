# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Cache: the prox oracle of the CP loop (reference: raocp/core/cache.py:8-393).

Same public methods and block-list conventions as the reference, but the
iterate lives in HBM inside a `libraocp_hip.so` context and every operator is a
HIP kernel launch (include/raocp_hip.h). The block lists handed to / returned
by the methods are converted to/from the reference's flat order (np.vstack of
the blocks, placeholders included) at this boundary only.

Differences from the reference (documented in DESIGN.md):
  * no per-iteration history: `update_cache` keeps the latest iterate as the
    "old" one (cache.py:186-196 appends the whole primal and dual lists every
    iteration, 1.17 GB after 20 iterations at 8k nodes);
    `_Cache__primal_cache` / `_Cache__dual_cache` hold iteration 0 only;
  * the AVaR kernel projection uses its closed form (Sherman-Morrison) instead of
    `null_space` + `lstsq`; `get_kernel_constraint_matrices` /
    `get_nullspace_matrices` still build the reference's matrices on demand.
"""
import numpy as np
import scipy.linalg

import raocp.core.raocp_spec as ps
from raocp.core import _native
from raocp.core._pack import pack_problem

__all__ = ["Cache"]


def _flatten(blocks):
    return np.concatenate([np.asarray(b, dtype=np.float64).reshape(-1) for b in blocks])


class Cache:
    """Oracle of functions for solving RAOCPs using proximal algorithms (HIP-backed)."""

    def __init__(self, problem_spec: ps.RAOCP, device=None, dtype="float64"):
        self.__raocp = problem_spec
        tree = problem_spec.tree
        self.__num_nodes = n = int(tree.num_nodes)
        self.__num_nonleaf_nodes = m = int(tree.num_nonleaf_nodes)
        self.__num_leaf_nodes = n - m
        self.__num_stages = tree.num_stages
        self.__state_size = nx = problem_spec.state_dynamics_at_node(1).shape[1]
        self.__control_size = nu = problem_spec.control_dynamics_at_node(1).shape[1]
        self.__initial_state = None
        self.__packed = pack_problem(problem_spec)
        # dtype (extension): "float32" runs the iterate, tables and products in fp32
        # (BASELINE configs[4]); vectors still cross this API as float64
        self.__ctx = _native.NativeContext(self.__packed, device=device, dtype=dtype)

        # block shapes of the reference's lists (cache.py:126-170)
        nch = self.__packed.nch.astype(np.int64)
        self.__segment_p = [None, 0, n, n + m, n + 2 * m, 2 * n + 2 * m, 3 * n + 2 * m]
        self.__segment_d = [None, 0, n, 2 * n, 3 * n, 4 * n, 5 * n, 6 * n, 7 * n, None, None,
                            7 * n, 8 * n, 9 * n, 10 * n, 11 * n]
        p_sizes = np.ones(3 * n + 2 * m, dtype=np.int64)
        p_sizes[0:n] = nx
        p_sizes[n:n + m] = nu
        p_sizes[n + m:n + 2 * m] = 2 * nch + 1
        d_sizes = np.ones(11 * n, dtype=np.int64)
        d_sizes[0:m] = 2 * nch + 1
        d_sizes[2 * n + 1:3 * n] = nx
        d_sizes[3 * n + 1:4 * n] = nu
        for i in range(m):
            if problem_spec.nonleaf_constraint_at_node(i).is_active:
                d_sizes[6 * n + i] = problem_spec.nonleaf_constraint_at_node(i).state_matrix.shape[0]
        d_sizes[7 * n + m:8 * n] = nx
        for i in range(m, n):
            if problem_spec.leaf_constraint_at_node(i).is_active:
                d_sizes[10 * n + i] = problem_spec.leaf_constraint_at_node(i).state_matrix.shape[0]
        self.__p_sizes, self.__d_sizes = p_sizes, d_sizes
        self.__p_split = np.cumsum(p_sizes)[:-1]
        self.__d_split = np.cumsum(d_sizes)[:-1]
        assert int(p_sizes.sum()) == self.__ctx.P and int(d_sizes.sum()) == self.__ctx.D

        self.__old_primal_flat = np.zeros(self.__ctx.P)
        self.__old_dual_flat = np.zeros(self.__ctx.D)
        self.__primal_cache = [self._blocks_p(self.__old_primal_flat)]
        self.__dual_cache = [self._blocks_d(self.__old_dual_flat)]
        self.__kernel_constraint_matrix = None
        self.__null_space_matrix = None

    # ----- flat <-> blocks
    def _blocks_p(self, flat):
        return [b.reshape(-1, 1) for b in np.split(np.asarray(flat, dtype=np.float64), self.__p_split)]

    def _blocks_d(self, flat):
        return [b.reshape(-1, 1) for b in np.split(np.asarray(flat, dtype=np.float64), self.__d_split)]

    @property
    def native(self):
        """The device context (raocp.core._native.NativeContext)."""
        return self.__ctx

    @property
    def packed(self):
        return self.__packed

    @property
    def primal_size(self):
        return self.__ctx.P

    @property
    def dual_size(self):
        return self.__ctx.D

    # ----- getters (cache.py:56-75)
    def get_raocp(self):
        return self.__raocp

    def get_primal(self):
        return self._blocks_p(self.__ctx.get_primal()), self._blocks_p(self.__old_primal_flat)

    def get_primal_segments(self):
        return self.__segment_p.copy()

    def get_dual(self):
        return self._blocks_d(self.__ctx.get_dual()), self._blocks_d(self.__old_dual_flat)

    def get_dual_segments(self):
        return self.__segment_d.copy()

    def get_kernel_constraint_matrices(self):
        self._build_kernel_matrices()
        return self.__kernel_constraint_matrix.copy()

    def get_nullspace_matrices(self):
        self._build_kernel_matrices()
        return self.__null_space_matrix.copy()

    def _build_kernel_matrices(self):
        # offline_projection_kernel (cache.py:235-242), only for API parity
        if self.__kernel_constraint_matrix is not None:
            return
        K, N = [], []
        for i in range(self.__num_nonleaf_nodes):
            risk = self.__raocp.risk_at_node(i)
            c = len(self.__raocp.tree.children_of(i))
            eye = np.eye(c)
            zeros = np.zeros((risk.matrix_f.shape[1], c))
            row1 = np.hstack((risk.matrix_e.T, -eye, -eye))
            row2 = np.hstack((risk.matrix_f.T, zeros, zeros))
            K.append(np.vstack((row1, row2)))
            N.append(scipy.linalg.null_space(K[-1]))
        self.__kernel_constraint_matrix, self.__null_space_matrix = K, N

    # ----- setters (cache.py:79-122)
    def cache_initial_state(self, state):
        self.__initial_state = state
        x0 = np.asarray(state, dtype=np.float64).reshape(-1)
        self.__old_primal_flat[:self.__state_size] = x0
        self.__primal_cache[0][0] = state
        self.__ctx.set_initial_state(x0)

    def _locate(self, i, segments, active):
        for s in reversed(active):
            if i >= segments[s]:
                return s, i - segments[s]
        return None, None

    def set_primal(self, candidate_primal):
        if len(candidate_primal) != len(self.__p_sizes):
            raise Exception("Candidate primal list is wrong length")
        for i, blk in enumerate(candidate_primal):
            shape = np.shape(blk)
            if shape != (int(self.__p_sizes[i]), 1):
                # the reference looks the index up in the DUAL segments (cache.py:90-95)
                segment, node = self._locate(i, self.__segment_d, range(1, 6))
                raise Exception(f"Candidate primal array shape error in segment {segment} at node {node},\n"
                                f"candidate shape: {shape},\n"
                                f"current shape: {(int(self.__p_sizes[i]), 1)}")
        self.__ctx.set_primal(_flatten(candidate_primal))

    def set_dual(self, candidate_dual):
        if len(candidate_dual) != len(self.__d_sizes):
            raise Exception("Candidate dual list is wrong length")
        for i, blk in enumerate(candidate_dual):
            shape = np.shape(blk)
            if shape != (int(self.__d_sizes[i]), 1):
                active = [s for s in range(1, 15) if s not in (8, 9, 10)]
                segment, node = self._locate(i, self.__segment_d, active)
                raise Exception(f"Candidate dual array shape error in segment {segment} at node {node},\n"
                                f"candidate shape: {shape},\n"
                                f"current shape: {(int(self.__d_sizes[i]), 1)}")
        self.__ctx.set_dual(_flatten(candidate_dual))

    def set_primal_flat(self, z):
        self.__ctx.set_primal(z)

    def set_dual_flat(self, eta):
        self.__ctx.set_dual(eta)

    def get_primal_flat(self):
        return self.__ctx.get_primal()

    def get_dual_flat(self):
        return self.__ctx.get_dual()

    def update_cache(self):
        """The current iterate becomes the 'old' one (cache.py:186-196, without history)."""
        self.__old_primal_flat = self.__ctx.get_primal()
        self.__old_dual_flat = self.__ctx.get_dual()

    def seed_device_iterate(self):
        """Load the 'old' primal / dual (the iterate the reference's CP loop continues from,
        cache.py:58-66) into the device context before a solve."""
        self.__ctx.set_primal(self.__old_primal_flat)
        self.__ctx.set_dual(self.__old_dual_flat)

    def _set_old(self, z, eta):
        self.__old_primal_flat = np.asarray(z, dtype=np.float64).copy()
        self.__old_dual_flat = np.asarray(eta, dtype=np.float64).copy()

    # ----- prox of f (cache.py:248-317)
    def proximal_of_f(self, solver_parameter):
        self.proximal_of_relaxation_s_at_stage_zero(solver_parameter)
        self.project_on_dynamics()
        self.project_on_kernel()

    def proximal_of_relaxation_s_at_stage_zero(self, solver_parameter):
        self.__ctx.relax_s0(float(np.asarray(solver_parameter).reshape(-1)[0]))

    def project_on_dynamics(self):
        self.__ctx.project_on_dynamics()

    def project_on_kernel(self):
        self.__ctx.project_on_kernel()

    # ----- prox of g* (cache.py:321-393)
    def proximal_of_g_conjugate(self, solver_parameter):
        self.__ctx.prox_gconj(float(solver_parameter))

    def modify_dual(self, solver_parameter):
        self.__ctx.dual_scale(float(solver_parameter))

    def add_halves(self):
        self.__ctx.dual_add_halves()

    def project_on_constraints_nonleaf(self):
        self.__ctx.dual_project(1)

    def project_on_constraints_leaf(self):
        self.__ctx.dual_project(2)

    def modify_projection(self, solver_parameter, modified_dual):
        self.__ctx.dual_moreau(float(solver_parameter), _flatten(modified_dual))
