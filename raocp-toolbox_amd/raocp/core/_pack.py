"""Packer: RAOCP problem spec -> flat arrays for the device context (include/raocp_hip.h).

What it produces
  * tree arrays (ancestor, stage, first child, child count) — the kernels rely on
    the BFS, stage-contiguous, contiguous-children numbering that
    MarkovChainScenarioTreeFactory builds (scenario_tree.py:273-315); the C side
    re-validates it;
  * per-mode matrix tables + per-node int32 indices. Tables are deduplicated by
    object identity: the builder shares one Dynamics/Quadratic/Rectangle object
    between all nodes of a mode, so a Markov tree with M modes uploads M matrices,
    not n (the reference keeps a deep copy per node, raocp_spec.py:127-182);
  * AVaR data: alpha and the b-vector entries (conditional probabilities), taken
    from each node's risk object so the device sees the reference's exact doubles;
  * the offline products of the dynamics projection (cache.py:207-233): for every
    nonleaf node R~ = I + sum B'PB, K = -R~^-1 sum B'PA, Abar_j = A_j + B_j K,
    P = I + K'K + sum Abar'P Abar, plus M = K' + sum Abar'PB. Nodes whose subtrees
    have the same signature (same child dynamics, same child classes) get
    bit-identical results, so they are computed once per class (SURVEY.md 8(f)
    row 2) with the reference's numpy/scipy calls (cho_factor / cho_solve).
"""
import numpy as np
import scipy.linalg

import raocp.core.risks as risks
import raocp.core.constraints.rectangle as rectangle

__all__ = ["PackedProblem", "pack_problem"]


class _Table:
    """Deduplicating matrix table keyed by object identity (and, with by_value, by the
    matrix's bytes: per-mode cost objects holding equal weights share one entry, so the
    L / L^T kernels see one table row where the modes' weights coincide)."""

    def __init__(self, shape, strict=True, by_value=False):
        self.shape = shape
        self.mats = []
        self._ids = {}
        self._vals = {} if by_value else None
        self.strict = strict
        self.mismatch = None

    def index(self, mat):
        key = id(mat)
        if key not in self._ids:
            arr = np.asarray(mat, dtype=np.float64)
            if arr.shape != self.shape:
                msg = f"matrix of shape {arr.shape} where {self.shape} is required"
                if self.strict:
                    raise ValueError(msg)
                # L / L^T weights may be inconsistent as long as L is never applied: the
                # reference's own tests build such problems (tests/test_cache.py:35-54)
                self.mismatch = self.mismatch or msg
                arr = np.full(self.shape, np.nan)
            arr = np.ascontiguousarray(arr)
            vkey = arr.tobytes() if self._vals is not None and not np.isnan(arr).any() else None
            if vkey is not None and vkey in self._vals:
                self._ids[key] = self._vals[vkey]
            else:
                self._ids[key] = len(self.mats)
                self.mats.append(arr)
                if vkey is not None:
                    self._vals[vkey] = self._ids[key]
        return self._ids[key]

    def array(self):
        if not self.mats:
            return np.zeros((1,) + self.shape)
        return np.ascontiguousarray(np.stack(self.mats))


class PackedProblem:
    """Arrays in the layout of raocp_tree_desc / raocp_problem_desc (int32 / float64, C-contiguous)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def _i32(a):
    return np.ascontiguousarray(np.asarray(a), dtype=np.int32)


def _f64(a):
    return np.ascontiguousarray(np.asarray(a), dtype=np.float64)


def pack_problem(spec):
    tree = spec.tree
    n = int(tree.num_nodes)
    m = int(tree.num_nonleaf_nodes)
    nx = spec.state_dynamics_at_node(1).shape[1]
    nu = spec.control_dynamics_at_node(1).shape[1]
    anc = tree.ancestors.astype(np.int64)
    stage = tree.stages.astype(np.int64)
    ch_start = np.zeros(m, dtype=np.int64)
    nch = np.zeros(m, dtype=np.int64)
    for i in range(m):
        ch = tree.children_of(i)
        if len(ch) == 0:
            raise ValueError(f"nonleaf node {i} has no children")
        ch_start[i] = ch[0]
        nch[i] = len(ch)
        if ch[-1] - ch[0] + 1 != len(ch):
            raise ValueError("children must form a contiguous id range (BFS numbering)")
    rank = np.zeros(n, dtype=np.int64)
    for i in range(m):
        rank[ch_start[i]:ch_start[i] + nch[i]] = np.arange(nch[i])

    # ---- L / L^T weights
    t_sq, t_sr, t_sp = (_Table((nx, nx), False, True), _Table((nu, nu), False, True),
                        _Table((nx, nx), False, True))
    i_sq = np.zeros(n, dtype=np.int64)
    i_sr = np.zeros(n, dtype=np.int64)
    i_sp = np.zeros(n, dtype=np.int64)
    t_a, t_b = _Table((nx, nx)), _Table((nx, nu))
    i_a = np.zeros(n, dtype=np.int64)
    i_b = np.zeros(n, dtype=np.int64)
    for j in range(1, n):
        cost = spec.nonleaf_cost_at_node(j)
        i_sq[j] = t_sq.index(cost.sqrt_state_weights)
        i_sr[j] = t_sr.index(cost.sqrt_control_weights)
        i_a[j] = t_a.index(spec.state_dynamics_at_node(j))
        i_b[j] = t_b.index(spec.control_dynamics_at_node(j))
    for l in range(m, n):
        i_sp[l] = t_sp.index(spec.leaf_cost_at_node(l).sqrt_state_weights)

    # ---- risks (cache.py:172-182: only AVaR is supported)
    alpha_r = np.zeros(m)
    cond = np.zeros(n)
    for i in range(m):
        r = spec.risk_at_node(i)
        if type(r) is not risks.AVaR:
            raise Exception(f"Risk at node {i} not defined")
        b = np.asarray(r.vector_b, dtype=np.float64).reshape(-1)
        if b.size != 2 * nch[i] + 1:
            raise ValueError(f"risk at node {i} has {b.size} entries for {nch[i]} children")
        alpha_r[i] = r.alpha
        cond[ch_start[i]:ch_start[i] + nch[i]] = b[:nch[i]]

    # ---- boxes
    def box_index(cons, rows, table, ids):
        if not cons.is_active:
            return -1
        if not isinstance(cons, rectangle.Rectangle):
            raise NotImplementedError(f"{type(cons).__name__} constraints are not supported by the HIP path")
        key = id(cons)
        if key not in ids:
            lo, hi = np.asarray(cons.lower).reshape(-1), np.asarray(cons.upper).reshape(-1)
            if lo.size != rows:
                raise Exception("Rectangle constraint - input vector does not equal expected size")
            if any(v is None for v in lo) or any(v is None for v in hi):
                raise TypeError("Rectangle constraint with a None bound cannot be projected")
            ids[key] = len(table)
            table.append((lo.astype(np.float64), hi.astype(np.float64)))
        return ids[key]

    box_nl, box_l, ids_nl, ids_l = [], [], {}, {}
    i_box_nl = np.array([box_index(spec.nonleaf_constraint_at_node(i), nx + nu, box_nl, ids_nl) for i in range(m)],
                        dtype=np.int64)
    i_box_l = np.full(n, -1, dtype=np.int64)
    for l in range(m, n):
        i_box_l[l] = box_index(spec.leaf_constraint_at_node(l), nx, box_l, ids_l)

    # ---- offline dynamics products per subtree class (cache.py:207-233)
    # For the device sweep (raocp_dyn.hip) the backward recursion is re-associated as
    #   h = sum_j B_j' q_j,  a = sum_j A_j' q_j,  d = Rinv (u - h),
    #   q = (-x + K'(h - u)) + a + M d,   M = K' + sum_j Abar_j' P_j B_j
    # and the forward one as x_j = A_j x + B_j u (u = K x + d), so only the per-mode
    # A, B and per-class Rinv, K, M are needed. Classes are numbered by stage.
    I_x, I_u = np.eye(nx), np.eye(nu)
    A_tab, B_tab = t_a.array(), t_b.array()
    cls = np.full(n, -1, dtype=np.int64)   # -1: leaf (P = I)
    P_cls, K_cls, Rinv_cls, M_cls, stage_cls = [], [], [], [], []
    memo = {}

    def P_of(j):
        return I_x if cls[j] < 0 else P_cls[cls[j]]

    for i in range(m - 1, -1, -1):
        kids = range(ch_start[i], ch_start[i] + nch[i])
        key = tuple((int(i_a[j]), int(i_b[j]), int(cls[j])) for j in kids)
        ci = memo.get(key)
        if ci is None:
            sum_r, sum_k = 0, 0
            for j in kids:
                Bj, Aj, Pj = B_tab[i_b[j]], A_tab[i_a[j]], P_of(j)
                sum_r = sum_r + Bj.T @ Pj @ Bj
                sum_k = sum_k + Bj.T @ Pj @ Aj
            cho = scipy.linalg.cho_factor(I_u + sum_r)
            K = scipy.linalg.cho_solve(cho, -sum_k)
            sum_p = 0
            Mc = K.T.copy()
            for j in kids:
                Bj, Aj, Pj = B_tab[i_b[j]], A_tab[i_a[j]], P_of(j)
                Ab = Aj + Bj @ K
                sum_p = sum_p + Ab.T @ Pj @ Ab
                Mc = Mc + Ab.T @ (Pj @ Bj)
            ci = len(P_cls)
            memo[key] = ci
            P_cls.append(I_x + K.T @ K + sum_p)
            K_cls.append(K)
            Rinv_cls.append(scipy.linalg.cho_solve(cho, I_u))
            M_cls.append(Mc)
            stage_cls.append(int(stage[i]))
        cls[i] = ci
    # renumber classes by stage (a class is stage-specific: equal subtree signature => equal height)
    order = np.argsort(np.asarray(stage_cls), kind="stable")
    new_id = np.empty(len(order), dtype=np.int64)
    new_id[order] = np.arange(len(order))
    i_k = new_id[cls[:m]]
    K_tab = _f64(np.stack([K_cls[o] for o in order]))
    Rinv_tab = _f64(np.stack([Rinv_cls[o] for o in order]))
    M_tab = _f64(np.stack([M_cls[o] for o in order]))
    class_stage = np.asarray(stage_cls, dtype=np.int64)[order]

    def stack(lst, shape):
        return _f64(np.stack(lst)) if lst else np.zeros((1,) + shape)

    def boxes(table, rows):
        if not table:
            return np.zeros((1, rows)), np.zeros((1, rows))
        return _f64([t[0] for t in table]), _f64([t[1] for t in table])

    lo_nl, hi_nl = boxes(box_nl, nx + nu)
    lo_l, hi_l = boxes(box_l, nx)
    return PackedProblem(
        n=n, m=m, nx=nx, nu=nu, N=int(stage[-1]),
        anc=_i32(anc), stage=_i32(stage), ch_start=_i32(ch_start), nch=_i32(nch), rank=_i32(rank),
        sqrt_q=t_sq.array(), sqrt_r=t_sr.array(), sqrt_pf=t_sp.array(),
        i_sq=_i32(i_sq), i_sr=_i32(i_sr), i_sp=_i32(i_sp),
        alpha_r=_f64(alpha_r), cond=_f64(cond),
        n_box_nl=len(box_nl), n_box_l=len(box_l), box_nl_lo=lo_nl, box_nl_hi=hi_nl, box_l_lo=lo_l, box_l_hi=hi_l,
        i_box_nl=_i32(i_box_nl), i_box_l=_i32(i_box_l),
        A=A_tab, B=B_tab, K=K_tab, Rinv=Rinv_tab, M=M_tab,
        i_a=_i32(i_a), i_b=_i32(i_b), i_k=_i32(i_k), class_stage=_i32(class_stage),
        n_classes=len(order),
        l_error=t_sq.mismatch or t_sr.mismatch or t_sp.mismatch,
    )
