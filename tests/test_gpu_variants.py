"""GPU parity of the kernel variants kept selectable: the eager stopping test after every
iteration (RAOCP_DEFER_CHECK=0) against the default deferred one; the block L^T kernel
k_ell_t against the oracle; the streaming L^T (k_ellt3, default on
uniform trees) against the block kernel (RAOCP_ELLT3=0) and the oracle.

Tolerances as in test_gpu_parity.py.
"""
import os

import numpy as np
import pytest

import raocp.core as core
from raocp.problems import build_problem, recipe_config
from helpers import problem_from_golden, rel_err, trace_rel_err

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


@pytest.mark.parametrize("iters,stop", [(0, None), (1, None), (23, None), (24, None), (30, None), (60, 37), (60, 24)])
def test_deferred_stopping_test_matches_eager(iters, stop):
    """The default deferred stopping test (iteration k's test in an extra workgroup of
    iteration k + 1's first dynamics launch, one k_cp_check per graph batch) against
    k_cp_check after every iteration: same status, iteration count, history and final
    iterate, bit for bit, at batch boundaries (24 iterations per graph) and on early stops."""
    r = recipe_config(2)
    tree, prob = build_problem(r)
    dfr = core.Cache(prob)
    eag = _with_env({"RAOCP_DEFER_CHECK": "0"}, lambda: core.Cache(prob))
    alpha = 0.999 / dfr.native.step_size()
    tol = 0.0
    if stop is not None:  # a tolerance the run meets at iteration `stop` (or before)
        _, err, _ = eag.native.cp_run(r["x0"], iters, 0.0, alpha)
        tol = float(err[stop].max())
    out = []
    for cache in (dfr, eag):
        status, err, derr = cache.native.cp_run(r["x0"], iters, tol, alpha)
        out.append((status, err, derr, cache.get_primal_flat(), cache.get_dual_flat()))
    (s1, e1, d1, z1, y1), (s2, e2, d2, z2, y2) = out
    assert s1 == s2 and e1.shape == e2.shape
    assert np.array_equal(e1, e2) and np.array_equal(d1, d2)
    assert np.array_equal(z1, z2) and np.array_equal(y1, y2)
    if stop is not None:
        assert s1 == 0 and e1.shape[0] <= stop + 1  # stopped early


@pytest.mark.parametrize("cfg", [2, 3, 4, "4-modes"])
def test_ell_t_block_kernel_matches_oracle(cfg):
    """k_ell_t (RAOCP_ELLT3=0): per-parent MFMA tiles on regular blocks, the LDS-staged product
    path where a block mixes weight tables (config 4-modes), against the oracle."""
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(4 if cfg == "4-modes" else cfg)
    if cfg == "4-modes":
        r["Q"] = np.array([(1.0 + k) * q for k, q in enumerate(r["Q"])])
    tree, prob = build_problem(r)
    blk = _with_env({"RAOCP_ELLT3": "0"}, lambda: core.Cache(prob))
    rng = np.random.default_rng(11)
    ee = rng.standard_normal(blk.dual_size)
    assert rel_err(blk.native.ell_t(ee), OracleProblem(prob).ell_t(ee)) <= 1e-12


@pytest.mark.parametrize("cfg", ["chain", 2, "2-nobox", "2-leafbox", 4, "4-c2", "stop", "stop-nobox"])
def test_ell_t_streaming_vs_block_and_oracle(cfg):
    """k_ellt3 (streaming wave tasks, uniform tables and branching C <= 4; raocp_ell3.hip)
    against k_ell_t (RAOCP_ELLT3=0) and the oracle (operators.py:55-94) on random duals:
    a chain (C = 1), config 2 (C = 2) with all, no and leaf-only boxes (eta7 / eta14 terms),
    config 4 (C = 3, nx = 32) and a binary tree at nx = 32. The same for L (k_ell3 against
    k_ell, operators.py:19-53), and both with the eta7 / eta14 offsets read from the tables
    (RAOCP_BOX_MODE=0) instead of computed from the all / none box patterns. "stop": a binary
    tree whose stopping time (4) is below the horizon (10), so the branching is not uniform:
    k_ell3 takes its child-tile branch (eta7 from the flat tasks) and L^T runs k_ell_t."""
    from oracle.raocp_oracle import OracleProblem
    from raocp.problems import recipe_synthetic
    if cfg == "chain":
        r = recipe_synthetic(np.ones((1, 1)), np.ones(1), 40, 40, 20, 8, seed=3)
    elif cfg == "4-c2":
        r = recipe_synthetic(np.full((2, 2), .5), np.full(2, .5), 9, 9, 32, 12, seed=4)
    elif cfg in ("stop", "stop-nobox"):
        r = recipe_synthetic(np.full((2, 2), .5), np.full(2, .5), 10, 4, 20, 8, seed=5)
        if cfg == "stop-nobox":
            r["nl_min"] = r["nl_max"] = None
    elif cfg in ("2-nobox", "2-leafbox"):
        r = recipe_config(2)
        r["nl_min"] = r["nl_max"] = None
        if cfg == "2-nobox":
            r["l_min"] = r["l_max"] = None
    else:
        r = recipe_config(cfg)
    tree, prob = build_problem(r)
    stream = core.Cache(prob)
    block = _with_env({"RAOCP_ELLT3": "0"}, lambda: core.Cache(prob))
    rng = np.random.default_rng(12)
    ee = rng.standard_normal(stream.dual_size)
    a, b = stream.native.ell_t(ee), block.native.ell_t(ee)
    ref = OracleProblem(prob).ell_t(ee)
    assert rel_err(a, ref) <= 1e-12 and rel_err(a, b) <= 1e-12
    # tau_0 is never written (operators.py:55-94 writes tau_j for children only)
    tmpl = rng.standard_normal(stream.primal_size)
    a2 = stream.native.ell_t(ee, template=tmpl)
    pk = stream.packed
    t0 = pk.n * pk.nx + pk.m * pk.nu + int(np.sum(2 * pk.nch[:pk.m] + 1))  # flat index of tau_0
    assert a2[t0] == tmpl[t0]
    keep = np.ones(a2.size, bool)
    keep[t0] = False
    assert np.array_equal(a2[keep], a[keep])
    tabs = _with_env({"RAOCP_BOX_MODE": "0"}, lambda: core.Cache(prob))
    assert np.array_equal(tabs.native.ell_t(ee), a)
    zz = rng.standard_normal(stream.primal_size)
    lz = stream.native.ell(zz)
    assert rel_err(lz, OracleProblem(prob).ell(zz)) <= 1e-12
    assert np.array_equal(tabs.native.ell(zz), lz)
    blk = _with_env({"RAOCP_ELL3": "0"}, lambda: core.Cache(prob))
    assert rel_err(blk.native.ell(zz), lz) <= 1e-12
