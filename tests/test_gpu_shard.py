"""GPU: subtree sharding — R shards of one tree, each owning a block of
the subtrees below the replicated top, exchanging the roots' q rows, the roots' eta2 /
xi2 entries and the residual maxima each iteration. Here the shards share the one
device of the test box and exchange through device copies (raocp_group_cp_run); the
multi-GPU transport is RCCL with the same packing (bench.py --shard).

Parity: the residual histories and the owned parts of the final iterate equal those of
the unsharded solve on the same dynamics and CP kernels -- the fused k_cp3 (a shard runs it as two
launches around X1, the cut's parents reading their children's eta2 entries from the
exchange) or the two-launch k_cpd* / k_cpp* (RAOCP_CP3=0) -- bit for bit: the per-node
arithmetic is identical and only max reductions are regrouped, which is exact. The two
kernel families agree within 1e-10 and match the oracle within the north_star tolerance.
Configs 2 (the headline tree) and 4 (the tree the sharded bench leg runs, BASELINE
configs[3]) at R = 2, 4, 8; config 5 in fp32 (BASELINE configs[4]) at R = 2, 4.
"""
import os

import numpy as np
import pytest

import raocp.core as core
from raocp.core._native import group_cp_run
from raocp.problems import build_problem, recipe_config

pytestmark = pytest.mark.gpu


def _cache(cfg):
    r = recipe_config(cfg, seed=0)
    tree, prob = build_problem(r)
    return r, tree, prob


@pytest.fixture(scope="module")
def c2():
    return _cache(2)


def _kern_cache(prob, kern, dtype=None):
    """A context on the fused CP kernel k_cp3 ("fused", the default) or the two-launch
    k_cpd* / k_cpp* ("two", RAOCP_CP3=0)."""
    # the dynamics a shard runs (the tiered sweep; fp32 / config 4: dyn3) and the CP kernel it
    # runs (k_cp3: a shard's task list; the unsharded defaults at config 2 / configs 4, 5 are
    # k_cp6 / k_cp5, the same arithmetic with a different FMA contraction, test_gpu_cp6.py,
    # test_gpu_cp5.py)
    env = {"RAOCP_DR": "0", "RAOCP_CP4": "0", "RAOCP_CP5": "0", "RAOCP_CP6": "0"}
    if kern == "two":
        env["RAOCP_CP3"] = "0"
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return core.Cache(prob, dtype=dtype) if dtype else core.Cache(prob)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _two_launch_cache(prob):
    return _kern_cache(prob, "two")


_ORACLE = {}


def _oracle_run(cfg, prob, x0, iters, alpha):
    from oracle.raocp_oracle import OracleProblem
    key = (cfg, iters, alpha)
    if key not in _ORACLE:
        _ORACLE[key] = OracleProblem(prob).chock(x0, iters, 0.0, alpha=alpha)
    return _ORACLE[key]


def _owned_x_slices(ctx):
    lo, hi = ctx.shard_owned()
    return [(int(a), int(b)) for a, b in zip(lo, hi)]


_CFG = {}


@pytest.mark.parametrize("kern", ["fused", "two"])
@pytest.mark.parametrize("cfg", [2, 4])
@pytest.mark.parametrize("R", [2, 4, 8])
def test_sharded_solve_matches_unsharded(cfg, R, kern):
    if cfg not in _CFG:
        _CFG[cfg] = _cache(cfg)
    r, tree, prob = _CFG[cfg]
    base = _kern_cache(prob, kern)
    assert base.native.kernel_info(10).startswith(("k_cp3", "k_cp4")) == (kern == "fused")
    lam = base.native.step_size()
    alpha = 0.999 / lam
    iters = 40 if cfg == 2 else 12
    st0, err0, derr0 = base.native.cp_run(r["x0"], iters, 0.0, alpha)
    z0 = base.get_primal_flat()
    other = _kern_cache(prob, "two" if kern == "fused" else "fused")
    stf, errf, _ = other.native.cp_run(r["x0"], iters, 0.0, alpha)
    assert stf == st0 and np.max(np.abs(errf - err0) / np.abs(err0)) <= 1e-10
    # the unsharded default (config 2: the regular-tree sweep k_dr)
    dflt = core.Cache(prob)
    std, errd, _ = dflt.native.cp_run(r["x0"], iters, 0.0, alpha)
    assert std == st0 and np.max(np.abs(errd - err0) / np.abs(err0)) <= 1e-10
    st_o, err_o, _, z_o, _, _ = _oracle_run(cfg, prob, r["x0"], iters, alpha)
    assert np.max(np.abs(err0 - err_o) / np.abs(err_o)) <= 1e-8
    assert np.max(np.abs(z0 - z_o)) <= 1e-10 * np.max(np.abs(z_o))
    shards = [_kern_cache(prob, kern) for _ in range(R)]
    for k, s in enumerate(shards):
        s.native.shard(k, R)
    st, err, derr = group_cp_run([s.native for s in shards], r["x0"], iters, 0.0, alpha)
    assert st == st0 and err.shape == err0.shape
    assert np.array_equal(err, err0)
    assert np.array_equal(derr, derr0)
    nx = base.packed.nx
    covered = np.zeros(tree.num_nodes, dtype=bool)
    for s in shards:
        z = s.get_primal_flat()
        for (a, b) in _owned_x_slices(s.native):
            if b > a:
                np.testing.assert_array_equal(z[a * nx:b * nx], z0[a * nx:b * nx])
                covered[a:b] = True
    assert covered.all()


def test_sharded_stopping_and_status(c2):
    """The stopping test sees the all-reduced residuals: every shard stops together at
    the same iteration as the unsharded solve (tolerance reached before max_iters)."""
    r, tree, prob = c2
    base = _two_launch_cache(prob)
    alpha = 0.999 / base.native.step_size()
    st0, err0, _ = base.native.cp_run(r["x0"], 400, 5e-2, alpha)
    shards = [_two_launch_cache(prob) for _ in range(2)]
    for k, s in enumerate(shards):
        s.native.shard(k, 2)
    st, err, _ = group_cp_run([s.native for s in shards], r["x0"], 400, 5e-2, alpha)
    assert (st, err.shape) == (st0, err0.shape)
    assert np.array_equal(err, err0)


def test_shard_setup_rejects_small_trees():
    r, tree, prob = _cache(1)
    c = core.Cache(prob)
    with pytest.raises(Exception):
        c.native.shard(0, 2)


def test_rccl_transport_single_rank():
    """The RCCL exchange path (all-gathers + all-reduce inside the captured graph) with one
    forced shard reproduces the unsharded solve bit for bit. Own process: torch must not
    be loaded next to the RCCL the library binds (bench.py SocketGroup)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("RAOCP_SHARD_FORCE", None)
    res = subprocess.run([sys.executable, os.path.join(root, "tools", "rccl_single_rank.py")], capture_output=True,
                         text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert "bit-identical" in res.stdout


@pytest.mark.parametrize("kern", ["fused", "two"])
@pytest.mark.parametrize("R", [2, 4, 8])
def test_fp32_sharded_config5_matches_unsharded(R, kern):
    """BASELINE configs[4] ("fp32, 8 x MI355X"): one config-5 tree in fp32 split across R
    shards. The per-stage streaming sweep (raocp_dyn3.hip) runs the owned parents of every
    stage below the cut and the replicated top, exchanging the roots' q rows (X2, fp32);
    the CP kernels (k_cp3<float> in two launches, or k_cpd2 / k_cpp2<float>) run the owned
    families with the X1 exchange. The residual history and the owned iterate equal the
    unsharded fp32 solve on the same kernels bit for bit (only max reductions are
    regrouped); the two kernel families agree to fp32 rounding (1e-4 per trace entry)."""
    r = recipe_config(5, seed=0)
    tree, prob = build_problem(r)
    base = _kern_cache(prob, kern, "float32")
    shards = [_kern_cache(prob, kern, "float32") for _ in range(R)]
    assert base.native.kernel_info(9).startswith("k_dy3_back<float")
    alpha = 0.999 / base.native.step_size(rtol=1e-7)
    iters = 6
    st0, err0, derr0 = base.native.cp_run(r["x0"], iters, 0.0, alpha)
    z0 = base.get_primal_flat()
    for k, s in enumerate(shards):
        s.native.shard(k, R)
    st, err, derr = group_cp_run([s.native for s in shards], r["x0"], iters, 0.0, alpha)
    assert st == st0 and err.shape == err0.shape == (iters + 1, 3)
    assert np.array_equal(err, err0) and np.array_equal(derr, derr0)
    nx = base.packed.nx
    covered = np.zeros(tree.num_nodes, dtype=bool)
    for s in shards:
        z = s.get_primal_flat()
        for (a, b) in _owned_x_slices(s.native):
            if b > a:
                np.testing.assert_array_equal(z[a * nx:b * nx], z0[a * nx:b * nx])
                covered[a:b] = True
    assert covered.all()
    other = _kern_cache(prob, "two" if kern == "fused" else "fused", "float32")
    stf, errf, _ = other.native.cp_run(r["x0"], iters, 0.0, alpha)
    assert stf == st0 and np.max(np.abs(errf - err0) / np.abs(err0)) <= 1e-4


@pytest.mark.parametrize("R", [2, 4, 8])
@pytest.mark.parametrize("cfg,dtype", [(4, "float64"), (5, "float32")])
def test_sharded_default_kernels_match_unsharded(cfg, dtype, R):
    """The shipped CP kernels on the sharded path (BASELINE configs[3] fp64, configs[4] fp32):
    k_cp5 with no pins on either side. A shard runs k_cp5_leaf's eta2 tasks over the
    replicated top and its own stages, its own leaves, and its own families plus the top above
    the cut's parents; X1 delivers the roots' s of the half step, then the cut's parents'
    family tiles run alone. The dynamics run k_dy3 with its merged top (k_dy3_top_back / _fwd)
    over the replicated stages above the cut, as the unsharded default does. Residual histories and the owned iterate equal the unsharded
    default solve bit for bit (only max reductions are regrouped)."""
    r = recipe_config(cfg, seed=0)
    tree, prob = build_problem(r)
    base = core.Cache(prob, dtype=dtype)
    assert base.native.kernel_info(10).startswith("k_cp5_leaf")
    alpha = 0.999 / base.native.step_size(rtol=1e-7 if dtype == "float32" else 1e-14)
    iters = 12 if cfg == 4 else 6
    st0, err0, derr0 = base.native.cp_run(r["x0"], iters, 0.0, alpha)
    z0 = base.get_primal_flat()
    shards = [core.Cache(prob, dtype=dtype) for _ in range(R)]
    for k, s in enumerate(shards):
        s.native.shard(k, R)
        assert s.native.kernel_info(10).startswith("k_cp5_leaf")
        assert "k_dy3_top_back" in s.native.kernel_info(9)  # the merged top over the replicated stages
    st, err, derr = group_cp_run([s.native for s in shards], r["x0"], iters, 0.0, alpha)
    assert st == st0 and err.shape == err0.shape == (iters + 1, 3)
    assert np.array_equal(err, err0) and np.array_equal(derr, derr0)
    nx = base.packed.nx
    covered = np.zeros(tree.num_nodes, dtype=bool)
    for s in shards:
        z = s.get_primal_flat()
        for (a, b) in _owned_x_slices(s.native):
            if b > a:
                np.testing.assert_array_equal(z[a * nx:b * nx], z0[a * nx:b * nx])
                covered[a:b] = True
    assert covered.all()


def test_sharded_default_kernels_stop_with_unsharded():
    """Early stop through the sharded k_cp5 path (config 4, R = 2): the stopping test sees the
    maxima over shards and fires at the unsharded default solve's iteration, mid-run."""
    r = recipe_config(4, seed=0)
    tree, prob = build_problem(r)
    base = core.Cache(prob)
    alpha = 0.999 / base.native.step_size()
    _, e_full, _ = base.native.cp_run(r["x0"], 40, 0.0, alpha)
    e = e_full.max(axis=1)
    # a tolerance first met mid-run: the first new running minimum of the error after k = 3
    ks = [k for k in range(4, len(e)) if e[k] < e[:k].min()]
    if not ks:
        pytest.skip("the config-4 trace has no new minimum after iteration 3")
    tol = float(e[ks[0]])
    st0, err0, derr0 = base.native.cp_run(r["x0"], 40, tol, alpha)
    assert st0 == 0 and err0.shape[0] == ks[0] + 1
    shards = [core.Cache(prob) for _ in range(2)]
    for k, s in enumerate(shards):
        s.native.shard(k, 2)
    st, err, derr = group_cp_run([s.native for s in shards], r["x0"], 40, tol, alpha)
    assert st == st0 and err.shape == err0.shape
    assert np.array_equal(err, err0) and np.array_equal(derr, derr0)
