"""GPU parity: the HIP path (through the C-ABI, via the drop-in classes) against the
golden fixtures produced by the reference (tests/golden/gen_golden.py) and against
the oracle at sizes the oracle finishes in seconds.

Tolerances: fp64 everywhere. Single operator applications 1e-12 relative (only the
summation order differs from numpy/BLAS); CP residual traces 1e-8 relative per
entry (BASELINE.json north_star: "within 1e-8 relative").

Tests that exercise the dynamics projection run under both of its engines: the tiered
subtree kernels (default) and the per-stage fallback that trees whose subtrees do not
fit LDS take (RAOCP_DYN_PER_STAGE=1 at context creation), via the `dyn` parameter.
"""
import contextlib
import os

import numpy as np
import pytest

import raocp.core as core
from raocp.problems import build_problem, recipe_config
from helpers import problem_from_golden, rel_err, trace_rel_err

pytestmark = pytest.mark.gpu

OPS = ["main", "ops2x2", "bin6", "c1n5"]
PROX = ["main", "bin6", "cache3", "c1n5"]
DYN = ["tiers", "per_stage"]


@contextlib.contextmanager
def _env(key, value):
    old = os.environ.get(key)
    if value is None:
        os.environ.pop(key, None)
    else:
        os.environ[key] = value
    try:
        yield
    finally:
        if old is None:
            os.environ.pop(key, None)
        else:
            os.environ[key] = old


@contextlib.contextmanager
def dyn_engine(mode):
    """Contexts created inside use the tiered dynamics kernels or the per-stage fallback (not
    the streaming per-stage sweep k_dy3, the default of fp64 trees of >= 64k nodes, which
    tests/test_gpu_dyn3.py covers)."""
    with _env("RAOCP_DYN_PER_STAGE", "1" if mode == "per_stage" else "0"), _env("RAOCP_DYN3", "0"):
        yield


@contextlib.contextmanager
def cp_kernels(mode):
    """Contexts created inside use the CP kernels the library picks for the tree ("auto": the
    fused streaming k_cp3 on uniform trees of the benchmark sizes, else scalar below ~4k node
    tiles and MFMA above), the two-launch MFMA kernels (raocp_cp2.hip) or the scalar ones
    (raocp_cp.hip)."""
    with _env("RAOCP_CP_V1", {"auto": None, "cp3": None, "mfma": "0", "scalar": "1"}[mode]), \
            _env("RAOCP_CP3", None if mode in ("auto", "cp3") else "0"), _env("RAOCP_CP5", "0" if mode == "cp3" else None), \
            _env("RAOCP_CP6", "0" if mode == "cp3" else None):
        yield


@pytest.fixture(scope="module")
def ops_kat(golden):
    return golden("ops_kat")


@pytest.fixture(scope="module")
def prox_kat(golden):
    return golden("prox_kat")


def _cache(z, name):
    r, tree, prob = problem_from_golden(z, name)
    return r, core.Cache(prob)


@pytest.mark.parametrize("name", OPS)
def test_ell_and_transpose_match_reference(ops_kat, name):
    z = ops_kat
    r, cache = _cache(z, name)
    op = core.Operator(cache)
    assert cache.primal_size == z[f"{name}/ops_z"].size and cache.dual_size == z[f"{name}/ops_eta"].size
    lz = op.linop_ell(z[f"{name}/ops_z"].reshape(-1, 1)).reshape(-1)
    assert rel_err(lz, z[f"{name}/ops_Lz"]) <= 1e-12
    lte = op.linop_ell_transpose(z[f"{name}/ops_eta"].reshape(-1, 1)).reshape(-1)
    assert rel_err(lte, z[f"{name}/ops_LTeta"]) <= 1e-12


@pytest.mark.parametrize("name", OPS)
def test_block_api_keeps_unwritten_template_slots(ops_kat, name):
    z = ops_kat
    r, cache = _cache(z, name)
    op = core.Operator(cache)
    prim = cache._blocks_p(z[f"{name}/ops_z"])
    out_d = cache._blocks_d(z[f"{name}/ops_tmpl_dual"])
    op.ell(prim, out_d)
    assert rel_err(np.concatenate([b.ravel() for b in out_d]), z[f"{name}/ops_ell_out"]) <= 1e-12
    dual = cache._blocks_d(z[f"{name}/ops_eta"])
    out_p = cache._blocks_p(z[f"{name}/ops_tmpl_primal"])
    op.ell_transpose(dual, out_p)
    assert rel_err(np.concatenate([b.ravel() for b in out_p]), z[f"{name}/ops_ellT_out"]) <= 1e-12


@pytest.mark.parametrize("name", OPS)
def test_adjoint_identity(ops_kat, name):
    # tests/test_operators.py:101-116 / 323-335: <z, L'eta> = <Lz, eta>
    z = ops_kat
    r, cache = _cache(z, name)
    rng = np.random.default_rng(7)
    for _ in range(3):
        zz = rng.standard_normal(cache.primal_size)
        ee = rng.standard_normal(cache.dual_size)
        a = zz @ cache.native.ell_t(ee)
        b = cache.native.ell(zz) @ ee
        assert abs(a - b) <= 1e-10 * max(1.0, abs(a))


@pytest.mark.parametrize("dyn", DYN)
@pytest.mark.parametrize("name", PROX)
def test_prox_f_and_steps_match_reference(prox_kat, name, dyn):
    z = prox_kat
    with dyn_engine(dyn):
        r, cache = _cache(z, name)
    alpha = float(z[f"{name}/prox_alpha"])
    zin = z[f"{name}/prox_z"]
    cache.cache_initial_state(r["x0"].reshape(-1, 1))
    for op, key in (("dyn", "prox_dyn"), ("ker", "prox_kernel"), ("f", "prox_f")):
        cache.set_primal_flat(zin)
        if op == "dyn":
            cache.project_on_dynamics()
        elif op == "ker":
            cache.project_on_kernel()
        else:
            cache.proximal_of_f(alpha)
        got = cache.get_primal_flat()
        assert rel_err(got, z[f"{name}/{key}"]) <= 1e-12, op


@pytest.mark.parametrize("name", PROX)
def test_prox_gconj_and_steps_match_reference(prox_kat, name):
    z = prox_kat
    r, cache = _cache(z, name)
    alpha = float(z[f"{name}/prox_alpha"])
    ein = z[f"{name}/prox_eta"]
    cache.set_dual_flat(ein)
    cache.proximal_of_g_conjugate(alpha)
    assert rel_err(cache.get_dual_flat(), z[f"{name}/prox_gconj"]) <= 1e-12
    cache.set_dual_flat(ein)
    cache.project_on_constraints_nonleaf()
    assert rel_err(cache.get_dual_flat(), z[f"{name}/prox_proj_nonleaf"]) <= 1e-12
    cache.set_dual_flat(ein)
    cache.project_on_constraints_leaf()
    assert rel_err(cache.get_dual_flat(), z[f"{name}/prox_proj_leaf"]) <= 1e-12
    cache.set_dual_flat(ein)
    cache.modify_dual(alpha)
    cache.add_halves()
    assert rel_err(cache.get_dual_flat(), z[f"{name}/prox_modify_halves"]) <= 1e-15


def _run_chock(z, name, pin, dyn="tiers", cpk="auto"):
    r, tree, prob = problem_from_golden(z, name)
    with dyn_engine(dyn), cp_kernels(cpk):
        solver = core.Solver(problem_spec=prob)
    alpha = float(z[f"{name}/cp_alpha"]) if pin else None
    status = solver.chock(initial_state=r["x0"].reshape(-1, 1), max_iters=int(z[f"{name}/cp_max_iters"]),
                          tol=float(z[f"{name}/cp_tol"]), step_size=alpha)
    return solver, status


@pytest.mark.parametrize("pin,dyn,cpk", [(True, "tiers", "auto"), (False, "tiers", "auto"), (True, "per_stage", "auto"),
                                         (True, "tiers", "mfma")])
def test_main_py_trace(golden, pin, dyn, cpk):
    """main.py end to end: 937 iterations, status 0, residual trace vs the reference's
    (which itself matches the published 4-3-residuals.tex to 3.4e-12)."""
    z = golden("main_trace")
    solver, status = _run_chock(z, "main", pin, dyn, cpk)
    assert status == int(z["main/cp_status"]) == 0
    err = solver.error_cache
    assert err.shape == z["main/cp_error"].shape == (937, 3)
    assert trace_rel_err(err, z["main/cp_error"]) <= 1e-8
    assert trace_rel_err(solver.delta_error_cache, z["main/cp_delta_error"]) <= 1e-8
    assert trace_rel_err(err, z["main/tex_trace"]) <= 1e-8
    zf = solver.cache.get_primal_flat()
    ef = solver.cache.get_dual_flat()
    assert rel_err(zf, z["main/cp_z"]) <= 1e-9 and rel_err(ef, z["main/cp_eta"]) <= 1e-9
    if not pin:
        assert abs(solver.step_size - float(z["main/cp_alpha"])) <= 1e-12 * float(z["main/cp_alpha"])


@pytest.mark.parametrize("dyn,cpk", [("tiers", "auto"), ("per_stage", "auto"), ("tiers", "mfma")])
@pytest.mark.parametrize("name", ["bin6", "c1n5", "ops2x2"])
def test_small_trajectories(golden, name, dyn, cpk):
    z = golden("traj_small")
    solver, status = _run_chock(z, name, True, dyn, cpk)
    assert status == int(z[f"{name}/cp_status"])
    assert trace_rel_err(solver.error_cache, z[f"{name}/cp_error"]) <= 1e-8
    assert trace_rel_err(solver.delta_error_cache, z[f"{name}/cp_delta_error"]) <= 1e-8
    assert rel_err(solver.cache.get_primal_flat(), z[f"{name}/cp_z"]) <= 1e-9


def test_step_size_matches_arpack(golden):
    for f, names in (("main_trace", ["main"]), ("traj_small", ["bin6", "c1n5", "ops2x2"])):
        z = golden(f)
        for name in names:
            r, tree, prob = problem_from_golden(z, name)
            lam = core.Cache(prob).native.step_size()
            assert abs(lam - float(z[f"{name}/cp_lambda"])) <= 1e-11 * lam, name


def test_single_iteration_quirks(golden):
    # max_iters=0 runs one iteration and returns 1; the error cache is 1-D (solver.py:148-153)
    z = golden("main_trace")
    r, tree, prob = problem_from_golden(z, "main")
    s = core.Solver(problem_spec=prob)
    assert s.chock(r["x0"].reshape(-1, 1), max_iters=0, tol=1e-3, step_size=float(z["main/cp_alpha"])) == 1
    assert s.error_cache.shape == (3,)
    assert trace_rel_err(s.error_cache, z["main/cp_error"][0]) <= 1e-10
    # tol met exactly at k == max_iters returns 1
    s2 = core.Solver(problem_spec=prob)
    assert s2.chock(r["x0"].reshape(-1, 1), max_iters=936, tol=1e-3, step_size=float(z["main/cp_alpha"])) == 1
    assert s2.error_cache.shape == (937, 3)


def test_nan_in_box_raises(golden):
    z = golden("prox_kat")
    r, cache = _cache(z, "main")
    e = z["main/prox_eta"].copy()
    e[-1] = np.nan  # last slot is an eta14 entry (leaf box)
    cache.set_dual_flat(e)
    with pytest.raises(ValueError):
        cache.project_on_constraints_leaf()


# ---------------------------------------------------------------------------------------
# the benchmark configuration (BASELINE configs[1]: 8,191 nodes, nx=20, nu=8) vs the oracle
# ---------------------------------------------------------------------------------------
@pytest.fixture(scope="module", params=[("tiers", "auto"), ("per_stage", "auto"), ("tiers", "mfma")],
                ids=["tiers", "per_stage", "tiers-mfma"])
def c2(request):
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(2)
    tree, prob = build_problem(r)
    with dyn_engine(request.param[0]), cp_kernels(request.param[1]):
        cache = core.Cache(prob)
    return r, prob, cache, OracleProblem(prob)


def test_c2_operators_vs_oracle(c2):
    r, prob, cache, orc = c2
    rng = np.random.default_rng(11)
    zz = rng.standard_normal(cache.primal_size)
    ee = rng.standard_normal(cache.dual_size)
    assert rel_err(cache.native.ell(zz), orc.ell(zz)) <= 1e-12
    assert rel_err(cache.native.ell_t(ee), orc.ell_t(ee)) <= 1e-12
    cache.cache_initial_state(r["x0"])
    cache.set_primal_flat(zz)
    cache.proximal_of_f(0.3)
    assert rel_err(cache.get_primal_flat(), orc.prox_f(zz, 0.3, r["x0"])) <= 1e-11
    cache.set_dual_flat(ee)
    cache.proximal_of_g_conjugate(0.3)
    assert rel_err(cache.get_dual_flat(), orc.prox_gconj(ee, 0.3)) <= 1e-12


def test_c2_bench_runs_the_requested_iterations(c2):
    """bench.py's timed call: raocp_cp_prepare(x0, K) then raocp_cp_bench(NULL, K) runs
    exactly K iterations from x0 (a whole graph batch plus a remainder) and leaves the same
    iterate as raocp_cp_bench(x0, K) and as a K-iteration cp_run."""
    r, prob, cache, orc = c2
    nat = cache.native
    alpha = 0.999 / nat.step_size()
    K = 29
    nat.cp_run(r["x0"], K - 1, 0.0, alpha)
    z_run, e_run = nat.get_primal(), nat.get_dual()
    nat.cp_bench(r["x0"], K, alpha)
    assert np.array_equal(nat.get_primal(), z_run) and np.array_equal(nat.get_dual(), e_run)
    nat.cp_prepare(K, r["x0"], alpha)
    ms = nat.cp_bench(None, K, alpha)
    assert ms > 0
    assert np.array_equal(nat.get_primal(), z_run) and np.array_equal(nat.get_dual(), e_run)
    with pytest.raises(Exception, match="raocp_cp_prepare"):
        nat.cp_bench(None, K, alpha)  # a prepared run is consumed by one bench call


def test_c2_cp_trace_vs_oracle(c2):
    r, prob, cache, orc = c2
    lam = cache.native.step_size()
    lam_o, _ = orc.step_size()
    assert abs(lam - lam_o) <= 1e-11 * lam
    alpha = 0.999 / lam
    status, err, derr = cache.native.cp_run(r["x0"], 19, 0.0, alpha)
    st_o, err_o, derr_o, z_o, e_o, _ = orc.chock(r["x0"], 19, 0.0, alpha=alpha)
    assert status == st_o == 1 and err.shape == (20, 3)
    assert trace_rel_err(err, err_o) <= 1e-8
    assert trace_rel_err(derr, derr_o) <= 1e-8
    assert rel_err(cache.get_primal_flat(), z_o) <= 1e-10
    assert rel_err(cache.get_dual_flat(), e_o) <= 1e-10


@pytest.mark.parametrize("cfg", [3, 4, "4-modes"])
def test_large_operators_vs_oracle(cfg):
    """L and L^T at the HBM-sized configs (87k / 88k nodes,
    nx = 20 / 32): many node-range blocks, multi-pass row loops, adjoint identity.
    "4-modes": config 4 with a different cost per mode, so consecutive children use
    different weight tables (the register rows reload)."""
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(4 if cfg == "4-modes" else cfg)
    if cfg == "4-modes":
        r["Q"] = np.array([(1.0 + k) * q for k, q in enumerate(r["Q"])])
        r["R"] = np.array([(2.0 + k) * q for k, q in enumerate(r["R"])])
    tree, prob = build_problem(r)
    cache, orc = core.Cache(prob), OracleProblem(prob)
    rng = np.random.default_rng(5)
    zz = rng.standard_normal(cache.primal_size)
    ee = rng.standard_normal(cache.dual_size)
    lz, lte = cache.native.ell(zz), cache.native.ell_t(ee)
    assert rel_err(lz, orc.ell(zz)) <= 1e-12
    assert rel_err(lte, orc.ell_t(ee)) <= 1e-12
    a, b = zz @ lte, lz @ ee
    assert abs(a - b) <= 1e-10 * max(abs(a), 1.0)


@pytest.mark.parametrize("dyn", DYN)
@pytest.mark.parametrize("cfg", [2, 3, 4])
def test_projections_full_size_vs_oracle_and_idempotent(cfg, dyn):
    """The dynamics and kernel projections (cache.py:259-317) at the HBM-sized configs:
    against the oracle, and size-independent properties: a projection applied twice is
    the projection (idempotence), and its output satisfies x_j = A_j x_i + B_j u_i,
    x_0 = x0 (feasibility; relative to the state scale)."""
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(cfg)
    tree, prob = build_problem(r)
    with dyn_engine(dyn):
        cache = core.Cache(prob)
    orc = OracleProblem(prob)
    nat = cache.native
    rng = np.random.default_rng(17)
    zz = rng.standard_normal(cache.primal_size)
    cache.cache_initial_state(r["x0"])
    nat.set_primal(zz)
    nat.project_on_dynamics()
    z1 = nat.get_primal()
    assert rel_err(z1, orc.project_on_dynamics(zz, r["x0"])) <= 1e-11
    nat.project_on_dynamics()
    assert rel_err(nat.get_primal(), z1) <= 1e-11
    X = z1[orc.X0:orc.U0].reshape(orc.n, orc.nx)
    U = z1[orc.U0:orc.Y0].reshape(orc.m, orc.nu)
    j = np.arange(1, orc.n)
    par = orc.anc[j]
    pred = np.stack([orc.A[orc.iA[k]] @ X[par[t]] + orc.B[orc.iB[k]] @ U[par[t]] for t, k in enumerate(j)])
    assert np.max(np.abs(X[j] - pred)) <= 1e-10 * max(1.0, np.max(np.abs(X)))
    assert np.array_equal(X[0], np.asarray(r["x0"], dtype=float).reshape(-1))
    nat.set_primal(zz)
    nat.project_on_kernel()
    z2 = nat.get_primal()
    assert rel_err(z2, orc.project_on_kernel(zz)) <= 1e-12
    nat.project_on_kernel()
    assert rel_err(nat.get_primal(), z2) <= 1e-12


@pytest.mark.parametrize("cfg,cpk", [(3, "auto"), (4, "auto"), (4, "cp3"), (3, "scalar"), ("4-modes", "auto")])
def test_large_cp_trace_vs_oracle(cfg, cpk):
    """The whole CP loop (solver.py:124-161) at the HBM-sized configs (SURVEY.md 8(d)
    config 3: Markov 4 modes, 87,381 nodes, nx = 20; config 4: branching 3, 88,573 nodes,
    nx = 32, nu = 12): the fused CP kernels, the dynamics tiers and prox g* at those sizes,
    10 iterations against the oracle; then prox g* alone on a random dual."""
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(4 if cfg == "4-modes" else cfg)
    if cfg == "4-modes":  # a cost per mode: blocks mixing weight tables (scalar kernels)
        r["Q"] = np.array([(1.0 + k) * q for k, q in enumerate(r["Q"])])
        r["R"] = np.array([(2.0 + k) * q for k, q in enumerate(r["R"])])
    tree, prob = build_problem(r)
    with cp_kernels(cpk):
        cache = core.Cache(prob)
    orc = OracleProblem(prob)
    alpha = 0.999 / cache.native.step_size()
    status, err, derr = cache.native.cp_run(r["x0"], 9, 0.0, alpha)
    st_o, err_o, derr_o, z_o, e_o, _ = orc.chock(r["x0"], 9, 0.0, alpha=alpha)
    assert status == st_o == 1 and err.shape == (10, 3)
    assert trace_rel_err(err, err_o) <= 1e-8
    assert trace_rel_err(derr, derr_o) <= 1e-8
    assert rel_err(cache.get_primal_flat(), z_o) <= 1e-10
    assert rel_err(cache.get_dual_flat(), e_o) <= 1e-10
    ee = np.random.default_rng(23).standard_normal(cache.dual_size)
    cache.set_dual_flat(ee)
    cache.proximal_of_g_conjugate(0.3)
    assert rel_err(cache.get_dual_flat(), orc.prox_gconj(ee, 0.3)) <= 1e-12


def test_chock_warm_start_matches_reference_fixture(golden):
    """The reference's own second Solver.chock on one solver (tests/golden/warm_start.npz,
    generated by tests/golden/gen_golden.py gen_warm): 60 iterations from x0, then 40 from
    x0 / 2 continuing from the cached primal / dual (solver.py:97-102, cache.py:79-82)."""
    z = golden("warm_start")
    r, tree, prob = problem_from_golden(z, "warm")
    s = core.Solver(problem_spec=prob)
    for call in (0, 1):
        key = f"warm/call{call}/"
        st = s.chock(z[key + "x0"].reshape(-1, 1), max_iters=int(z[key + "max_iters"]), tol=0.0,
                     step_size=float(z[key + "alpha"]))
        assert st == int(z[key + "status"])
        assert trace_rel_err(s.error_cache, z[key + "error"]) <= 1e-8
        assert trace_rel_err(s.delta_error_cache, z[key + "delta_error"]) <= 1e-8
        assert rel_err(s.cache.get_primal_flat(), z[key + "z"]) <= 1e-9
        assert rel_err(s.cache.get_dual_flat(), z[key + "eta"]) <= 1e-9


def test_chock_warm_starts_like_reference(golden):
    """A second chock continues from the first one's iterate with the new x0 in node 0's
    state (solver.py:27-61 read the cache's old primal / dual; cache.py:79-82), and a dual
    made current by set_dual + update_cache is where the next solve starts."""
    from oracle.raocp_oracle import OracleProblem
    z = golden("main_trace")
    r, tree, prob = problem_from_golden(z, "main")
    alpha = float(z["main/cp_alpha"])
    x0 = r["x0"].reshape(-1, 1)
    orc = OracleProblem(prob)
    s = core.Solver(problem_spec=prob)
    s.chock(x0, max_iters=20, tol=0.0, step_size=alpha)
    _, err1, _, zo, eo, _ = orc.chock(x0, 20, 0.0, alpha=alpha)
    assert trace_rel_err(s.error_cache, err1) <= 1e-8
    x0b = 0.5 * x0
    assert s.chock(x0b, max_iters=15, tol=0.0, step_size=alpha) == 1
    _, err2, derr2, zo2, eo2, _ = orc.chock(x0b, 15, 0.0, alpha=alpha, p0=zo, d0=eo)
    assert trace_rel_err(s.error_cache, err2) <= 1e-8
    assert trace_rel_err(s.delta_error_cache, derr2) <= 1e-8
    assert rel_err(s.cache.get_primal_flat(), zo2) <= 1e-9
    assert rel_err(s.cache.get_dual_flat(), eo2) <= 1e-9
    # a dual set and committed before the first solve
    s2 = core.Solver(problem_spec=prob)
    # a dual as prox g* leaves it (placeholder slots exactly 0, as in every reference dual)
    e0 = orc.prox_gconj(np.random.default_rng(3).standard_normal(s2.cache.dual_size), alpha)
    s2.cache.set_dual(s2.cache._blocks_d(e0))
    s2.cache.update_cache()
    s2.chock(x0, max_iters=10, tol=0.0, step_size=alpha)
    _, err3, _, zo3, _, _ = orc.chock(x0, 10, 0.0, alpha=alpha, p0=np.zeros(orc.P), d0=e0)
    assert trace_rel_err(s2.error_cache, err3) <= 1e-8
    assert rel_err(s2.cache.get_primal_flat(), zo3) <= 1e-9


def test_nan_initial_state_is_not_converged(golden):
    """A NaN in x0 on a problem without boxes: the residuals are NaN, `max(error) <= tol`
    is false every iteration (solver.py:137-161), so the solve runs to max_iters and
    returns 1 with NaN in the error cache (the max reductions propagate NaN)."""
    z = golden("ops_kat")
    r, tree, prob = problem_from_golden(z, "ops2x2")
    s = core.Solver(problem_spec=prob)
    x0 = r["x0"].astype(float).copy()
    x0[0] = np.nan
    assert s.chock(x0.reshape(-1, 1), max_iters=5, tol=1e-3, step_size=0.1) == 1
    assert s.error_cache.shape == (6, 3)
    assert np.isnan(s.error_cache).any()


def test_output_utilities_headless(golden, tmp_path, capsys, monkeypatch):
    """Solver.plot_residuals / plot_solution / print_states / print_inputs (solver.py:173-253)
    after main.py's solve, with the Agg backend: the residual file carries the published
    4-3-residuals.tex trace, every leaf-to-root path of the solution plot is the solved
    iterate, and the prints list every state / input block."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    z = golden("main_trace")
    solver, status = _run_chock(z, "main", True)
    monkeypatch.chdir(tmp_path)
    plt.close("all")
    solver.plot_residuals(show=False)
    ax = plt.gca()
    assert [t.get_text() for t in ax.get_legend().get_texts()] == ["xi_0", "xi_1", "xi_2"]
    for q, ln in enumerate(ax.get_lines()[:3]):
        assert trace_rel_err(ln.get_ydata(), z["main/cp_error"][:, q]) <= 1e-8
    tex = core.Solver.read_residuals_tex(str(tmp_path / "4-3-residuals.tex"))
    assert trace_rel_err(tex, z["main/tex_trace"]) <= 1e-8
    plt.close("all")
    solver.plot_solution(show=False)
    fig = plt.gcf()
    axs = np.array(fig.axes).reshape(2, -1)
    r, tree, prob = problem_from_golden(z, "main")
    nx, nu = 3, 2
    assert axs.shape == (2, nx)
    zf = solver.cache.get_primal_flat()
    X = zf[:tree.num_nodes * nx].reshape(-1, nx)
    leaves = tree.nodes_at_stage(tree.num_stages - 1)
    for e in range(nx):
        lines = axs[0, e].get_lines()
        assert len(lines) == len(leaves)
        j = leaves[0]
        path = [X[j, e]]
        while tree.ancestor_of(j) >= 0:
            j = tree.ancestor_of(j)
            path.append(X[j, e])
        assert np.allclose(lines[0].get_ydata(), path, rtol=0, atol=0)
    for e in range(nu):
        assert len(axs[1, e].get_lines()) == len(leaves)
    plt.close("all")
    capsys.readouterr()
    solver.print_states()
    solver.print_inputs()
    out = capsys.readouterr().out
    assert out.startswith("states =\n")
    assert out.count("[[") == tree.num_nodes + tree.num_nonleaf_nodes


@pytest.mark.parametrize("cfg", [2, 4])
def test_dyn2_fp64_projection_and_cp_trace(cfg):
    """The per-stage MFMA dynamics sweep (raocp_dyn2.hip, the engine of fp32 contexts) in
    fp64 (RAOCP_DYN2=1): the projection against the oracle at 1e-11 and 10 CP iterations at
    the trace tolerance."""
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(cfg)
    tree, prob = build_problem(r)
    with _env("RAOCP_DYN2", "1"):
        cache = core.Cache(prob)
    orc = OracleProblem(prob)
    zz = np.random.default_rng(17).standard_normal(cache.primal_size)
    cache.cache_initial_state(r["x0"])
    cache.native.set_primal(zz)
    cache.native.project_on_dynamics()
    assert rel_err(cache.native.get_primal(), orc.project_on_dynamics(zz, r["x0"])) <= 1e-11
    alpha = 0.999 / cache.native.step_size()
    status, err, derr = cache.native.cp_run(r["x0"], 9, 0.0, alpha)
    st_o, err_o, derr_o, z_o, e_o, _ = orc.chock(r["x0"], 9, 0.0, alpha=alpha)
    assert trace_rel_err(err, err_o) <= 1e-8 and trace_rel_err(derr, derr_o) <= 1e-8
    assert rel_err(cache.get_primal_flat(), z_o) <= 1e-10
