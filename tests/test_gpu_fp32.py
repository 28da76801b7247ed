"""GPU parity of fp32 contexts (BASELINE.json configs[4]: "n_x = 64, n_u = 16 padded to MFMA
tile, fp32"): L and L^T (operators.py:19-94) in fp32 on the MFMA node blocks against the
oracle in fp64.

Tolerance (fp32): every output entry is a dot product of at most 64 fp32 products, so the
error is a few ulp of the row scale; the tests bound it by 2e-6 relative to the largest
reference entry (fp32 epsilon 1.19e-7 times 16), per operator application. Size-independent
checks at the full config-5 size: the adjoint identity <L z, eta> = <z, L^T eta> to 1e-5
relative (a sum over 10^8 products in fp32 dot partials accumulated in fp64)."""
import numpy as np
import pytest

import raocp.core as core
from raocp.problems import build_problem, recipe_config
from helpers import problem_from_golden, rel_err, trace_rel_err

pytestmark = pytest.mark.gpu

TOL32 = 2e-6


@pytest.mark.parametrize("name", ["main", "bin6", "c1n5"])
def test_fp32_ell_matches_reference(golden, name):
    z = golden("ops_kat")
    r, tree, prob = problem_from_golden(z, name)
    cache = core.Cache(prob, dtype="float32")
    lz = cache.native.ell(z[f"{name}/ops_z"])
    assert rel_err(lz, z[f"{name}/ops_Lz"]) <= TOL32
    lte = cache.native.ell_t(z[f"{name}/ops_eta"])
    assert rel_err(lte, z[f"{name}/ops_LTeta"]) <= TOL32


@pytest.fixture(scope="module")
def c5():
    from oracle.raocp_oracle import OracleProblem
    r = recipe_config(5)
    tree, prob = build_problem(r)
    return r, prob, core.Cache(prob, dtype="float32"), OracleProblem(prob)


def test_fp32_config5_operators_vs_oracle(c5):
    """349,525 nodes, nx = 64, nu = 16 (383.4 MB per L in fp32)."""
    r, prob, cache, orc = c5
    assert cache.packed.n == 349525
    rng = np.random.default_rng(5)
    zz = rng.standard_normal(cache.primal_size)
    ee = rng.standard_normal(cache.dual_size)
    lz, lte = cache.native.ell(zz), cache.native.ell_t(ee)
    assert rel_err(lz, orc.ell(zz)) <= TOL32
    assert rel_err(lte, orc.ell_t(ee)) <= TOL32
    a, b = zz @ lte, lz @ ee
    assert abs(a - b) <= 1e-5 * max(abs(a), 1.0)


def test_fp32_step_size_close_to_fp64():
    """Lanczos on L'L in fp32 (vectors and products fp32, dot partials fp64) agrees with the
    fp64 context's lambda_max to fp32 accuracy (config 2)."""
    r = recipe_config(2)
    tree, prob = build_problem(r)
    l64 = core.Cache(prob).native.step_size()
    l32 = core.Cache(prob, dtype="float32").native.step_size(rtol=1e-7)
    assert abs(l32 - l64) <= 1e-5 * l64


def _cp_drift(c32, c64, x0, K):
    """K + 1 CP iterations of an fp32 and an fp64 context with the fp64 step size: relative
    trace errors (per entry) and iterate errors (to the largest entry)."""
    alpha = 0.999 / c64.native.step_size()
    s32, e32, d32 = c32.native.cp_run(x0, K, 0.0, alpha)
    s64, e64, d64 = c64.native.cp_run(x0, K, 0.0, alpha)
    assert s32 == s64 == 1 and e32.shape == e64.shape == (K + 1, 3)
    return (trace_rel_err(e32, e64), trace_rel_err(d32, d64), rel_err(c32.get_primal_flat(), c64.get_primal_flat()),
            rel_err(c32.get_dual_flat(), c64.get_dual_flat()), alpha, e64)


def test_fp32_mixed_weight_tables_ops2x2(golden):
    """ops2x2 has a different cost per mode (raocp_spec.py:118-131, with_markovian_nonleaf_costs),
    so a family's children use different sqrtQ / sqrtR tables: fp32 contexts run the node-block
    kernels k_cpd / k_cpp<float> (raocp_cp.hip), which read a table per child. 30 iterations
    against the fp64 context and the oracle (fp64): traces within 1e-4 per entry, iterates
    within 1e-5 of the largest entry (fp32 rounding over 30 iterations)."""
    from oracle.raocp_oracle import OracleProblem
    r, tree, prob = problem_from_golden(golden("ops_kat"), "ops2x2")
    c32, c64 = core.Cache(prob, dtype="float32"), core.Cache(prob)
    assert c32.native.kernel_info(10) == "k_cpd<float, 0, 0> + k_cpp<float, 0, 0>"
    K = 29
    te, td, zr, er, alpha, e64 = _cp_drift(c32, c64, r["x0"], K)
    print(f"fp32 mixed ops2x2: traces {te:.2e} / {td:.2e}, iterate {zr:.2e} / {er:.2e}")
    assert te <= 1e-4 and td <= 1e-4 and zr <= 1e-5 and er <= 1e-5
    _, eo, _, zo, _, _ = OracleProblem(prob).chock(r["x0"], max_iters=K, tol=0.0, alpha=alpha)
    assert trace_rel_err(e64, eo) <= 1e-8
    assert rel_err(c32.get_primal_flat(), zo) <= 1e-5


def test_fp32_mixed_weight_tables_config4_modes():
    """Config 4 with a cost per mode (the consecutive children of every family on different
    tables, as in test_gpu_parity's "4-modes"): fp32 k_cpd / k_cpp<float> against the fp64
    context over 20 iterations (traces 1e-4 per entry, iterates 1e-5)."""
    r = recipe_config(4)
    r["Q"] = np.array([(1.0 + k) * q for k, q in enumerate(r["Q"])])
    r["R"] = np.array([(2.0 + k) * q for k, q in enumerate(r["R"])])
    tree, prob = build_problem(r)
    c32, c64 = core.Cache(prob, dtype="float32"), core.Cache(prob)
    assert c32.native.kernel_info(10).startswith("k_cpd<float")
    te, td, zr, er, _, _ = _cp_drift(c32, c64, r["x0"], 19)
    print(f"fp32 mixed config 4: traces {te:.2e} / {td:.2e}, iterate {zr:.2e} / {er:.2e}")
    assert te <= 1e-4 and td <= 1e-4 and zr <= 1e-5 and er <= 1e-5


def test_fp32_node_block_kernels_match_mfma_kernels():
    """RAOCP_CP_V1=1 forces k_cpd / k_cpp<float> on a tree with one table per block
    (config 2): the same iterations as the fused fp32 k_cp3 up to fp32 rounding."""
    import os
    r = recipe_config(2)
    tree, prob = build_problem(r)
    os.environ["RAOCP_CP_V1"] = "1"
    os.environ["RAOCP_CP3"] = "0"
    try:
        v1 = core.Cache(prob, dtype="float32")
    finally:
        del os.environ["RAOCP_CP_V1"], os.environ["RAOCP_CP3"]
    v3 = core.Cache(prob, dtype="float32")
    assert v1.native.kernel_info(10).startswith("k_cpd<float")
    assert v3.native.kernel_info(10).startswith("k_cp3<float")
    te, td, zr, er, _, _ = _cp_drift(v1, v3, r["x0"], 19)
    print(f"fp32 v1 vs k_cp3 config 2: traces {te:.2e} / {td:.2e}, iterate {zr:.2e} / {er:.2e}")
    assert te <= 1e-4 and td <= 1e-4 and zr <= 1e-5 and er <= 1e-5


def test_fp32_dynamics_projection_config5(c5):
    """The per-stage dynamics sweep k_dy3<float> (raocp_dyn3.hip: per-stage table images,
    MFMA node blocks) at config 5 against the fp64 oracle (cache.py:259-288): 2e-5 relative to
    the largest entry (a backward and a forward recursion of 9 stages of 64 x 80 products),
    and feasibility x_j = A_j x_i + B_j u_i of its output to fp32 accuracy."""
    r, prob, cache, orc = c5
    rng = np.random.default_rng(17)
    zz = rng.standard_normal(cache.primal_size)
    cache.cache_initial_state(r["x0"])
    cache.native.set_primal(zz)
    cache.native.project_on_dynamics()
    z1 = cache.native.get_primal()
    ref = orc.project_on_dynamics(zz, r["x0"])
    assert rel_err(z1, ref) <= 2e-5
    X = z1[orc.X0:orc.U0].reshape(orc.n, orc.nx)
    U = z1[orc.U0:orc.Y0].reshape(orc.m, orc.nu)
    j = np.arange(1, orc.n, 997)
    pred = np.stack([orc.A[orc.iA[k]] @ X[orc.anc[k]] + orc.B[orc.iB[k]] @ U[orc.anc[k]] for k in j])
    assert np.max(np.abs(X[j] - pred)) <= 1e-5 * max(1.0, np.max(np.abs(X)))


def test_fp32_cp_loop_config5_vs_oracle(c5):
    """Three iterations of the whole CP loop (solver.py:124-161) in fp32 at config 5 against
    the fp64 oracle with the same step size: residual traces within 1e-3 relative per entry
    and the final iterate within 1e-4 of its largest entry (fp32 rounding through the
    iteration's chain of L, prox and L^T)."""
    r, prob, cache, orc = c5
    lam = cache.native.step_size(rtol=1e-7)
    alpha = 0.999 / lam
    status, err, derr = cache.native.cp_run(r["x0"], 2, 0.0, alpha)
    st_o, err_o, derr_o, z_o, e_o, _ = orc.chock(r["x0"], 2, 0.0, alpha=alpha)
    assert status == st_o == 1 and err.shape == (3, 3)
    assert np.max(np.abs(err - err_o) / np.abs(err_o)) <= 1e-3
    assert np.max(np.abs(derr - derr_o) / np.abs(derr_o)) <= 1e-3
    assert rel_err(cache.get_primal_flat(), z_o) <= 1e-4
    assert rel_err(cache.get_dual_flat(), e_o) <= 1e-4


def _c5_fixture(golden):
    try:
        return golden("c5_cp")
    except FileNotFoundError:
        pytest.skip("tests/golden/c5_cp.npz missing (tests/golden/gen_c5_cp.py)")


def _c5_against_fixture(cache, fx, K, x0):
    """cp_run of K iterations (tol = 0) at the fixture's step size; the oracle's K-iteration
    traces and iterate samples / norms (tests/golden/gen_c5_cp.py)."""
    alpha = float(fx["alpha"])
    status, err, derr = cache.native.cp_run(x0, K - 1, 0.0, alpha)
    z, eta = cache.get_primal_flat(), cache.get_dual_flat()
    pre = f"k{K}/"
    assert status == 1 and err.shape == fx[pre + "err"].shape == (K, 3)
    te = float(np.max(np.abs(err - fx[pre + "err"]) / np.abs(fx[pre + "err"])))
    td = float(np.max(np.abs(derr - fx[pre + "derr"]) / np.abs(fx[pre + "derr"])))
    zs = float(np.max(np.abs(z[fx["ip"]] - fx[pre + "z_sample"])) / fx[pre + "z_norms"][1])
    es = float(np.max(np.abs(eta[fx["id"]] - fx[pre + "eta_sample"])) / fx[pre + "eta_norms"][1])
    zn = abs(np.linalg.norm(z) / fx[pre + "z_norms"][0] - 1)
    en = abs(np.linalg.norm(eta) / fx[pre + "eta_norms"][0] - 1)
    print(f"config 5, {K} iterations: traces {te:.2e} / {td:.2e}, iterate samples {zs:.2e} / {es:.2e}, "
          f"norms {zn:.2e} / {en:.2e}")
    return te, td, zs, es, zn, en


def test_fp32_cp_loop_config5_20_iterations_vs_oracle(c5, golden):
    """20 iterations of the fp32 CP loop at config 5 (k_cp5_leaf + k_cp5_fams<float> + k_dy3<float>)
    against the fp64 oracle at the oracle's own step size (c5_cp.npz: the oracle's traces and
    iterate samples, 6 min of CPU per run, hence stored). Tolerances from fp32 rounding
    through 20 nonexpansive CP steps: the residual traces 2e-3 relative per entry, the iterate
    samples 2e-4 of the largest entry, the iterate norms 1e-4 relative."""
    r, prob, cache, orc = c5
    fx = _c5_fixture(golden)
    assert np.array_equal(fx["x0"], np.asarray(r["x0"], float))
    te, td, zs, es, zn, en = _c5_against_fixture(cache, fx, 20, r["x0"])
    assert te <= 2e-3 and td <= 2e-3 and zs <= 2e-4 and es <= 2e-4 and zn <= 1e-4 and en <= 1e-4


def test_fp64_config5_path_10_iterations_vs_oracle(golden):
    """The fp64 context at nx = 64, nu = 16 (the reference the fp32 drift test of
    test_gpu_cp3.py compares with: k_cpd2 / k_cpp2<double> + k_dy3<double, 64, 16>) for 10
    iterations against the oracle (c5_cp.npz): traces 1e-8 relative per entry (BASELINE.json
    north_star), iterate samples 1e-10 of the largest entry."""
    r = recipe_config(5)
    fx = _c5_fixture(golden)
    cache = core.Cache(build_problem(r)[1])
    te, td, zs, es, zn, en = _c5_against_fixture(cache, fx, 10, r["x0"])
    assert te <= 1e-8 and td <= 1e-8 and zs <= 1e-10 and es <= 1e-10 and zn <= 1e-12 and en <= 1e-12
