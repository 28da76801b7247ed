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
from helpers import problem_from_golden, rel_err

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


def test_fp32_rejects_mixed_weight_blocks(golden):
    """ops2x2 has a different cost per mode, so a family's children use different sqrtQ
    tables: the fp32 MFMA blocks need one table per block, and context creation says so."""
    r, tree, prob = problem_from_golden(golden("ops_kat"), "ops2x2")
    from raocp.core._native import RaocpError
    with pytest.raises(RaocpError, match="one weight table"):
        core.Cache(prob, dtype="float32")


def test_fp32_dynamics_projection_config5(c5):
    """The per-stage MFMA dynamics sweep (raocp_dyn2.hip) in fp32 at config 5 against the
    fp64 oracle (cache.py:259-288): 2e-5 relative to the largest entry (a backward and a
    forward recursion of 9 stages of 64 x 80 products), and feasibility x_j = A_j x_i + B_j u_i
    of its output to fp32 accuracy."""
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
