"""CPU: the host side of the boundary.

* the packer (raocp/core/_pack.py) -> per-class K, Rinv, M tables equal the reference's
  per-node offline products (prox_kat fixtures), and the device's re-associated
  dynamics sweep (raocp_dyn.hip), restated here in numpy on the PACKED arrays,
  reproduces the reference's project_on_dynamics output;
* the C-ABI library loads and exports every symbol include/raocp_hip.h declares;
* the product path fails loudly (RuntimeError) when the extension is missing.
No compute call touches a GPU here.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from raocp.core._pack import pack_problem
from raocp.core import _native
from helpers import problem_from_golden, rel_err

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "raocp_hip.h")
PROX = ["main", "bin6", "cache3", "c1n5"]


def _declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(raocp_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert sorted(_native.EXPORTED_SYMBOLS) == _declared_symbols()


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libraocp_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [s for s in _declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # the error channel works without a device
    _native.load_library()
    assert isinstance(_native.load_library().raocp_last_error(), (bytes, type(None)))


def test_missing_extension_fails_loudly(monkeypatch):
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", "/nonexistent/libraocp_hip.so")
    with pytest.raises(RuntimeError, match="HIP extension missing"):
        _native.load_library()


def test_tree_arrays_and_invariants(golden):
    z = golden("prox_kat")
    for name in PROX:
        r, tree, prob = problem_from_golden(z, name)
        pk = pack_problem(prob)
        assert pk.n == tree.num_nodes and pk.m == tree.num_nonleaf_nodes
        assert np.all(np.diff(pk.stage) >= 0)                 # stage-contiguous ids
        assert np.all(np.diff(pk.anc[1:]) >= 0)               # BFS parents
        assert np.array_equal(pk.ch_start[1:], pk.ch_start[:-1] + pk.nch[:-1])   # contiguous children
        for i in range(pk.m):
            assert list(tree.children_of(i)) == list(range(pk.ch_start[i], pk.ch_start[i] + pk.nch[i]))
        # classes are numbered by stage
        assert np.all(np.diff(pk.class_stage) >= 0)
        assert np.array_equal(pk.class_stage[pk.i_k], pk.stage[:pk.m])


@pytest.mark.parametrize("name", PROX)
def test_packed_offline_tables_match_reference(golden, name):
    z = golden("prox_kat")
    r, tree, prob = problem_from_golden(z, name)
    pk = pack_problem(prob)
    m = pk.m
    assert rel_err(pk.K[pk.i_k], z[f"{name}/off_K"]) <= 1e-12
    # M = K' + sum_j Abar_j' P_j B_j from the reference's own P / Abar
    P, Abar = z[f"{name}/off_P"], z[f"{name}/off_Abar"]
    for i in range(m):
        ch = range(pk.ch_start[i], pk.ch_start[i] + pk.nch[i])
        M = pk.K[pk.i_k[i]].T + sum(Abar[j].T @ P[j] @ pk.B[pk.i_b[j]] for j in ch)
        # M is a difference of O(1) terms that may cancel to ~0: compare against their scale
        scale = np.abs(pk.K[pk.i_k[i]]).max() + sum(np.abs(Abar[j].T @ P[j] @ pk.B[pk.i_b[j]]).max() for j in ch)
        assert np.max(np.abs(pk.M[pk.i_k[i]] - M)) <= 1e-12 * scale
        Rt = np.eye(pk.nu) + sum(pk.B[pk.i_b[j]].T @ P[j] @ pk.B[pk.i_b[j]] for j in ch)
        assert rel_err(pk.Rinv[pk.i_k[i]] @ Rt, np.eye(pk.nu)) <= 1e-11


def _device_form_projection(pk, zin, x0):
    """The sweep raocp_dyn.hip executes (per-stage, vectorised over nodes), on packed data."""
    n, m, nx, nu = pk.n, pk.m, pk.nx, pk.nu
    X = zin[:n * nx].reshape(n, nx).copy()
    U = zin[n * nx:n * nx + m * nu].reshape(m, nu).copy()
    q = -X.copy()                      # leaves: q = -x
    d = np.zeros((m, nu))
    A, B = pk.A[pk.i_a], pk.B[pk.i_b]  # per node (row 0 unused)
    for s in range(pk.N - 1, -1, -1):
        ids = np.nonzero(pk.stage[:m] == s)[0]
        for i in ids:
            ch = range(pk.ch_start[i], pk.ch_start[i] + pk.nch[i])
            h = sum(B[j].T @ q[j] for j in ch)
            a = sum(A[j].T @ q[j] for j in ch)
            c = pk.i_k[i]
            d[i] = pk.Rinv[c] @ (U[i] - h)
            q[i] = (-X[i] + pk.K[c].T @ (h - U[i])) + a + pk.M[c] @ d[i]
    X[0] = x0
    for s in range(pk.N):
        for i in np.nonzero(pk.stage[:m] == s)[0]:
            U[i] = pk.K[pk.i_k[i]] @ X[i] + d[i]
            for j in range(pk.ch_start[i], pk.ch_start[i] + pk.nch[i]):
                X[j] = A[j] @ X[i] + B[j] @ U[i]
    out = zin.copy()
    out[:n * nx] = X.ravel()
    out[n * nx:n * nx + m * nu] = U.ravel()
    return out


@pytest.mark.parametrize("name", PROX)
def test_device_form_dynamics_matches_reference(golden, name):
    """The re-associated recursion (h, a, d, q with M) equals cache.py:259-288."""
    z = golden("prox_kat")
    r, tree, prob = problem_from_golden(z, name)
    pk = pack_problem(prob)
    out = _device_form_projection(pk, z[f"{name}/prox_z"], r["x0"])
    assert rel_err(out, z[f"{name}/prox_dyn"]) <= 1e-11


def test_unsupported_inputs_are_rejected():
    import raocp.core as core
    import raocp.core.constraints.no_constraint as no_c
    from raocp.problems import build_problem, recipe_main
    tree, prob = build_problem(recipe_main())
    pk = pack_problem(prob)
    assert pk.l_error is None
    # a non-AVaR risk is refused with the reference's message (cache.py:175-178)

    class OtherRisk:
        is_risk = True
    prob.list_of_risks[0] = OtherRisk()
    with pytest.raises(Exception, match="Risk at node 0 not defined"):
        pack_problem(prob)
    assert core is not None and no_c is not None
