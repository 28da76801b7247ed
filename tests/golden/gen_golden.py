"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
(smokinmirror/raocp-toolbox at /root/reference) in this container.

This script is the only place that imports the reference. It runs here only
(the reference never travels to the GPU box); the .npz files it writes are the
fixtures the test-suite and the oracle are pinned against.

    python -B tests/golden/gen_golden.py            # writes tests/golden/*.npz
    python -B tests/golden/gen_golden.py warm       # only warm_start.npz

The reference needs `turtle` (tkinter) and `tikzplotlib`, both absent here:
they are stubbed as empty modules (scenario_tree.py:4, solver.py:8 import them
but the paths exercised here never call them). `cvxpy` is not needed.

Each problem is described by a "recipe" of plain arrays (stored in the fixture)
so the build's own builder can re-create the same problem without the
reference. Recipes mirror main.py:11-80, tests/test_operators.py:20-66,
tests/test_cache.py:19-76 and SURVEY.md section 8(d) (synthetic configs).
"""
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

for _name in ("turtle", "tikzplotlib"):
    sys.modules.setdefault(_name, types.ModuleType(_name))
import matplotlib  # noqa: E402

matplotlib.use("Agg")
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import raocp.core as core  # noqa: E402  (the REFERENCE package)
import raocp.core.solver as ref_solver  # noqa: E402
import raocp.core.constraints.rectangle as rectangle  # noqa: E402
import raocp.core.dynamics as ref_dynamics  # noqa: E402

assert os.path.realpath(core.__file__).startswith(REF), core.__file__


# ----------------------------------------------------------------------------------------------
# recipes
# ----------------------------------------------------------------------------------------------

def recipe_main():
    """main.py:11-79 verbatim."""
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0.0], [0.0, 0.3, 0.7]])
    v = np.array([0.1, 0.6, 0.3])
    factor = 0.1
    Aw = factor * np.array([[1, 2, 1], [1, 1, 2], [2, 1, 1]])
    Bw = factor * np.array([[1, 0], [1, 0], [0, 2]])
    A = np.array([0.5 * Aw, Aw, -0.5 * Aw])
    B = np.array([-0.5 * Bw, Bw, 0.5 * Bw])
    Q = factor * np.eye(3)
    R = factor * np.eye(2)
    x_lim, u_lim = 7, .1
    return dict(P=p, v=v, N=4, tau=3, A=A, B=B,
                Q=np.array([.2 * Q] * 3), R=np.array([.2 * R] * 3), Pf=factor * .1 * np.eye(3),
                alpha_r=.95,
                nl_min=np.concatenate([-x_lim * np.ones(3), -u_lim * np.ones(2)]),
                nl_max=np.concatenate([x_lim * np.ones(3), u_lim * np.ones(2)]),
                l_min=-x_lim * np.ones(3), l_max=x_lim * np.ones(3),
                x0=np.array([5., -6., -1.]))


def recipe_ops2x2():
    """tests/test_operators.py:20-66 (no constraints, 2x2 dynamics/costs)."""
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0], [0, 0.3, 0.7]])
    v = np.array([0.5, 0.4, 0.1])
    I2 = np.eye(2)
    return dict(P=p, v=v, N=4, tau=3, A=np.array([I2, 2 * I2, 3 * I2]), B=np.array([I2, 2 * I2, 3 * I2]),
                Q=np.array([10 * I2, 20 * I2, 30 * I2]), R=np.array([I2, 2 * I2, 3 * I2]), Pf=5 * I2,
                alpha_r=0.5, nl_min=None, nl_max=None, l_min=None, l_max=None, x0=np.array([1., -1.]))


def recipe_cache3():
    """tests/test_cache.py:19-76: 3x3 dynamics with 2x2 costs (quirk: L is never applied)."""
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0], [0, 0.3, 0.7]])
    v = np.array([0.5, 0.4, 0.1])
    I3, I2 = np.eye(3), np.eye(2)
    return dict(P=p, v=v, N=4, tau=3, A=np.array([I3, 2 * I3, 3 * I3]), B=np.array([I3, 2 * I3, 3 * I3]),
                Q=np.array([10 * I2, 20 * I2, 30 * I2]), R=np.array([I2, 2 * I2, 3 * I2]), Pf=5 * I2,
                alpha_r=0.5, nl_min=-2 * np.ones(6), nl_max=2 * np.ones(6),
                l_min=-0.5 * np.ones(3), l_max=0.5 * np.ones(3), x0=np.array([0.3, -0.2, 0.1]))


def recipe_synthetic(P, v, N, tau, nx, nu, seed=0, alpha_r=0.9):
    """SURVEY.md 8(d) common problem data: rng=default_rng(seed); per mode A then B ~ 0.1 N(0,1);
    Q=R=0.1I, Pf=0.01I, boxes +-1, x0 ~ N(0,1) drawn after A/B."""
    rng = np.random.default_rng(seed)
    M = P.shape[0]
    A = np.zeros((M, nx, nx))
    B = np.zeros((M, nx, nu))
    for k in range(M):
        A[k] = 0.1 * rng.standard_normal((nx, nx))
        B[k] = 0.1 * rng.standard_normal((nx, nu))
    x0 = rng.standard_normal(nx)
    return dict(P=P, v=v, N=N, tau=tau, A=A, B=B,
                Q=np.array([0.1 * np.eye(nx)] * M), R=np.array([0.1 * np.eye(nu)] * M), Pf=0.01 * np.eye(nx),
                alpha_r=alpha_r, nl_min=-np.ones(nx + nu), nl_max=np.ones(nx + nu),
                l_min=-np.ones(nx), l_max=np.ones(nx), x0=x0)


def recipe_bin6():
    return recipe_synthetic(np.full((2, 2), .5), np.array([.5, .5]), 6, 6, 20, 8, seed=0)


def recipe_c1n5():
    """BASELINE configs[0] wording: main.py chain, 3 modes, horizon N=5, nx=4, nu=2 (tau=3: ragged)."""
    p = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0.0], [0.0, 0.3, 0.7]])
    return recipe_synthetic(p, np.array([0.1, 0.6, 0.3]), 5, 3, 4, 2, seed=3, alpha_r=0.95)


# ----------------------------------------------------------------------------------------------
# build a REFERENCE problem from a recipe (mirrors main.py:27-76)
# ----------------------------------------------------------------------------------------------

def build_ref(r):
    tree = core.MarkovChainScenarioTreeFactory(transition_prob=r["P"], initial_distribution=r["v"],
                                               num_stages=r["N"], stopping_time=r["tau"]).create()
    nl, l = core.Nonleaf(), core.Leaf()
    M = r["A"].shape[0]
    dyn = [ref_dynamics.Dynamics(r["A"][k], r["B"][k]) for k in range(M)]
    nl_costs = [core.Quadratic(nl, r["Q"][k], r["R"][k]) for k in range(M)]
    prob = core.RAOCP(scenario_tree=tree) \
        .with_markovian_dynamics(dyn) \
        .with_markovian_nonleaf_costs(nl_costs) \
        .with_all_leaf_costs(core.Quadratic(l, r["Pf"])) \
        .with_all_risks(core.AVaR(r["alpha_r"]))
    if r["nl_min"] is not None:
        prob = prob.with_all_nonleaf_constraints(
            rectangle.Rectangle(nl, r["nl_min"].reshape(-1, 1), r["nl_max"].reshape(-1, 1)))
    if r["l_min"] is not None:
        prob = prob.with_all_leaf_constraints(
            rectangle.Rectangle(l, r["l_min"].reshape(-1, 1), r["l_max"].reshape(-1, 1)))
    return tree, prob


def recipe_arrays(name, r):
    out = {}
    for k, val in r.items():
        if val is None:
            continue
        out[f"{name}/{k}"] = np.asarray(val)
    return out


def tree_arrays(name, tree):
    n = tree.num_nodes
    anc = np.array([tree.ancestor_of(i) for i in range(n)])
    stages = np.array([tree.stage_of(i) for i in range(n)])
    values = np.array([tree.value_at_node(i) for i in range(n)])
    probs = np.asarray(tree._ScenarioTree__probability, dtype=float)
    m = tree.num_nonleaf_nodes
    ch_off = [0]
    ch = []
    for i in range(m):
        c = list(tree.children_of(i))
        ch += c
        ch_off.append(len(ch))
    cond = np.concatenate([tree.conditional_probabilities_of_children(i) for i in range(m)])
    return {f"{name}/tree_anc": anc, f"{name}/tree_stage": stages, f"{name}/tree_value": values,
            f"{name}/tree_prob": probs, f"{name}/tree_num_nonleaf": np.array(m),
            f"{name}/tree_children": np.array(ch), f"{name}/tree_children_off": np.array(ch_off),
            f"{name}/tree_cond_prob": cond}


def flat(blocks):
    return np.vstack(blocks).reshape(-1).astype(float)


def unflat(template, vec):
    out = list(template)
    cur = 0
    for i, t in enumerate(template):
        out[i] = vec[cur: cur + t.size].reshape(-1, 1).copy()
        cur += t.size
    assert cur == vec.size
    return out


def block_sizes(template):
    return np.array([t.size for t in template])


# ----------------------------------------------------------------------------------------------
# fixtures
# ----------------------------------------------------------------------------------------------

def parse_tex_trace(path):
    """4-3-residuals.tex: three `table {% ... };` blocks with `iter value` rows (solver.py:187-199)."""
    series, cur = [], None
    with open(path) as f:
        for line in f:
            s = line.strip()
            if s.startswith("table {%"):
                cur = []
                continue
            if cur is not None:
                if s.startswith("}"):
                    series.append(np.array(cur))
                    cur = None
                else:
                    a, b = s.split()
                    cur.append((int(a), float(b)))
    assert len(series) == 3
    it = series[0][:, 0]
    return np.stack([s_[:, 1] for s_ in series], axis=1), it


def gen_ops(out):
    rng = np.random.default_rng(1)
    for name, rf in (("main", recipe_main), ("ops2x2", recipe_ops2x2), ("bin6", recipe_bin6), ("c1n5", recipe_c1n5)):
        r = rf()
        tree, prob = build_ref(r)
        cache = core.Cache(prob)
        op = core.Operator(cache)
        _, tp = cache.get_primal()
        _, td = cache.get_dual()
        zf = rng.standard_normal(sum(t.size for t in tp))
        ef = rng.standard_normal(sum(t.size for t in td))
        lz = op.linop_ell(zf.reshape(-1, 1)).reshape(-1)
        lte = op.linop_ell_transpose(ef.reshape(-1, 1)).reshape(-1)
        # block-list API with a NON-zero output template: unwritten slots keep caller values
        tmpl_d = [rng.standard_normal(t.shape) for t in td]
        out_d = list(tmpl_d)
        op.ell(unflat(tp, zf), out_d)
        tmpl_p = [rng.standard_normal(t.shape) for t in tp]
        out_p = list(tmpl_p)
        op.ell_transpose(unflat(td, ef), out_p)
        out.update(recipe_arrays(name, r))
        out.update(tree_arrays(name, tree))
        out.update({f"{name}/ops_z": zf, f"{name}/ops_eta": ef, f"{name}/ops_Lz": lz, f"{name}/ops_LTeta": lte,
                    f"{name}/ops_tmpl_dual": flat(tmpl_d), f"{name}/ops_ell_out": flat(out_d),
                    f"{name}/ops_tmpl_primal": flat(tmpl_p), f"{name}/ops_ellT_out": flat(out_p),
                    f"{name}/primal_block_sizes": block_sizes(tp), f"{name}/dual_block_sizes": block_sizes(td),
                    f"{name}/seg_p": np.array(cache.get_primal_segments()[1:]),
                    f"{name}/seg_d": np.array([s if s is not None else -1 for s in cache.get_dual_segments()[1:]])})
        print(f"ops {name}: n={tree.num_nodes} |P|={zf.size} |D|={ef.size}")


def gen_prox(out):
    rng = np.random.default_rng(2)
    for name, rf in (("main", recipe_main), ("bin6", recipe_bin6), ("cache3", recipe_cache3), ("c1n5", recipe_c1n5)):
        r = rf()
        tree, prob = build_ref(r)
        n, m = tree.num_nodes, tree.num_nonleaf_nodes
        out.update(recipe_arrays(name, r))
        out.update(tree_arrays(name, tree))
        # offline products (cache.py:207-233)
        c = core.Cache(prob)
        P = np.array(c._Cache__P)
        K = np.array(c._Cache__K[:m])
        Abar = np.array([c._Cache__sum_of_dynamics[j] if j > 0 else np.zeros_like(P[0]) for j in range(n)])
        out.update({f"{name}/off_P": P, f"{name}/off_K": K, f"{name}/off_Abar": Abar})
        _, tp = c.get_primal()
        _, td = c.get_dual()
        nP = sum(t.size for t in tp)
        nD = sum(t.size for t in td)
        x0 = r["x0"].reshape(-1, 1)
        alpha = float(rng.uniform(0.1, 0.9))

        def fresh_primal(vec):
            cc = core.Cache(prob)
            cc.cache_initial_state(x0)
            cc.set_primal(unflat(tp, vec))
            return cc

        zin = rng.standard_normal(nP)
        zin[sum(t.size for t in tp[:c.get_primal_segments()[4]])] = 0.0  # tau_0 (never read)
        cc = fresh_primal(zin); cc.project_on_dynamics(); dyn = flat(cc.get_primal()[0])
        cc = fresh_primal(zin); cc.project_on_kernel(); ker = flat(cc.get_primal()[0])
        cc = fresh_primal(zin); cc.proximal_of_f(alpha); pf = flat(cc.get_primal()[0])

        ein = rng.standard_normal(nD)

        def fresh_dual(vec):
            cc = core.Cache(prob)
            cc.set_dual(unflat(td, vec))
            return cc

        cc = fresh_dual(ein); cc.proximal_of_g_conjugate(alpha); pg = flat(cc.get_dual()[0])
        cc = fresh_dual(ein); cc.project_on_constraints_nonleaf(); pnl = flat(cc.get_dual()[0])
        cc = fresh_dual(ein); cc.project_on_constraints_leaf(); pl = flat(cc.get_dual()[0])
        cc = fresh_dual(ein); cc.modify_dual(alpha); cc.add_halves(); mh = flat(cc.get_dual()[0])
        out.update({f"{name}/prox_alpha": np.array(alpha), f"{name}/prox_z": zin, f"{name}/prox_dyn": dyn,
                    f"{name}/prox_kernel": ker, f"{name}/prox_f": pf, f"{name}/prox_eta": ein,
                    f"{name}/prox_gconj": pg, f"{name}/prox_proj_nonleaf": pnl, f"{name}/prox_proj_leaf": pl,
                    f"{name}/prox_modify_halves": mh})
        print(f"prox {name}: n={n} alpha={alpha:.4f}")


def run_chock(name, r, max_iters, tol, out, pin_lambda=None):
    tree, prob = build_ref(r)
    solver = core.Solver(problem_spec=prob)
    orig = ref_solver.eigs
    captured = {}

    def eigs_capture(op, *a, **k):
        if pin_lambda is not None:
            vals = np.array([pin_lambda + 0j])
        else:
            vals, vecs = orig(op, *a, **k)
        captured["lam"] = float(np.real(max(vals)))
        return vals, None

    ref_solver.eigs = eigs_capture
    try:
        status = solver.chock(initial_state=r["x0"].reshape(-1, 1), max_iters=max_iters, tol=tol)
    finally:
        ref_solver.eigs = orig
    cache = solver._Solver__cache
    z, _ = cache.get_primal()
    e, _ = cache.get_dual()
    lam = captured["lam"]
    out.update(recipe_arrays(name, r))
    out.update(tree_arrays(name, tree))
    out.update({f"{name}/cp_lambda": np.array(lam), f"{name}/cp_alpha": np.array(0.999 / lam),
                f"{name}/cp_max_iters": np.array(max_iters), f"{name}/cp_tol": np.array(tol),
                f"{name}/cp_status": np.array(status),
                f"{name}/cp_error": np.atleast_2d(solver._Solver__error_cache),
                f"{name}/cp_delta_error": np.atleast_2d(solver._Solver__delta_error_cache),
                f"{name}/cp_z": flat(z), f"{name}/cp_eta": flat(e)})
    print(f"chock {name}: status={status} iters={np.atleast_2d(solver._Solver__error_cache).shape[0]} "
          f"lambda={lam!r}")


def gen_warm(out):
    """Two chock calls on ONE reference Solver (main.py's problem): the second continues from
    the cached primal / dual of the first with a new initial state written into node 0's
    state (solver.py:97-102 with cache.py:79-82). Both traces, step sizes and iterates."""
    r = recipe_main()
    tree, prob = build_ref(r)
    solver = core.Solver(problem_spec=prob)
    orig = ref_solver.eigs
    lams = []

    def eigs_capture(op, *a, **k):
        vals, _ = orig(op, *a, **k)
        lams.append(float(np.real(max(vals))))
        return vals, None

    ref_solver.eigs = eigs_capture
    out.update(recipe_arrays("warm", r))
    out.update(tree_arrays("warm", tree))
    try:
        for call, (x0, iters) in enumerate(((r["x0"], 60), (r["x0"] / 2, 40))):
            status = solver.chock(initial_state=x0.reshape(-1, 1), max_iters=iters, tol=0.0)
            cache = solver._Solver__cache
            z, _ = cache.get_primal()
            e, _ = cache.get_dual()
            out.update({f"warm/call{call}/x0": x0, f"warm/call{call}/max_iters": np.array(iters),
                        f"warm/call{call}/status": np.array(status), f"warm/call{call}/lambda": np.array(lams[-1]),
                        f"warm/call{call}/alpha": np.array(0.999 / lams[-1]),
                        f"warm/call{call}/error": np.atleast_2d(solver._Solver__error_cache),
                        f"warm/call{call}/delta_error": np.atleast_2d(solver._Solver__delta_error_cache),
                        f"warm/call{call}/z": flat(z), f"warm/call{call}/eta": flat(e)})
            print(f"warm call {call}: status={status} rows={np.atleast_2d(solver._Solver__error_cache).shape[0]} "
                  f"lambda={lams[-1]!r}")
    finally:
        ref_solver.eigs = orig


def gen_trees(out):
    rng = np.random.default_rng(5)
    p3 = np.array([[0.1, 0.8, 0.1], [0.4, 0.6, 0], [0, 0.3, 0.7]])
    p4 = rng.random((4, 4)) + 0.1
    p4 /= p4.sum(axis=1, keepdims=True)
    p4z = p4.copy()
    p4z[0, 2] = 0.0
    p4z[3, 1] = 0.0
    p4z /= p4z.sum(axis=1, keepdims=True)
    cases = {
        "t_test": (p3, np.array([0.5, 0.5, 0.0]), 4, 3),           # tests/test_scenario_tree.py:11-19
        "t_main": (p3, np.array([0.1, 0.6, 0.3]), 4, 3),           # main.py:11-20
        "t_tauN": (p3, np.array([0.1, 0.6, 0.3]), 4, 4),           # tau == N (probability length n+1)
        "t_tau1": (p3, np.array([0.5, 0.4, 0.1]), 5, 1),
        "t_N1": (p3, np.array([0.5, 0.4, 0.1]), 1, 1),
        "t_bin": (np.full((2, 2), .5), np.array([.5, .5]), 5, 5),
        "t_m4": (p4, np.full(4, .25), 4, 4),
        "t_m4z": (p4z, np.array([.4, 0., .3, .3]), 5, 3),
    }
    names = []
    for name, (P, v, N, tau) in cases.items():
        tree = core.MarkovChainScenarioTreeFactory(P, v, N, tau).create()
        out.update(tree_arrays(name, tree))
        out[f"{name}/P"] = P
        out[f"{name}/v"] = v
        out[f"{name}/N"] = np.array(N)
        out[f"{name}/tau"] = np.array(tau)
        names.append(name)
        print(f"tree {name}: n={tree.num_nodes} m={tree.num_nonleaf_nodes} probs={len(tree._ScenarioTree__probability)}")
    out["names"] = np.array(names)


def main():
    np.random.seed(12345)  # ARPACK start vectors come from numpy's global RNG inside scipy
    if sys.argv[1:] == ["warm"]:  # only the warm-start fixture (added in round 3)
        w = {}
        gen_warm(w)
        np.savez_compressed(os.path.join(OUT, "warm_start.npz"), **w)
        return
    ops = {}
    gen_ops(ops)
    np.savez_compressed(os.path.join(OUT, "ops_kat.npz"), **ops)

    prox = {}
    gen_prox(prox)
    np.savez_compressed(os.path.join(OUT, "prox_kat.npz"), **prox)

    trees = {}
    gen_trees(trees)
    np.savez_compressed(os.path.join(OUT, "tree_kat.npz"), **trees)

    tr = {}
    run_chock("main", recipe_main(), 2000, 1e-3, tr)
    tex, it = parse_tex_trace(os.path.join(REF, "4-3-residuals.tex"))
    tr["main/tex_trace"] = tex
    tr["main/tex_iter"] = it
    rel = np.max(np.abs(tr["main/cp_error"] - tex) / np.abs(tex))
    print(f"main trace vs 4-3-residuals.tex: max rel err {rel:.3e}")
    np.savez_compressed(os.path.join(OUT, "main_trace.npz"), **tr)

    tr = {}
    run_chock("bin6", recipe_bin6(), 49, 0.0, tr)
    run_chock("c1n5", recipe_c1n5(), 199, 0.0, tr)
    run_chock("ops2x2", recipe_ops2x2(), 30, 0.0, tr)
    np.savez_compressed(os.path.join(OUT, "traj_small.npz"), **tr)


if __name__ == "__main__":
    main()
