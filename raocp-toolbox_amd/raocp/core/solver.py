# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Chambolle–Pock solver (reference: raocp/core/solver.py:12-253).

`chock` runs the whole loop on the GPU: step size by device Lanczos on L'L
(replacing ARPACK `eigs`, solver.py:104-118), then `raocp_cp_run`, which
replays the CP iteration as a captured hipGraph (dynamics sweeps, fused
L + prox_g* + xi2 kernel, fused L^T + AVaR-kernel projection + residual kernel,
on-device stopping test) and only syncs with the host every 24 iterations. Like the
reference, a solve continues from the cache's current (old) primal / dual.
Residual histories, return codes and the two timer prints are the reference's.
The host-orchestrated half steps (`primal_k_plus_half` ...) are kept for API
parity; each of their operators is still a HIP kernel.
"""
import time

import numpy as np

import raocp.core.cache as cache
import raocp.core.operators as ops
import raocp.core.raocp_spec as spec

__all__ = ["Solver"]


class Solver:
    def __init__(self, problem_spec: spec.RAOCP, device=None, dtype="float64"):
        self.__raocp = problem_spec
        self.__cache = cache.Cache(self.__raocp, device=device, dtype=dtype)
        self.__operator = ops.Operator(self.__cache)
        self.__initial_state = None
        self.__parameter_1 = None
        self.__parameter_2 = None
        self.__error = [np.zeros(1)] * 3
        self.__delta_error = [np.zeros(1)] * 3
        self.__error_cache = None
        self.__delta_error_cache = None

    @property
    def cache(self):
        return self.__cache

    @property
    def step_size(self):
        return self.__parameter_1

    # ----- host-orchestrated half steps (solver.py:27-61)
    def primal_k_plus_half(self):
        _, template = self.__cache.get_primal()
        _, old_dual = self.__cache.get_dual()
        self.__operator.ell_transpose(old_dual, template)
        _, old_primal = self.__cache.get_primal()
        self.__cache.set_primal([a - self.__parameter_1 * b for a, b in zip(old_primal, template)])

    def primal_k_plus_one(self):
        self.__cache.proximal_of_f(self.__parameter_1)

    def dual_k_plus_half(self):
        _, template = self.__cache.get_dual()
        primal, old_primal = self.__cache.get_primal()
        self.__operator.ell([2 * a - b for a, b in zip(primal, old_primal)], template)
        _, old_dual = self.__cache.get_dual()
        self.__cache.set_dual([a + self.__parameter_2 * b for a, b in zip(old_dual, template)])

    def dual_k_plus_one(self):
        self.__cache.proximal_of_g_conjugate(self.__parameter_2)

    def _calculate_chock_errors(self):
        p_new, p = self.__cache.get_primal()
        d_new, d = self.__cache.get_dual()
        a1, a2 = self.__parameter_1, self.__parameter_2
        d_minus = [x - y for x, y in zip(d, d_new)]
        _, lt = self.__cache.get_primal()
        self.__operator.ell_transpose(d_minus, lt)
        xi_1 = [(x - y) / a1 - z for x, y, z in zip(p, p_new, lt)]
        p_diff = [x - y for x, y in zip(p_new, p)]
        _, lp = self.__cache.get_dual()
        self.__operator.ell(p_diff, lp)
        xi_2 = [x / a2 + y for x, y in zip(d_minus, lp)]
        _, lt2 = self.__cache.get_primal()
        self.__operator.ell_transpose(xi_2, lt2)
        xi_0 = [x + y for x, y in zip(xi_1, lt2)]
        delta_2 = [x - y for x, y in zip(d_new, d)]
        _, lt3 = self.__cache.get_primal()
        self.__operator.ell_transpose(delta_2, lt3)
        delta_0 = [x - y for x, y in zip(p_diff, lt3)]
        return xi_0, xi_1, xi_2, delta_0, p_diff, delta_2

    # ----- the CP loop (solver.py:97-171)
    def compute_step_size(self):
        lam = self.__cache.native.step_size()
        self.__parameter_1 = self.__parameter_2 = 0.999 / lam
        return lam

    def chock(self, initial_state, max_iters=10, tol=1e-5, step_size=None):
        """Chambolle-Pock algorithm. Returns 0 if converged (k < max_iters), else 1.
        `step_size` (extension) pins alpha instead of estimating 0.999/||L||^2."""
        self.__initial_state = initial_state
        self.__cache.cache_initial_state(initial_state)
        if step_size is None:
            self.compute_step_size()
        else:
            self.__parameter_1 = self.__parameter_2 = float(step_size)
        x0 = np.asarray(initial_state, dtype=np.float64).reshape(-1)
        # the loop continues from the cached old primal / dual (x0 in node 0's state), as
        # the reference's does: a second chock warm-starts from the first one's iterate
        self.__cache.seed_device_iterate()
        print("timer started")
        tick = time.perf_counter()
        status, err, derr = self.__cache.native.cp_run(x0, int(max_iters), float(tol), self.__parameter_1,
                                                       warm=True)
        tock = time.perf_counter()
        print(f"timer stopped in {tock - tick:0.4f} seconds")
        self.__error = list(err[-1])
        self.__delta_error = list(derr[-1])
        # one row per iteration; a single iteration leaves a 1-D array (solver.py:148-153)
        self.__error_cache = err if err.shape[0] > 1 else err[0]
        self.__delta_error_cache = derr if derr.shape[0] > 1 else derr[0]
        self.__cache.update_cache()
        return status

    # ----- outputs (solver.py:173-253)
    @property
    def error_cache(self):
        return self.__error_cache

    @property
    def delta_error_cache(self):
        return self.__delta_error_cache

    def print_states(self):
        primal, _ = self.__cache.get_primal()
        seg_p = self.__cache.get_primal_segments()
        print("states =\n")
        for i in range(seg_p[1], seg_p[2]):
            print(f"{primal[i]}\n")

    def print_inputs(self):
        primal, _ = self.__cache.get_primal()
        seg_p = self.__cache.get_primal_segments()
        print("inputs =\n")
        for i in range(seg_p[2], seg_p[3]):
            print(f"{primal[i]}\n")

    @staticmethod
    def _tikz_save(name, fallback=None):
        """tikzplotlib.save(name) as the reference does (solver.py:199, 253); tikzplotlib is
        optional (absent in this image): `fallback(name)` then writes the file itself."""
        try:
            import tikzplotlib
        except ImportError:
            if fallback is not None:
                fallback(name)
            return
        tikzplotlib.save(name)

    def _write_residuals_tex(self, name):
        """The pgfplots file tikzplotlib writes for plot_residuals (the layout of the
        reference's published 4-3-residuals.tex): log-y axis, one table per xi series."""
        ec = np.atleast_2d(self.__error_cache)
        colors = [("steelblue31119180", "31,119,180"), ("darkorange25512714", "255,127,14"),
                  ("forestgreen4416044", "44,160,44")]
        pos = ec[np.isfinite(ec) & (ec > 0)]
        lines = ["% pgfplots residual trace (layout of tikzplotlib's output for Solver.plot_residuals)",
                 "\\begin{tikzpicture}", ""]
        lines += [f"\\definecolor{{{c}}}{{RGB}}{{{rgb}}}" for c, rgb in colors]
        lines += ["", "\\begin{axis}[", "legend cell align={left},", "log basis y={10},",
                  "title={Residual values of Chambolle-Pock algorithm iterations},", "xlabel={iteration},",
                  f"xmin={-0.05 * (len(ec) - 1)!r}, xmax={1.05 * (len(ec) - 1)!r},"]
        if pos.size:
            lines.append(f"ymin={float(pos.min()) / 5!r}, ymax={float(pos.max()) * 2!r},")
        lines += ["ylabel={log(residual value)},", "ymode=log", "]"]
        for q, (c, _) in enumerate(colors):
            lines += [f"\\addplot [thick, {c}]", "table {%"]
            lines += [f"{k} {float(v)!r}" for k, v in enumerate(ec[:, q])]
            lines += ["};", f"\\addlegendentry{{xi_{q}}}"]
        lines += ["\\end{axis}", "", "\\end{tikzpicture}", ""]
        with open(name, "w") as f:
            f.write("\n".join(lines))

    @staticmethod
    def read_residuals_tex(name):
        """The three xi series of a residuals .tex file (this class's or tikzplotlib's) as a
        (k, 3) array."""
        series, cur = [], None
        for line in open(name):
            line = line.strip()
            if line.startswith("table {"):
                cur = []
            elif line.startswith("};") and cur is not None:
                series.append(cur)
                cur = None
            elif cur is not None and line:
                cur.append(float(line.split()[1]))
        return np.array(series).T

    def plot_residuals(self, show=True):
        import matplotlib.pyplot as plt
        ec = np.atleast_2d(self.__error_cache)
        for q in range(3):
            plt.semilogy(ec[:, q], linewidth=2, linestyle="solid")
        plt.title("Residual values of Chambolle-Pock algorithm iterations")
        plt.ylabel(r"log(residual value)", fontsize=12)
        plt.xlabel(r"iteration", fontsize=12)
        plt.legend(("xi_0", "xi_1", "xi_2"))
        self._tikz_save('4-3-residuals.tex', self._write_residuals_tex)
        if show:
            plt.show()

    def plot_solution(self, show=True):
        import matplotlib.pyplot as plt
        primal, _ = self.__cache.get_primal()
        seg_p = self.__cache.get_primal_segments()
        x = primal[seg_p[1]: seg_p[2]]
        u = primal[seg_p[2]: seg_p[3]]
        tree = self.__raocp.tree
        last = tree.num_stages - 1
        fig, axs = plt.subplots(2, np.size(x[0]), sharex="all", sharey="row", squeeze=False)
        fig.set_size_inches(15, 8)
        fig.set_dpi(80)

        def path(j, vals, element):
            pts = [[tree.stage_of(j), vals[j][element][0]]]
            while tree.ancestor_of(j) >= 0:
                j = tree.ancestor_of(j)
                pts.append([tree.stage_of(j), vals[j][element][0]])
            return np.array(pts)

        leaves = tree.nodes_at_stage(last)
        for e in range(np.size(x[0])):
            for leaf in leaves:
                pts = path(leaf, x, e)
                axs[0, e].plot(pts[:, 0], pts[:, 1])
            axs[0, e].set_title(f"state element, x_{e}(t)")
        for e in range(np.size(u[0])):
            for leaf in leaves:
                pts = path(tree.ancestor_of(leaf), u, e)
                axs[1, e].plot(pts[:, 0], pts[:, 1])
            axs[1, e].set_title(f"control element, u_{e}(t)")
        for ax in axs.flat:
            ax.set(xlabel='stage, t', ylabel='value')
            ax.label_outer()
        fig.tight_layout()
        self._tikz_save('python-solution.tex')
        if show:
            plt.show()
