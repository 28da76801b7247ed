// Host-side AddressSanitizer driver for the C-ABI ("race detection /
// sanitizers"): raocp_capi.hip's host code (tree validation, layout and block-table
// builders, tier planner, graph capture, shard tables) built with -fsanitize=address on
// the host only (device code is never instrumented) and driven through every entry point.
//   abi_driver cpu : argument / tree validation and error paths (no device needed)
//   abi_driver gpu : full lifecycle on device 0 (create, operators, prox, step size,
//                    CP runs, bench helpers, sharding with the device-copy transport)
// Exit status 0 = every check passed and ASan reported nothing.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/raocp_hip.h"

static int g_fail = 0;
#define CHECK(cond)                                                              \
    do {                                                                         \
        if (!(cond)) {                                                           \
            fprintf(stderr, "CHECK failed at %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond, \
                    raocp_last_error());                                         \
            ++g_fail;                                                            \
        }                                                                        \
    } while (0)

// a complete binary tree of depth N (stages 0..N), nx states, nu inputs, one mode
struct Problem {
    int n, m, nx, nu, N;
    std::vector<int32_t> anc, stage, ch_start, nch, i0n, i_k, i_box_nl, i_box_l;
    std::vector<double> sq, sr, sp, alpha_r, cond, bnl_lo, bnl_hi, bl_lo, bl_hi, A, B, K, Rinv, M;
    raocp_tree_desc t{};
    raocp_problem_desc p{};
    Problem(int N_, int nx_, int nu_) : N(N_), nx(nx_), nu(nu_) {
        n = (1 << (N + 1)) - 1;
        m = (1 << N) - 1;
        anc.resize(n); stage.resize(n); ch_start.resize(m); nch.resize(m);
        for (int i = 0; i < n; ++i) {
            anc[i] = i == 0 ? -1 : (i - 1) / 2;
            int s = 0;
            while ((2 << s) - 1 <= i) ++s;
            stage[i] = s;
        }
        for (int i = 0; i < m; ++i) { ch_start[i] = 2 * i + 1; nch[i] = 2; }
        i0n.assign(n, 0);
        i_k.resize(m);
        for (int i = 0; i < m; ++i) i_k[i] = stage[i];
        i_box_nl.assign(m, 0);
        i_box_l.assign(n, 0);
        auto eye = [](int r, double v) { std::vector<double> a(r * r, 0.0); for (int k = 0; k < r; ++k) a[k * r + k] = v; return a; };
        sq = eye(nx, 0.3); sr = eye(nu, 0.3); sp = eye(nx, 0.1);
        alpha_r.assign(m, 0.9);
        cond.assign(n, 0.5);
        bnl_lo.assign(nx + nu, -1.0); bnl_hi.assign(nx + nu, 1.0);
        bl_lo.assign(nx, -1.0); bl_hi.assign(nx, 1.0);
        A.assign(nx * nx, 0.0);
        for (int k = 0; k < nx; ++k) A[k * nx + k] = 0.5;
        // B = 0 makes the offline products exact for any P (cache.py:207-233): R~ = I,
        // K = 0, Abar = A, M = K' + sum Abar' P B = 0, so the projection is the true one
        B.assign(nx * nu, 0.0);
        K.assign(N * nu * nx, 0.0);
        Rinv.assign(N * nu * nu, 0.0);
        for (int c = 0; c < N; ++c) for (int k = 0; k < nu; ++k) Rinv[c * nu * nu + k * nu + k] = 1.0;
        M.assign(N * nx * nu, 0.0);
        t = raocp_tree_desc{n, m, nx, nu, anc.data(), stage.data(), ch_start.data(), nch.data()};
        p.n_sq = p.n_sr = p.n_sp = 1;
        p.sqrt_q = sq.data(); p.sqrt_r = sr.data(); p.sqrt_pf = sp.data();
        p.i_sq = p.i_sr = p.i_sp = i0n.data();
        p.alpha_r = alpha_r.data(); p.cond = cond.data();
        p.n_box_nl = p.n_box_l = 1;
        p.box_nl_lo = bnl_lo.data(); p.box_nl_hi = bnl_hi.data();
        p.box_l_lo = bl_lo.data(); p.box_l_hi = bl_hi.data();
        p.i_box_nl = i_box_nl.data(); p.i_box_l = i_box_l.data();
        p.n_a = p.n_b = 1; p.n_k = N;
        p.A = A.data(); p.B = B.data(); p.K = K.data(); p.Rinv = Rinv.data(); p.M = M.data();
        p.i_a = p.i_b = i0n.data(); p.i_k = i_k.data();
        p.dtype = RAOCP_F64;
    }
};

static void cpu_checks() {
    raocp_ctx* c = nullptr;
    Problem pb(4, 4, 2);
    CHECK(raocp_ctx_create(nullptr, &pb.p, 0, &c) == RAOCP_ERR_ARG && c == nullptr);
    CHECK(strlen(raocp_last_error()) > 0);
    // invariant violations, each caught by the validation before any device call
    {
        Problem b(4, 4, 2);
        b.stage[5] = 1;  // stage decreases
        b.t.stage = b.stage.data();
        CHECK(raocp_ctx_create(&b.t, &b.p, 0, &c) == RAOCP_ERR_TREE);
    }
    {
        Problem b(4, 4, 2);
        b.ch_start[3] = 8;  // children not contiguous in parent order
        CHECK(raocp_ctx_create(&b.t, &b.p, 0, &c) == RAOCP_ERR_TREE);
    }
    {
        Problem b(4, 4, 2);
        b.t.m = b.t.n;  // no leaves
        CHECK(raocp_ctx_create(&b.t, &b.p, 0, &c) == RAOCP_ERR_ARG);
    }
    {
        Problem b(4, 4, 2);
        b.anc[0] = 0;
        CHECK(raocp_ctx_create(&b.t, &b.p, 0, &c) == RAOCP_ERR_TREE);
    }
    // null-context entry points fail cleanly
    int64_t P = 0, D = 0;
    CHECK(raocp_sizes(nullptr, &P, &D) != RAOCP_OK);
    CHECK(raocp_cp_prepare(nullptr, nullptr, 1, 0.1) != RAOCP_OK);
    float ms = 0;
    CHECK(raocp_cp_bench(nullptr, nullptr, 1, 0.1, &ms) != RAOCP_OK);
    raocp_ctx_destroy(nullptr);
}

static void gpu_checks() {
    for (int dtype : {RAOCP_F64, RAOCP_F32}) {
        Problem pb(6, 20, 8);
        pb.p.dtype = dtype;
        raocp_ctx* c = nullptr;
        CHECK(raocp_ctx_create(&pb.t, &pb.p, 0, &c) == RAOCP_OK && c);
        if (!c) return;
        int64_t P = 0, D = 0;
        CHECK(raocp_sizes(c, &P, &D) == RAOCP_OK && P > 0 && D > 0);
        std::vector<double> z(P), eta(D), z2(P, 0.0), eta2(D, 0.0), x0(pb.nx, 0.3);
        for (int64_t i = 0; i < P; ++i) z[i] = std::sin(0.1 * i);
        for (int64_t i = 0; i < D; ++i) eta[i] = std::cos(0.1 * i);
        CHECK(raocp_ell(c, z.data(), eta2.data(), 0) == RAOCP_OK);
        CHECK(raocp_ell_t(c, eta.data(), z2.data(), 0) == RAOCP_OK);
        double lam = 0;
        CHECK(raocp_step_size(c, &lam, 300, 1e-12) == RAOCP_OK && lam > 0);
        const double alpha = 0.999 / lam;
        CHECK(raocp_set_initial_state(c, x0.data()) == RAOCP_OK);
        CHECK(raocp_set_primal(c, z.data(), 0) == RAOCP_OK);
        CHECK(raocp_project_on_dynamics(c) == RAOCP_OK);
        if (dtype == RAOCP_F64) {
            CHECK(raocp_prox_f(c, alpha) == RAOCP_OK);
            CHECK(raocp_set_dual(c, eta.data(), 0) == RAOCP_OK);
            CHECK(raocp_prox_gconj(c, alpha) == RAOCP_OK);
        }
        const int K = 30;
        std::vector<double> err(3 * (K + 1)), derr(3 * (K + 1));
        int status = -1, iters = 0;
        CHECK(raocp_cp_run(c, x0.data(), K, 0.0, alpha, &status, &iters, err.data(), derr.data()) == RAOCP_OK);
        CHECK(iters == K + 1 && status == 1);
        CHECK(raocp_get_primal(c, z2.data(), 0) == RAOCP_OK && raocp_get_dual(c, eta2.data(), 0) == RAOCP_OK);
        float ms = 0;
        CHECK(raocp_cp_prepare(c, x0.data(), 29, alpha) == RAOCP_OK);
        CHECK(raocp_cp_bench(c, nullptr, 29, alpha, &ms) == RAOCP_OK);
        CHECK(raocp_cp_bench(c, nullptr, 29, alpha, &ms) == RAOCP_ERR_STATE);  // consumed
        CHECK(raocp_op_bench(c, 0, 10, &ms) == RAOCP_OK);
        CHECK(raocp_op_bench_rot(c, 1, 6, 3, &ms) == RAOCP_OK && ms > 0);
        CHECK(raocp_op_bench_rot(c, 2, 6, 3, &ms) == RAOCP_ERR_ARG);
        char kn[128];
        for (int op : {0, 1, 2, 6, 9, 10}) CHECK(raocp_kernel_info(c, op, kn, (int)sizeof(kn)) == RAOCP_OK && kn[0]);
        CHECK(raocp_kernel_info(c, 5, kn, (int)sizeof(kn)) == RAOCP_ERR_ARG);
        CHECK(raocp_reset_iterate(c) == RAOCP_OK);
        CHECK(raocp_get_primal(c, z2.data(), 0) == RAOCP_OK);
        for (int64_t i = 0; i < P; ++i) CHECK(z2[i] == 0.0);
        raocp_ctx_destroy(c);
    }
    // sharding: 2 shards in one process, device copies as the transport
    Problem pb(6, 20, 8);
    raocp_ctx* cs[2] = {nullptr, nullptr};
    for (int r = 0; r < 2; ++r) {
        CHECK(raocp_ctx_create(&pb.t, &pb.p, 0, &cs[r]) == RAOCP_OK);
        if (cs[r]) CHECK(raocp_shard_setup(cs[r], 2, r) == RAOCP_OK);
    }
    if (cs[0] && cs[1]) {
        double lam = 0;
        CHECK(raocp_step_size(cs[0], &lam, 300, 1e-12) == RAOCP_OK);
        std::vector<double> x0(pb.nx, 0.3), err(3 * 21), derr(3 * 21);
        int status = -1, iters = 0;
        CHECK(raocp_group_cp_run(cs, 2, x0.data(), 20, 0.0, 0.999 / lam, &status, &iters, err.data(), derr.data()) ==
              RAOCP_OK);
        CHECK(iters == 21);
        int32_t lo[16], hi[16];
        CHECK(raocp_shard_owned(cs[1], lo, hi, 16) >= 0);
    }
    for (auto* c : cs) raocp_ctx_destroy(c);
}

int main(int argc, char** argv) {
    const bool gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
    cpu_checks();
    if (gpu) gpu_checks();
    printf("abi_driver %s: %s\n", gpu ? "gpu" : "cpu", g_fail ? "FAILED" : "ok");
    fflush(stdout);
    return g_fail ? 1 : 0;
}
