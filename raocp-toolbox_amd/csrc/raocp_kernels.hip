// raocp_kernels.hip — HIP kernels for gfx950 (MI355X) implementing raocp's
// Chambolle–Pock inner loop on the reference's flat block layout.
//
// Mapping ("lanes over rows"): every kernel processes one kind of tree node
// ("group type"); a node is handled by a GROUP of G consecutive lanes, lane r of
// the group producing row r of that node's output blocks. A 256-thread workgroup
// holds floor(256/G) groups. Rows of one node are contiguous in the flat layout,
// so stores are coalesced; the node's inputs (parent state, child duals) are read
// once per lane from L1/L2 as broadcasts, and matrix tables are stored so lane r
// reads column-contiguous elements. Group reductions (SOC norms, AVaR kernel
// sums) go through LDS with workgroup barriers.
//
// Reference formulas are cited as /root/reference file:line.

#include "raocp_common.h"

namespace raocp {

constexpr int kBlock = 256;


// diagnostic timestamp (100 MHz constant clock), thread 0 only, when enabled
__device__ __forceinline__ void stamp(const Dev& p, int slot) {
    if (kDiag && p.stamps && threadIdx.x == 0 && blockIdx.x == 0) p.stamps[slot] = __builtin_amdgcn_s_memrealtime();
}


__device__ __forceinline__ int e3(const Dev& p, int j) { return p.E3 + 1 + (j - 1) * p.nx; }
__device__ __forceinline__ int e4(const Dev& p, int j) { return p.E4 + 1 + (j - 1) * p.nu; }
__device__ __forceinline__ int e11(const Dev& p, int l) { return p.E11 + p.m + (l - p.m) * p.nx; }

__device__ __forceinline__ int cdiv_dev(int a, int b) { return (a + b - 1) / b; }

__device__ __forceinline__ u64 dbits(double v) { return (u64)__double_as_longlong(v); }

// ---- batched dot products ----------------------------------------------------------
// All loads of a chunk are issued before its FMAs (a sched_barrier keeps hipcc from
// interleaving each load with its FMA, which pays the memory latency per element);
// two accumulators halve the dependent-FMA chain. N > 0: compile-time length (fully
// unrolled); N == 0: runtime length n, plain loop.
template <int N>
struct Chunk {
    static constexpr int C = N <= 8 ? N : 8;
};

// sum_k m[k*ms] * v[k]
template <int N, class PM, class PV>
__device__ __forceinline__ double dotb(PM m, int ms, PV v, int n) {
    if constexpr (N == 0) {
        double s = 0.0;
        for (int k = 0; k < n; ++k) s = fma(m[k * ms], v[k], s);
        return s;
    } else {
        constexpr int C = Chunk<N>::C;
        double s0 = 0.0, s1 = 0.0;
        _Pragma("unroll") for (int k0 = 0; k0 < N; k0 += C) {
            double a[C], b[C];
            _Pragma("unroll") for (int k = 0; k < C; ++k) if (k0 + k < N) {
                a[k] = m[(k0 + k) * ms];
                b[k] = v[k0 + k];
            }
            __builtin_amdgcn_sched_barrier(0);
            _Pragma("unroll") for (int k = 0; k < C; ++k) if (k0 + k < N) {
                if (k & 1) s1 = fma(a[k], b[k], s1);
                else s0 = fma(a[k], b[k], s0);
            }
        }
        return s0 + s1;
    }
}

// a = sum_k m[k*ms] (2 z[k] - p[k]),  b = sum_k m[k*ms] (z[k] - p[k])   (L of 2z+ - p and z+ - p)
template <int N, class PM, class PV>
__device__ __forceinline__ void dot_zp(PM m, int ms, PV z, PV pp, int n, double& a, double& b) {
    if constexpr (N == 0) {
        double sa = 0.0, sb = 0.0;
        for (int k = 0; k < n; ++k) {
            const double mk = m[k * ms], zk = z[k], pk = pp[k];
            sa = fma(mk, 2.0 * zk - pk, sa);
            sb = fma(mk, zk - pk, sb);
        }
        a = sa;
        b = sb;
    } else {
        constexpr int C = N <= 4 ? N : 4;
        double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
        _Pragma("unroll") for (int k0 = 0; k0 < N; k0 += C) {
            double mm[C], zz[C], qq[C];
            _Pragma("unroll") for (int k = 0; k < C; ++k) if (k0 + k < N) {
                mm[k] = m[(k0 + k) * ms];
                zz[k] = z[k0 + k];
                qq[k] = pp[k0 + k];
            }
            __builtin_amdgcn_sched_barrier(0);
            _Pragma("unroll") for (int k = 0; k < C; ++k) if (k0 + k < N) {
                const double w = 2.0 * zz[k] - qq[k], v = zz[k] - qq[k];
                if (k & 1) { a1 = fma(mm[k], w, a1); b1 = fma(mm[k], v, b1); }
                else { a0 = fma(mm[k], w, a0); b0 = fma(mm[k], v, b0); }
            }
        }
        a = a0 + a1;
        b = b0 + b1;
    }
}

// L^T of three duals at once: sA = m.dA, sW = m.(dP - dA), sC = m.c
template <int N, bool FULL, class PM, class PV>
__device__ __forceinline__ void dot_lt3(PM m, int ms, PV dA, PV dP, PV cc, int n, double& sA, double& sW,
                                        double& sC) {
    if constexpr (N == 0) {
        double a = 0.0, w = 0.0, c = 0.0;
        for (int k = 0; k < n; ++k) {
            const double mk = m[k * ms], va = dA[k];
            a = fma(mk, va, a);
            if (FULL) {
                w = fma(mk, dP[k] - va, w);
                c = fma(mk, cc[k], c);
            }
        }
        sA = a;
        sW = w;
        sC = c;
    } else {
        constexpr int C = N <= 4 ? N : 4;
        double a0 = 0.0, a1 = 0.0, w0 = 0.0, w1 = 0.0, c0 = 0.0, c1 = 0.0;
        _Pragma("unroll") for (int k0 = 0; k0 < N; k0 += C) {
            double mm[C], va[C], vp[C], vc[C];
            _Pragma("unroll") for (int k = 0; k < C; ++k) if (k0 + k < N) {
                mm[k] = m[(k0 + k) * ms];
                va[k] = dA[k0 + k];
                if (FULL) {
                    vp[k] = dP[k0 + k];
                    vc[k] = cc[k0 + k];
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            _Pragma("unroll") for (int k = 0; k < C; ++k) if (k0 + k < N) {
                if (k & 1) {
                    a1 = fma(mm[k], va[k], a1);
                    if (FULL) { w1 = fma(mm[k], vp[k] - va[k], w1); c1 = fma(mm[k], vc[k], c1); }
                } else {
                    a0 = fma(mm[k], va[k], a0);
                    if (FULL) { w0 = fma(mm[k], vp[k] - va[k], w0); c0 = fma(mm[k], vc[k], c0); }
                }
            }
        }
        sA = a0 + a1;
        sW = w0 + w1;
        sC = c0 + c1;
    }
}

// block-wide max of non-negative doubles -> one plain store per block (the per-block
// partials are reduced by k_cp_check; no atomics on a single hot address)
__device__ void block_max_store(double v, double* dst, double* s_red) {
    for (int off = 32; off > 0; off >>= 1) v = nmax(v, __shfl_xor(v, off, 64));
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_red[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = s_red[0];
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) b = nmax(b, s_red[i]);
        *dst = b;
    }
}

struct GroupIdx {
    int gl, r, per, node;
    bool live;
};

__device__ __forceinline__ GroupIdx group_index(int G, int begin, int end, int bid = -1) {
    GroupIdx g;
    g.per = blockDim.x / G;
    g.gl = threadIdx.x / G;
    g.r = threadIdx.x - g.gl * G;
    g.node = begin + (bid < 0 ? (int)blockIdx.x : bid) * g.per + g.gl;
    g.live = g.gl < g.per && g.node < end;
    return g;
}

#include "raocp_dyn.hip"
#include "raocp_dynf.hip"

// ---- LDS-DMA staging for the CP kernels (see raocp_dyn.hip: dma_gen) ----------------
// copy nbytes from an arbitrarily aligned global address into LDS at dst (16-B aligned):
// chunks start at the 16-B boundary below src; returns the shift in doubles (0 or 1) at
// which the data starts in dst. Sources have >= 16 B of slack after their end.
template <class PT>
__device__ __forceinline__ int dma_any(ldsd* dst, PT src, int nbytes, int* rot = nullptr) {
    const uintptr_t a = (uintptr_t)src;
    const int sh = (int)(a & 15);
    const char* s0 = (const char*)(a - sh);
    const int chunks = (sh + nbytes + 15) >> 4;
    const int g = dma_gen(dst, chunks, [=](int ch) { return (const double*)(s0 + 16 * ch); }, rot ? *rot : 0);
    if (rot) *rot += g;
    return sh >> 3;
}

#include "raocp_ell.hip"

// ==============================================================================
// AVaR kernel projection of (y_i, tau_children, s_children) (cache.py:290-317),
// closed form: r_k = alpha y_k - y_{c+k} + y_{2c} - tau_k - s_k,
// w = (r - 1 sum(r)/(a+c))/a with a = alpha^2 + 3; then
// y_k -= alpha w_k, y_{c+k} += w_k, y_{2c} -= sum(w), tau_k += w_k, s_k += w_k.
// Group per nonleaf: cmax lanes (one per child) + 1 lane for y_{2c}.
// ==============================================================================
__device__ __forceinline__ void kernel_proj_group(const Dev& p, int i, int c, int cs, int r, bool live, int base,
                                                  double* s_x, double (&vals)[4], double& y2c) {
    // vals = {y_k, y_{c+k}, tau_j, s_j} for lane r < c; y2c valid in lane cmax
    // lanes with r outside [0, cmax] (x/u lanes of the fused kernel) only join the barriers
    const int cmax = p.cmax;
    const bool mine = r >= 0 && r <= cmax;
    const double al = live ? p.alpha_r[i] : 0.0;
    if (mine && r == cmax) s_x[base + cmax] = y2c;
    __syncthreads();
    double rk = 0.0;
    if (live && r >= 0 && r < c) rk = al * vals[0] - vals[1] + s_x[base + cmax] - vals[2] - vals[3];
    __syncthreads();
    if (mine && r < cmax) s_x[base + r] = rk;
    __syncthreads();
    double sr = 0.0;
    if (live) for (int q = 0; q < c; ++q) sr += s_x[base + q];
    const double a = al * al + 3.0;
    double w = 0.0;
    if (live && r >= 0 && r < c) w = (rk - sr / (a + (double)c)) / a;
    __syncthreads();
    if (mine && r < cmax) s_x[base + r] = w;
    __syncthreads();
    if (live && r >= 0 && r < c) {
        vals[0] -= al * w;
        vals[1] += w;
        vals[2] += w;
        vals[3] += w;
    }
    if (live && r == cmax) {
        double sw = 0.0;
        for (int q = 0; q < c; ++q) sw += s_x[base + q];
        y2c -= sw;
    }
}

__global__ void __launch_bounds__(kBlock) k_kernel_proj(Dev p, double* __restrict__ z) {
    __shared__ double s_x[kBlock];
    const int G = p.cmax + 1;
    GroupIdx g = group_index(G, 0, p.m);
    const int i = g.node, r = g.r, base = g.gl * G;
    int c = 0, cs = 0;
    if (g.live) { c = p.nch[i]; cs = p.ch_start[i]; }
    double vals[4] = {0, 0, 0, 0};
    double y2c = 0.0;
    double* y = z + p.Y0 + (g.live ? p.yrel[i] : 0);
    if (g.live && r < c) {
        const int j = cs + r;
        vals[0] = y[r]; vals[1] = y[c + r]; vals[2] = z[p.T0 + j]; vals[3] = z[p.S0 + j];
    }
    if (g.live && r == p.cmax) y2c = y[2 * c];
    kernel_proj_group(p, i, c, cs, r, g.live, base, s_x, vals, y2c);
    if (g.live && r < c) {
        const int j = cs + r;
        y[r] = vals[0]; y[c + r] = vals[1]; z[p.T0 + j] = vals[2]; z[p.S0 + j] = vals[3];
    }
    if (g.live && r == p.cmax) y[2 * c] = y2c;
}

__global__ void k_relax_s0(Dev p, double* z, double alpha) { z[p.S0] -= alpha; }

// ==============================================================================
// CP primal kernel: z_half = p - alpha L^T(d), s_0 -= alpha, AVaR kernel projection
// of (y, tau, s) fused (those are final after it); x, u go on to the dynamics sweep.
// FULL: also finishes the previous iteration's residuals (solver.py:63-95):
//   w = L^T(d_prev - eta+),  xi1 = (p_prev - z+)/alpha - w,  xi0 = xi1 + L^T xi2,
//   delta1 = z+ - p_prev,    delta0 = delta1 + w   (== delta1 - L^T(eta+ - d_prev))
// Buffers rotate with the iteration counter k (read from ctl):
//   FULL=false (initial): p = Z[k], d = E[k], out -> Z[k+1]
//   FULL=true (end of k): p_prev = Z[k], z+ = Z[k+1], d_prev = E[k], eta+ = E[k+1],
//                         out z_half(k+1) -> Z[k+2]
// Group types: nonleaf i (x rows, u rows, one lane per child for y/tau/s, one lane
// for y_2c and the root's s_0), leaf l (x rows).
// ==============================================================================
struct LtIn {
    const double* a;   // primary dual
    const double* b;   // secondary (FULL: d_prev) -> w uses b - a
    const double* c;   // xi2
};

template <bool FULL, int NXc, int NUc>
__global__ void __launch_bounds__(kBlock) k_cp_primal(Dev p, Ctl* __restrict__ ctl, Bufs bf,
                                                       const double* __restrict__ xi2,
                                                       double* __restrict__ part, int nbA, int blk0) {
    __shared__ double s_x[kBlock];
    __shared__ double s_red[4][kBlock / 64];
    const int bid = blockIdx.x + blk0;  // blk0: role offset (op_bench times one role alone)
    if (ctl->done) return;
    const int kk = 0;  // buffers arrive rotated for this iteration (enqueue_cp_iteration)
    const double alpha = ctl->alpha;
    const glbd* pz = pick3(bf, kk);                        // p (FULL: p_prev)
    const glbd* zp = pick3(bf, kk + 1);                    // z+ (FULL)
    glbd* out = FULL ? pick3(bf, kk + 2) : pick3(bf, kk + 1);
    const glbd* dA = FULL ? pick2(bf, kk + 1) : pick2(bf, kk);   // dual whose L^T makes z_half
    const glbd* dP = pick2(bf, kk);                              // d_prev (FULL)
    const glbd* src = FULL ? zp : pz;                            // primal the half step starts from
    const glbd* xi2g = (const glbd*)xi2;
    const int nx = NXc ? NXc : p.nx, nu = NUc ? NUc : p.nu;
    double m0 = 0.0, m1 = 0.0, m3 = 0.0, m4 = 0.0;   // |xi0| |xi1| |delta0| |delta1|
    auto account = [&](int e, double lt_half, double w, double ltxi2) {
        // e: flat primal index; lt_half = L^T(eta+) (FULL) ; returns nothing
        (void)lt_half;
        const double pp = pz[e], zz = zp[e];
        const double x1 = (pp - zz) / alpha - w;
        const double x0v = x1 + ltxi2;
        const double dl1 = zz - pp;
        const double dl0 = dl1 + w;
        m0 = nmax(m0, fabs(x0v)); m1 = nmax(m1, fabs(x1)); m3 = nmax(m3, fabs(dl0)); m4 = nmax(m4, fabs(dl1));
    };
    if (bid < nbA) {
        const int G = nx + nu + p.cmax + 1;
        GroupIdx g = group_index(G, 0, p.m, bid);
        const int i = g.node, r = g.r, base = g.gl * G;
        int c = 0, cs = 0, o7 = -1;
        if (g.live) { c = p.nch[i]; cs = p.ch_start[i]; o7 = p.e7off[i]; }
        if (g.live && r < nx + nu) {
            // x / u rows: sum over children of sqrtQ_j eta3_j (sqrtR_j eta4_j) + Gamma' eta7
            const bool isx = r < nx;
            const int rr = isx ? r : r - nx;
            double accA = 0.0, accW = 0.0, accC = 0.0;
            if (o7 >= 0) {
                const int e = o7 + (isx ? rr : nx + rr);
                accA = dA[e];
                if (FULL) { accW = dP[e] - dA[e]; accC = xi2[e]; }
            }
            for (int q = 0; q < c; ++q) {
                const int j = cs + q;
                double sA = 0.0, sW = 0.0, sC = 0.0;
                if (isx) {
                    const double* M = p.SQ + (size_t)p.iSQ[j] * nx * nx;
                    const int eb = e3(p, j);
                    dot_lt3<NXc, FULL>(M + rr, nx, dA + eb, dP + eb, xi2g + eb, nx, sA, sW, sC);
                } else {
                    const double* M = p.SR + (size_t)p.iSR[j] * nu * nu;
                    const int eb = e4(p, j);
                    dot_lt3<NUc, FULL>(M + rr, nu, dA + eb, dP + eb, xi2g + eb, nu, sA, sW, sC);
                }
                accA += sA;
                if (FULL) { accW += sW; accC += sC; }
            }
            const int e = isx ? p.X0 + i * nx + rr : p.U0 + i * nu + rr;
            out[e] = src[e] - alpha * accA;
            if (FULL) account(e, accA, accW, accC);
        }
        // AVaR kernel block: lane r - (nx+nu) < cmax -> child; == cmax -> y_2c (and root s_0)
        const int rk = r - (nx + nu);
        double vals[4] = {0, 0, 0, 0};
        double y2c = 0.0;
        const int yo = g.live ? p.yrel[i] : 0;
        const double e2A = g.live ? dA[p.E2 + i] : 0.0;
        double e2W = 0.0, e2C = 0.0;
        if (FULL && g.live) { e2W = dP[p.E2 + i] - dA[p.E2 + i]; e2C = xi2[p.E2 + i]; }
        if (g.live && rk >= 0 && rk < c) {
            const int j = cs + rk;
            const double b = p.cond[j];
            // y_k, y_{c+k}: eta1 - b eta2
            const int ey0 = p.Y0 + yo + rk, ey1 = p.Y0 + yo + c + rk;
            const int f0 = p.E1 + yo + rk, f1 = p.E1 + yo + c + rk;
            const double lt0 = dA[f0] - b * e2A, lt1 = dA[f1] - 0.0 * e2A;
            vals[0] = src[ey0] - alpha * lt0;
            vals[1] = src[ey1] - alpha * lt1;
            // tau_j = (eta5 + eta6)/2
            const double ltt = 0.5 * (dA[p.E5 + j] + dA[p.E6 + j]);
            vals[2] = src[p.T0 + j] - alpha * ltt;
            // s_j = eta2_j (nonleaf child) or (eta12 + eta13)/2 (leaf child)
            const double lts = j < p.m ? dA[p.E2 + j] : 0.5 * (dA[p.E12 + j] + dA[p.E13 + j]);
            vals[3] = src[p.S0 + j] - alpha * lts;
            if (FULL) {
                const double w0 = (dP[f0] - dA[f0]) - b * e2W, c0 = xi2[f0] - b * e2C;
                const double w1 = (dP[f1] - dA[f1]) - 0.0 * e2W, c1 = xi2[f1] - 0.0 * e2C;
                const double wt = 0.5 * ((dP[p.E5 + j] - dA[p.E5 + j]) + (dP[p.E6 + j] - dA[p.E6 + j]));
                const double ct = 0.5 * (xi2[p.E5 + j] + xi2[p.E6 + j]);
                double ws, cs2;
                if (j < p.m) { ws = dP[p.E2 + j] - dA[p.E2 + j]; cs2 = xi2[p.E2 + j]; }
                else {
                    ws = 0.5 * ((dP[p.E12 + j] - dA[p.E12 + j]) + (dP[p.E13 + j] - dA[p.E13 + j]));
                    cs2 = 0.5 * (xi2[p.E12 + j] + xi2[p.E13 + j]);
                }
                account(ey0, 0, w0, c0);
                account(ey1, 0, w1, c1);
                account(p.T0 + j, 0, wt, ct);
                account(p.S0 + j, 0, ws, cs2);
            }
        }
        if (g.live && rk == p.cmax) {
            const int f2 = p.E1 + yo + 2 * c, ey2 = p.Y0 + yo + 2 * c;
            y2c = src[ey2] - alpha * (dA[f2] - 1.0 * e2A);
            if (FULL) account(ey2, 0, (dP[f2] - dA[f2]) - 1.0 * e2W, xi2[f2] - 1.0 * e2C);
            if (i == 0) {
                // root s_0: L^T -> eta2_0 ; then the relaxation prox s_0 -= alpha (cache.py:253-257)
                out[p.S0] = (src[p.S0] - alpha * e2A) - alpha;
                if (FULL) account(p.S0, 0, e2W, e2C);
            }
        }
        kernel_proj_group(p, i, c, cs, rk, g.live && rk >= 0, base + nx + nu, s_x, vals, y2c);
        if (g.live && rk >= 0 && rk < c) {
            const int j = cs + rk;
            out[p.Y0 + yo + rk] = vals[0];
            out[p.Y0 + yo + c + rk] = vals[1];
            out[p.T0 + j] = vals[2];
            out[p.S0 + j] = vals[3];
        }
        if (g.live && rk == p.cmax) out[p.Y0 + yo + 2 * c] = y2c;
    } else {
        // leaf l: x = sqrtPf eta11 + eta14
        const int G = nx;
        const int lb = bid - nbA;
        const int per = blockDim.x / G, gl = threadIdx.x / G, r = threadIdx.x - gl * G;
        const int l = p.m + lb * per + gl;
        if (gl < per && l < p.n) {
            const double* M = p.SP + (size_t)p.iSP[l] * nx * nx;
            const int eb = e11(p, l);
            double sA = 0.0, sW = 0.0, sC = 0.0;
            dot_lt3<NXc, FULL>(M + r, nx, dA + eb, dP + eb, xi2g + eb, nx, sA, sW, sC);
            const int o14 = p.e14off[l - p.m];
            if (o14 >= 0) {
                sA += dA[o14 + r];
                if (FULL) { sW += dP[o14 + r] - dA[o14 + r]; sC += xi2[o14 + r]; }
            }
            const int e = p.X0 + l * nx + r;
            out[e] = src[e] - alpha * sA;
            if (FULL) account(e, sA, sW, sC);
        }
    }
    if (FULL) {
        double* prow = part + (size_t)bid * 6;
        block_max_store(m0, prow + 0, s_red[0]);
        block_max_store(m1, prow + 1, s_red[1]);
        block_max_store(m3, prow + 3, s_red[2]);
        block_max_store(m4, prow + 4, s_red[3]);
    }
}

// ==============================================================================
// CP dual kernel (solver.py:44-61 + cache.py:321-393 + residual part of 63-95):
//   a = L(2 z+ - p), b = L(z+ - p), eta_half = d + alpha a,
//   v = eta_half/alpha -+ 1/2 (eta5, eta12: -1/2; eta6, eta13: +1/2)
//   eta+ = alpha (v - Pi(v)),   xi2 = (d - eta+)/alpha + b,   delta2 = eta+ - d
// Pi: eta1 -> [max(0, .) (2c); identity], eta2 -> max(0, .), per child j the SOC on
// (eta3, eta4, eta5 | eta6), eta7 box, per leaf SOC on (eta11, eta12 | eta13), eta14 box.
// WITH_L = false is the standalone prox_gconj (Cache.proximal_of_g_conjugate) on `d`
// in place (eta_half = d).
// ==============================================================================
__device__ __forceinline__ double soc_apply(double v, bool is_t, double nf, double t) {
    // SecondOrderCone.project (cones.py:113-132) for one coordinate of the block
    if (nf <= t) return v;
    if (nf <= -t) return 0.0;
    const double s = (nf + t) / 2.0;
    return is_t ? s : s * (v / nf);
}

__device__ __forceinline__ double box_apply(double v, double lo, double hi, Ctl* ctl) {
    // Rectangle._constrain (rectangle.py:50-59)
    if (lo <= v && v <= hi) return v;
    if (v <= lo) return lo;
    if (v >= hi) return hi;
    atomicOr(&ctl->flags, 1);
    return v;
}

// mode (standalone only): bit0 PROX (scale, halves, Moreau output) else projection output Pi(d);
// bit1 process the nonleaf part (eta1..eta7, SOC per child); bit2 the leaf part (eta11..eta14).
enum { kDualProx = 1, kDualNonleaf = 2, kDualLeaf = 4, kDualAll = 7 };
constexpr int kStageDual = 1536;  // doubles of LDS staging per dual block (host checks the need)
constexpr int kStageMat = 2048;   // doubles of LDS for the L weight tables when they fit

template <bool WITH_L, int NXc, int NUc>
__global__ void __launch_bounds__(kBlock) k_cp_dual(Dev p, Ctl* __restrict__ ctl, Bufs bf,
                                                     double* __restrict__ xi2, double* dsolo,
                                                     double* __restrict__ part, int nbA, int nbB, int mode, int blk0) {
    const int bid = blockIdx.x + blk0;  // blk0: role offset (op_bench times one role alone)
    __shared__ double s_x[kBlock];
    __shared__ double s_red[2][kBlock / 64];
    __shared__ __attribute__((aligned(16))) double s_stage[kStageDual + kStageMat];
    if (WITH_L && ctl->done) return;
    if (!WITH_L) {
        const bool leafpart = bid >= nbA + nbB;
        if (leafpart && !(mode & kDualLeaf)) return;
        if (!leafpart && !(mode & kDualNonleaf)) return;
    }
    const bool prox = WITH_L || (mode & kDualProx);
    const int kk = 0;  // buffers arrive rotated for this iteration (enqueue_cp_iteration)
    const double alpha = ctl->alpha;
    const glbd* pz = pick3(bf, kk);
    const glbd* zp = pick3(bf, kk + 1);
    const glbd* d = WITH_L ? pick2(bf, kk) : (const glbd*)dsolo;
    glbd* eo = WITH_L ? pick2(bf, kk + 1) : (glbd*)dsolo;
    const int nx = NXc ? NXc : p.nx, nu = NUc ? NUc : p.nu;
    double m2 = 0.0, m5 = 0.0;
    // finalize one dual element given a = L(2z+ - p)[e], b = L(z+ - p)[e], projection result pv of v
    auto finish = [&](int e, double v, double pv, double b) {
        const double ep = prox ? alpha * (v - pv) : pv;
        eo[e] = ep;
        if (WITH_L) {
            const double de = d[e];
            const double x2 = (de - ep) / alpha + b;
            xi2[e] = x2;
            m2 = nmax(m2, fabs(x2));
            m5 = nmax(m5, fabs(ep - de));
        }
    };
    if (WITH_L && bid < nbA) {
        // child block j: rows eta3 (nx), eta4 (nu), eta5, eta6 -> one SOC of dim nx+nu+2.
        // Everything the block reads is staged into LDS by LDS-DMA first (one round trip):
        // the parents' x, u rows of z+ and p, the children's tau, the four dual ranges and
        // the child records {anc, iSQ, iSR}.
        const int G = nx + nu + 2;
        const int per = blockDim.x / G;
        const int j0 = 1 + bid * per, j1 = min(p.n, j0 + per), J = j1 - j0;
        const Rec br = p.dblk[bid];
        const int a0 = br.x, na = br.y - br.x + 1;
        ldsd* sb = (ldsd*)s_stage;
        int o = 0;
        auto region = [&](int count) { const int r0 = o; o += rup(count, 2) + 2; return r0; };
        const int oXz = region(na * nx), oXp = region(na * nx), oUz = region(na * nu), oUp = region(na * nu);
        const int oTz = region(J), oTp = region(J), oD3 = region(J * nx), oD4 = region(J * nu), oD5 = region(J),
                  oD6 = region(J), oCR = region(2 * J);
        const int hXz = dma_any(sb + oXz, zp + p.X0 + (size_t)a0 * nx, na * nx * 8);
        const int hXp = dma_any(sb + oXp, pz + p.X0 + (size_t)a0 * nx, na * nx * 8);
        const int hUz = dma_any(sb + oUz, zp + p.U0 + (size_t)a0 * nu, na * nu * 8);
        const int hUp = dma_any(sb + oUp, pz + p.U0 + (size_t)a0 * nu, na * nu * 8);
        const int hTz = dma_any(sb + oTz, zp + p.T0 + j0, J * 8);
        const int hTp = dma_any(sb + oTp, pz + p.T0 + j0, J * 8);
        const int hD3 = dma_any(sb + oD3, d + e3(p, j0), J * nx * 8);
        const int hD4 = dma_any(sb + oD4, d + e4(p, j0), J * nu * 8);
        const int hD5 = dma_any(sb + oD5, d + p.E5 + j0, J * 8);
        const int hD6 = dma_any(sb + oD6, d + p.E6 + j0, J * 8);
        dma_any(sb + oCR, (const glbd*)(p.crec + j0), J * 16);
        const int nQ = p.nSQ * nx * nx, nR = p.nSR * nu * nu;
        const bool mlds = nQ + nR + 4 <= kStageMat;  // weight tables staged too
        const int oSQ = kStageDual, oSR = oSQ + rup(nQ, 2);
        if (mlds) {
            dma_any(sb + oSQ, p.SQ, nQ * 8);
            dma_any(sb + oSR, p.SR, nR * 8);
        }
        dma_wait();
        lds_sync();
        const ldsd* Xz = sb + oXz + hXz; const ldsd* Xp = sb + oXp + hXp;
        const ldsd* Uz = sb + oUz + hUz; const ldsd* Up = sb + oUp + hUp;
        const ldsd* Tz = sb + oTz + hTz; const ldsd* Tp = sb + oTp + hTp;
        const ldsd* D3 = sb + oD3 + hD3; const ldsd* D4 = sb + oD4 + hD4;
        const ldsd* D5 = sb + oD5 + hD5; const ldsd* D6 = sb + oD6 + hD6;
        const ldsrec* CR = (const ldsrec*)(sb + oCR);
        const int gl = threadIdx.x / G, r = threadIdx.x - gl * G, base = gl * G;
        const int jj = gl, j = j0 + gl;
        const bool live = gl < per && j < j1;
        double v = 0.0, bb = 0.0, dv = 0.0;
        int e = -1;
        if (live) {
            const Rec cr = CR[jj];
            const int ai = cr.x - a0;
            double av = 0.0;
            if (r < nx) {
                e = e3(p, j) + r;
                dv = D3[jj * nx + r];
                if (mlds) dot_zp<NXc>(sb + oSQ + (size_t)cr.y * nx * nx + r, nx, Xz + ai * nx, Xp + ai * nx, nx, av, bb);
                else dot_zp<NXc>(p.SQ + (size_t)cr.y * nx * nx + r, nx, Xz + ai * nx, Xp + ai * nx, nx, av, bb);
            } else if (r < nx + nu) {
                const int rr = r - nx;
                e = e4(p, j) + rr;
                dv = D4[jj * nu + rr];
                if (mlds) dot_zp<NUc>(sb + oSR + (size_t)cr.z * nu * nu + rr, nu, Uz + ai * nu, Up + ai * nu, nu, av, bb);
                else dot_zp<NUc>(p.SR + (size_t)cr.z * nu * nu + rr, nu, Uz + ai * nu, Up + ai * nu, nu, av, bb);
            } else {
                const bool five = r == nx + nu;
                e = (five ? p.E5 : p.E6) + j;
                dv = five ? D5[jj] : D6[jj];
                const double zt = Tz[jj], pt = Tp[jj];
                av = 0.5 * (2.0 * zt - pt);
                bb = 0.5 * (zt - pt);
            }
            v = (dv + alpha * av) / alpha;
            if (r == nx + nu) v += -0.5;
            if (r == nx + nu + 1) v += 0.5;
        }
        // ||f||, f = rows 0..G-2, t = row G-1
        s_x[threadIdx.x] = (live && r < G - 1) ? v * v : 0.0;
        if (live && r == G - 1) s_x[threadIdx.x] = v;
        __syncthreads();
        if (live) {
            double ss = 0.0;
            for (int q = 0; q < G - 1; ++q) ss += s_x[base + q];
            const double nf = sqrt(ss), t = s_x[base + G - 1];
            const double pv = soc_apply(v, r == G - 1, nf, t);
            const double ep = alpha * (v - pv);
            eo[e] = ep;
            const double x2 = (dv - ep) / alpha + bb;
            xi2[e] = x2;
            m2 = nmax(m2, fabs(x2));
            m5 = nmax(m5, fabs(ep - dv));
        }
    } else if (bid < nbA) {  // standalone prox_g* (no L): direct global reads
        // child block j: rows eta3 (nx), eta4 (nu), eta5, eta6 -> one SOC of dim nx+nu+2
        const int G = nx + nu + 2;
        GroupIdx g = group_index(G, 1, p.n, bid);
        const int j = g.node, r = g.r, base = g.gl * G;
        double v = 0.0, bb = 0.0;
        int e = -1;
        if (g.live) {
            const int a = p.anc[j];
            double av = 0.0;
            if (r < nx) {
                e = e3(p, j) + r;
                if (WITH_L) {
                    const double* M = p.SQ + (size_t)p.iSQ[j] * nx * nx;
                    const glbd* xz = zp + p.X0 + (size_t)a * nx;
                    const glbd* xp = pz + p.X0 + (size_t)a * nx;
                    dot_zp<NXc>(M + r, nx, xz, xp, nx, av, bb);
                }
            } else if (r < nx + nu) {
                const int rr = r - nx;
                e = e4(p, j) + rr;
                if (WITH_L) {
                    const double* M = p.SR + (size_t)p.iSR[j] * nu * nu;
                    const glbd* uz = zp + p.U0 + (size_t)a * nu;
                    const glbd* up = pz + p.U0 + (size_t)a * nu;
                    dot_zp<NUc>(M + rr, nu, uz, up, nu, av, bb);
                }
            } else {
                e = (r == nx + nu ? p.E5 : p.E6) + j;
                if (WITH_L) {
                    const double zt = zp[p.T0 + j], pt = pz[p.T0 + j];
                    av = 0.5 * (2.0 * zt - pt);
                    bb = 0.5 * (zt - pt);
                }
            }
            const double eh = WITH_L ? d[e] + alpha * av : d[e];
            v = prox ? eh / alpha : eh;
            if (prox && r == nx + nu) v += -0.5;
            if (prox && r == nx + nu + 1) v += 0.5;
        }
        // ||f||, f = rows 0..G-2, t = row G-1
        s_x[threadIdx.x] = (g.live && r < G - 1) ? v * v : 0.0;
        if (g.live && r == G - 1) s_x[threadIdx.x] = v;
        __syncthreads();
        if (g.live) {
            double ss = 0.0;
            for (int q = 0; q < G - 1; ++q) ss += s_x[base + q];
            const double nf = sqrt(ss), t = s_x[base + G - 1];
            finish(e, v, soc_apply(v, r == G - 1, nf, t), bb);
        }
    } else if (bid < nbA + nbB) {
        // nonleaf i: eta1 (2c+1), eta2, eta7 (nx+nu)
        const int G = 2 * p.cmax + 2 + nx + nu;
        const int lb = bid - nbA;
        const int per = blockDim.x / G, gl = threadIdx.x / G, r = threadIdx.x - gl * G;
        const int i = lb * per + gl;
        if (gl < per && i < p.m) {
            const int c = p.nch[i], cs = p.ch_start[i];
            const int yo = p.yrel[i];
            if (r < 2 * c + 1) {
                const int e = p.E1 + yo + r;
                double av = 0.0, bb = 0.0;
                if (WITH_L) {
                    const double zy = zp[p.Y0 + yo + r], py = pz[p.Y0 + yo + r];
                    av = 2.0 * zy - py;
                    bb = zy - py;
                }
                const double v = prox ? (WITH_L ? d[e] + alpha * av : d[e]) / alpha : d[e];
                const double pv = r < 2 * c ? fmax(v, 0.0) : v;
                finish(e, v, pv, bb);
            } else if (r == 2 * p.cmax + 1) {
                const int e = p.E2 + i;
                double av = 0.0, bb = 0.0;
                if (WITH_L) {
                    const glbd* yz = zp + p.Y0 + yo;
                    const glbd* yp = pz + p.Y0 + yo;
                    double bya = 0.0, byb = 0.0;
                    for (int k = 0; k < c; ++k) {
                        const double cp = p.cond[cs + k];
                        bya = fma(cp, 2.0 * yz[k] - yp[k], bya);
                        byb = fma(cp, yz[k] - yp[k], byb);
                    }
                    bya += 2.0 * yz[2 * c] - yp[2 * c];
                    byb += yz[2 * c] - yp[2 * c];
                    const double zs = zp[p.S0 + i], ps = pz[p.S0 + i];
                    av = (2.0 * zs - ps) - bya;
                    bb = (zs - ps) - byb;
                }
                const double v = prox ? (WITH_L ? d[e] + alpha * av : d[e]) / alpha : d[e];
                finish(e, v, fmax(v, 0.0), bb);
            } else if (r >= 2 * p.cmax + 2) {
                const int rr = r - (2 * p.cmax + 2);
                const int o7 = p.e7off[i];
                if (o7 >= 0) {
                    const int e = o7 + rr;
                    double av = 0.0, bb = 0.0;
                    if (WITH_L) {
                        const int ez = rr < nx ? p.X0 + i * nx + rr : p.U0 + i * nu + rr - nx;
                        av = 2.0 * zp[ez] - pz[ez];
                        bb = zp[ez] - pz[ez];
                    }
                    const double v = prox ? (WITH_L ? d[e] + alpha * av : d[e]) / alpha : d[e];
                    const int bi = p.iBnl[i];
                    const double pv = box_apply(v, p.blo_nl[(size_t)bi * (nx + nu) + rr],
                                                p.bhi_nl[(size_t)bi * (nx + nu) + rr], ctl);
                    finish(e, v, pv, bb);
                }
            }
        }
    } else {
        // leaf l: eta11 (nx), eta12, eta13 -> SOC of dim nx+2 ; eta14 (nx) box
        const int G = 2 * nx + 2;
        const int lb = bid - nbA - nbB;
        const int per = blockDim.x / G, gl = threadIdx.x / G, r = threadIdx.x - gl * G;
        const int l = p.m + lb * per + gl;
        const bool live = gl < per && l < p.n;
        const int base = gl * G;
        double v = 0.0, bb = 0.0;
        int e = -1;
        if (live) {
            double av = 0.0;
            if (r < nx) {
                e = e11(p, l) + r;
                if (WITH_L) {
                    const double* M = p.SP + (size_t)p.iSP[l] * nx * nx;
                    const glbd* xz = zp + p.X0 + (size_t)l * nx;
                    const glbd* xp = pz + p.X0 + (size_t)l * nx;
                    dot_zp<NXc>(M + r, nx, xz, xp, nx, av, bb);
                }
            } else if (r < nx + 2) {
                e = (r == nx ? p.E12 : p.E13) + l;
                if (WITH_L) {
                    const double zs = zp[p.S0 + l], ps = pz[p.S0 + l];
                    av = 0.5 * (2.0 * zs - ps);
                    bb = 0.5 * (zs - ps);
                }
            } else {
                const int o14 = p.e14off[l - p.m];
                if (o14 >= 0) {
                    const int rr = r - nx - 2;
                    e = o14 + rr;
                    if (WITH_L) {
                        const int ez = p.X0 + l * nx + rr;
                        av = 2.0 * zp[ez] - pz[ez];
                        bb = zp[ez] - pz[ez];
                    }
                }
            }
            if (e >= 0) {
                v = prox ? (WITH_L ? d[e] + alpha * av : d[e]) / alpha : d[e];
                if (prox && r == nx) v += -0.5;
                if (prox && r == nx + 1) v += 0.5;
            }
        }
        s_x[threadIdx.x] = (live && r < nx + 1) ? v * v : 0.0;
        if (live && r == nx + 1) s_x[threadIdx.x] = v;
        __syncthreads();
        if (live && e >= 0) {
            if (r < nx + 2) {
                double ss = 0.0;
                for (int q = 0; q < nx + 1; ++q) ss += s_x[base + q];
                finish(e, v, soc_apply(v, r == nx + 1, sqrt(ss), s_x[base + nx + 1]), bb);
            } else {
                const int rr = r - nx - 2;
                const int bi = p.iBl[l];
                finish(e, v, box_apply(v, p.blo_l[(size_t)bi * nx + rr], p.bhi_l[(size_t)bi * nx + rr], ctl), bb);
            }
        }
    }
    if (WITH_L) {
        double* prow = part + (size_t)bid * 6;
        block_max_store(m2, prow + 2, s_red[0]);
        block_max_store(m5, prow + 5, s_red[1]);
    }
}

#include "raocp_cp2.hip"
#include "raocp_cp.hip"
#include "raocp_ell2.hip"
#include "raocp_ell3.hip"
#include "raocp_cp3.hip"
#include "raocp_dyn3.hip"
#include "raocp_dyn2.hip"

// ---- element-wise dual sub-steps of prox_g* (cache.py:329-347, 392-393)
__global__ void k_div(double* __restrict__ x, double a, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) x[i] = x[i] / a;
}
__global__ void k_add_const(double* __restrict__ x, double c, int begin, int end) {
    for (int i = begin + blockIdx.x * blockDim.x + threadIdx.x; i < end; i += gridDim.x * blockDim.x) x[i] = x[i] + c;
}
__global__ void k_moreau(double* __restrict__ x, const double* __restrict__ vhat, double a, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) x[i] = a * (vhat[i] - x[i]);
}
__global__ void k_zero_idx(double* __restrict__ x, const int* __restrict__ idx, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) x[idx[i]] = 0.0;
}

// the control block and the error word to pinned host memory (one thread, after its updates)
__device__ __forceinline__ void publish_ctl(const Ctl* ctl, CtlPub* pub, const unsigned* errw) {
    pub->ctl = *ctl;
    pub->err = errw ? *errw : 0u;
    __threadfence_system();
}

// end of iteration: record residuals, stopping test (solver.py:137-161)
// nanbit: as ChkArg::nanbit (0: the CP kernels raise bit 0 themselves); pub (a batch's last
// test): the control block and the error word errw published to pinned host memory
__global__ void __launch_bounds__(kBlock) k_cp_check(Ctl* ctl, double* hist, const double* __restrict__ part,
                                                      int rows, int nanbit, CtlPub* pub, const unsigned* errw) {
    __shared__ double s_m[6][kBlock];
    if (ctl->done) {
        if (pub && threadIdx.x == 0) publish_ctl(ctl, pub, errw);
        return;
    }
    double m[6] = {0, 0, 0, 0, 0, 0};
    // (four rows per lane per round: their loads go out together)
    _Pragma("unroll 4") for (int r = threadIdx.x; r < rows; r += blockDim.x)
        _Pragma("unroll") for (int q = 0; q < 6; ++q) m[q] = nmax(m[q], part[(size_t)r * 6 + q]);
    _Pragma("unroll") for (int q = 0; q < 6; ++q) s_m[q][threadIdx.x] = m[q];
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            _Pragma("unroll") for (int q = 0; q < 6; ++q) s_m[q][threadIdx.x] = nmax(s_m[q][threadIdx.x], s_m[q][threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const int k = ctl->k;
    for (int q = 0; q < 6; ++q) hist[(size_t)k * 6 + q] = s_m[q][0];
    const double err = nmax(nmax(s_m[0][0], s_m[1][0]), s_m[2][0]);  // NaN: not converged
    if (ctl->flags & nanbit) ctl->flags |= 1;
    if (k >= ctl->max_iters || err <= ctl->tol || (ctl->flags & 1)) {
        ctl->done = 1;
        ctl->final_k = k;
    } else {
        ctl->k = k + 1;
    }
    if (pub) publish_ctl(ctl, pub, errw);
}

// ---- subtree sharding (raocp_capi.hip, raocp_shard_setup): exchange packing and the
// residual reduction split around the all-reduce
// recv holds R slices of maxc rows of w doubles; slice r goes to dst rows lo_r .. lo_r + cnt_r
template <class T>
__global__ void k_scatter_rows(const T* __restrict__ recv, T* __restrict__ dst, const int* __restrict__ slc,
                               int R, int maxc, int w) {
    const int tot = R * maxc * w;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += gridDim.x * blockDim.x) {
        const int r = e / (maxc * w), rem = e - r * maxc * w, i = rem / w, k = rem - i * w;
        if (i < slc[2 * r + 1]) dst[(size_t)(slc[2 * r] + i) * w + k] = recv[e];
    }
}
// X1 record of a shard (stride 2 maxc + 16 doubles): the (a[i], b[i]) pairs of its owned
// roots, then the 16-double residual record of its PREVIOUS iteration (k_cp_reduce; the
// stopping test runs one iteration late, so the residual all-reduce rides on this
// all-gather: two collectives per iteration)
// (the message is fp64; T = the context's scalar type of a / b)
template <class T>
__global__ void k_pack_x1(double* __restrict__ send, const T* __restrict__ a, const T* __restrict__ b, int cnt,
                          int maxc, const double* __restrict__ red16) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
        send[2 * i] = a[i];
        send[2 * i + 1] = b[i];
    }
    if (blockIdx.x == 0 && threadIdx.x < 16) send[2 * maxc + threadIdx.x] = red16[threadIdx.x];
}
template <class T>
__global__ void k_unpack_x1(const double* __restrict__ recv, T* __restrict__ a, T* __restrict__ b,
                            const int* __restrict__ slc, int R, int maxc) {
    const int stride = 2 * maxc + 16;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < R * maxc; e += gridDim.x * blockDim.x) {
        const int r = e / maxc, i = e - r * maxc;
        if (i < slc[2 * r + 1]) {
            a[slc[2 * r] + i] = (T)recv[(size_t)r * stride + 2 * i];
            b[slc[2 * r] + i] = (T)recv[(size_t)r * stride + 2 * i + 1];
        }
    }
}
// local part of k_cp_check: this shard's six maxima -> red6[0..5], the NaN-in-box flag -> red6[6],
// NaN-maximum flags -> red6[8..13] (16 doubles, then all-reduced with max)
__global__ void __launch_bounds__(kBlock) k_cp_reduce(const Ctl* ctl, const double* __restrict__ part, int rows,
                                                      double* red6) {
    __shared__ double s_m[6][kBlock];
    if (ctl->done) return;
    double m[6] = {0, 0, 0, 0, 0, 0};
    for (int r = threadIdx.x; r < rows; r += blockDim.x)
        _Pragma("unroll") for (int q = 0; q < 6; ++q) m[q] = nmax(m[q], part[(size_t)r * 6 + q]);
    _Pragma("unroll") for (int q = 0; q < 6; ++q) s_m[q][threadIdx.x] = m[q];
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            _Pragma("unroll") for (int q = 0; q < 6; ++q) s_m[q][threadIdx.x] = nmax(s_m[q][threadIdx.x], s_m[q][threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x < 6) red6[threadIdx.x] = s_m[threadIdx.x][0];
    if (threadIdx.x == 6) red6[6] = (ctl->flags & 1) ? 1.0 : 0.0;  // NaN-in-box flag, all-reduced too
    if (threadIdx.x == 7) red6[7] = 0.0;
    // a NaN maximum is flagged in slots 8..13 (RCCL's max need not propagate NaN); slot 15
    // marks the record valid (cp_init zeroes it: iteration 0 has no previous record)
    if (threadIdx.x >= 8 && threadIdx.x < 16)
        red6[threadIdx.x] = threadIdx.x == 15 ? 1.0
                            : (threadIdx.x < 14 && s_m[threadIdx.x - 8][0] != s_m[threadIdx.x - 8][0]) ? 1.0 : 0.0;
}
// history + stopping test of the previous iteration from the R records gathered with X1
// (max over the shards; the same decision on every shard)
__global__ void k_cp_check_gather(Ctl* ctl, double* hist, const double* __restrict__ recv, int R, int maxc) {
    if (threadIdx.x != 0 || ctl->done) return;
    const int stride = 2 * maxc + 16;
    const double* r0 = recv + 2 * maxc;
    if (r0[15] == 0.0) return;  // no previous iteration yet
    double M[16];
    for (int q = 0; q < 16; ++q) M[q] = r0[q];
    for (int r = 1; r < R; ++r)
        for (int q = 0; q < 16; ++q) M[q] = nmax(M[q], recv[(size_t)r * stride + 2 * maxc + q]);
    const int k = ctl->k;
    for (int q = 0; q < 6; ++q) {
        if (M[8 + q] > 0.0) M[q] = __builtin_nan("");
        hist[(size_t)k * 6 + q] = M[q];
    }
    const double err = nmax(nmax(M[0], M[1]), M[2]);
    if (M[6] > 0.0) ctl->flags |= 1;
    if (k >= ctl->max_iters || err <= ctl->tol || (ctl->flags & 1)) {
        ctl->done = 1;
        ctl->final_k = k;
    } else {
        ctl->k = k + 1;
    }
}

// history + stopping test on the all-reduced maxima (same decision on every shard)
__global__ void k_cp_check_red(Ctl* ctl, double* hist, const double* __restrict__ red6) {
    if (threadIdx.x != 0 || ctl->done) return;
    const int k = ctl->k;
    double M[6];
    for (int q = 0; q < 6; ++q) {
        M[q] = red6[8 + q] > 0.0 ? __builtin_nan("") : red6[q];
        hist[(size_t)k * 6 + q] = M[q];
    }
    const double err = nmax(nmax(M[0], M[1]), M[2]);  // NaN: not converged
    if (red6[6] > 0.0) ctl->flags |= 1;
    if (k >= ctl->max_iters || err <= ctl->tol || (ctl->flags & 1)) {
        ctl->done = 1;
        ctl->final_k = k;
    } else {
        ctl->k = k + 1;
    }
}

// ---- vector helpers for Lanczos (step size); T = the context's scalar type, dot
// products accumulate in fp64
template <class T>
__global__ void k_dot_partial(const T* __restrict__ a, const T* __restrict__ b, int n, double* part) {
    __shared__ double s[kBlock / 64];
    double acc = 0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        acc = fma((double)a[i], (double)b[i], acc);
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += s[w];
        part[blockIdx.x] = t;
    }
}

__global__ void k_dot_final(const double* part, int nb, double* out) {
    __shared__ double s[kBlock];
    double acc = 0.0;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) acc += part[i];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = s[0];
}

// y = a*x + b*y
template <class T>
__global__ void k_axpby(double a, const T* __restrict__ x, double b, T* __restrict__ y, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        y[i] = (T)(a * (double)x[i] + b * (double)y[i]);
}

template <class T>
__global__ void k_scale_copy(double s, const T* __restrict__ x, T* __restrict__ y, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) y[i] = (T)(s * (double)x[i]);
}

// fp64 <-> fp32 copies (the host boundary of an fp32 context)
__global__ void k_to_f32(const double* __restrict__ x, float* __restrict__ y, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) y[i] = (float)x[i];
}
__global__ void k_to_f64(const float* __restrict__ x, double* __restrict__ y, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) y[i] = (double)x[i];
}

}  // namespace raocp
