// raocp_mega.hip — the persistent Chambolle–Pock engine: ONE launch runs a whole solve
// (Solver.chock, solver.py:97-171). Included by raocp_kernels.hip (namespace raocp).
//
// Ownership. The tree is cut at stage s. Workgroup 0 owns the TOP (stages 0 .. s-1): the
// primal rows of those nodes, the child-indexed rows (tau_j, s_j, eta3..6_j) of their
// children INCLUDING the roots of the subtrees (stage s), and the top nodes' own duals
// (eta1, eta2, eta7). Workgroup 1 + k owns the subtree rooted at the k-th node r of stage s:
// every other row of its nodes (x_r, u_r, y_r, eta1_r, eta2_r, eta7_r, and everything
// below). This is the family split of raocp_cp.hip: a family (parents + children) never
// straddles two owners except at the (P, r) edges, which couple through exactly:
//   UP[it]   (subtree k -> top, after its backward sweep): q_r of the dynamics recursion;
//            eta2_r of the previous iteration's eta+, d and xi2 (the top's s_r rows of L^T);
//            the subtree's residual maxima of the previous iteration and its NaN flag.
//   DOWN[it] (top -> every subtree, after the top's forward sweep): x_r of the projected
//            iterate and s_r (the top's kernel projection at P writes it), plus `stop`.
// Everything else a workgroup reads it wrote itself (same CU: plain loads after a barrier).
//
// One iteration `it` (buffers rotate as in raocp_capi.hip: p = Z[it%3], z+ = Z[(it+1)%3]
// (arrives as the half step), next half step Z[(it+2)%3], d = E[it%2], eta+ = E[(it+1)%2]):
//   subtree: backward sweep -> UP -> wait DOWN -> forward sweep -> dual (L, prox g*, xi2)
//            -> next primal half step + AVaR kernel projection + residual terms of `it`
//   top:     wait UP -> [deferred: its stage s-1 families' y / tau_r / s_r rows and kernel
//            projection of it-1, residual maxima of it-1 -> history row, stopping test]
//            -> backward + forward sweep of the top -> DOWN -> dual -> primal half step
// The stopping test of iteration k is taken at the start of iteration k+1 (whose first
// half only writes the NEXT half-step buffer), so the returned iterate is the reference's.
//
// Hand-offs (MI355X: per-XCD L2s are not coherent): every payload word is stored `sc1`
// (agent-scope relaxed atomic store), every storing wave drains (s_waitcnt vmcnt(0)), a
// workgroup barrier, then ONE lane stores the flag; the consumer polls the flag with `sc1`
// loads, then reads the payload with `sc1` loads only. Every spin is bounded
// (MegaArg::timeout, 100 MHz ticks): a timed-out workgroup sets ctl->flags bit 1 and
// leaves, so the others time out too and the launch drains.

constexpr int kMegaThreads = 512;   // full engine (dual / primal phases: 256 VGPRs per lane)
constexpr int kMegaDynThreads = 1024;  // dynamics-only engine
constexpr int kMegaLev = 16;  // levels per workgroup (the host plans within it)

struct MegaArg {
    double* Z[3];
    double* E[2];
    double* xi2;
    double* up;           // [nsub][ups] UP payloads
    unsigned* up_flag;    // [nsub]
    double* dn;           // [nsub][dns] DOWN payloads
    unsigned* dn_flag;    // [1]
    const Rec* lv;        // [nwg][kMegaLev + 1] level ranges {lo, hi, off, 0}
    const int* wl;        // [nwg] levels: top s (level s = the roots, not owned); subtree N - s
    const double* x0;
    double* hist;
    Ctl* ctl;
    double alpha, tol;
    int s, nsub, ups, dns, max_iters;
    int c_top1, c_sub0, c_sub1;  // class ranges: top [0, c_top1), subtrees [c_sub0, c_sub1)
    int maxch;                   // widest child level (P rows)
    int stage_cap;               // doubles of the LDS stage (aliases the dynamics rows)
    long long timeout;           // per wait, 100 MHz ticks
    unsigned long long* stamps;  // diagnostics: [nwg][64] (nullptr = off)
    unsigned* epoch;             // dynamics-only engine: launches so far (flag tags grow across launches)
};

typedef __attribute__((address_space(1))) unsigned int glbd32;

__device__ __forceinline__ unsigned ld_flag(const unsigned* f) {
    return __hip_atomic_load((gu32*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(unsigned* f, unsigned v) {
    __hip_atomic_store((gu32*)f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every storing wave: drain its sc1 stores, then the barrier, then one lane signals
__device__ __forceinline__ void mega_publish(unsigned* flag, unsigned v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) st_flag(flag, v);
}

// LDS layout of a workgroup (doubles); the host mirrors it (raocp_capi.hip, mega_plan).
// [W | RG | KM | sqrtQ, sqrtR, sqrtPf | area | NL | CH | SX | E2]: the area holds the
// dynamics rows (XQ, U, DR, P) during the sweeps and the phase stage during dual / primal.
struct MegaLds {
    int oW, oRG, oKM, oMAT, oXQ, oU, oDR, oP, oNL, oCH, oSX, oE2, total;
    __host__ __device__ MegaLds(int nkind, int ncls, int nall, int nnl, int maxch, int nb, int nx, int nu, int nmat,
                                int stage_cap, int nthreads = kMegaThreads) {
        const int KP = rup(nx, 2 * kKS), NUP = rup(nu, 2), PS = NUP + rup(nx, 2);
        const int SKP = tstride(KP), SNU = tstride(NUP), R = nx + nu;
        oW = 0;
        oRG = oW + nkind * R * SKP;
        oKM = oRG + ncls * R * SNU;
        oMAT = oKM + ncls * nu * SKP;
        oXQ = oMAT + rup(nmat, 2);
        oU = oXQ + nall * KP;
        oDR = oU + nnl * NUP;
        oP = oDR + nnl * NUP;
        const int dyn = oP + rup(maxch * PS, 2) - oXQ;
        oNL = oXQ + (dyn > stage_cap ? dyn : stage_cap);
        oCH = oNL + 2 * nnl;
        oSX = oCH + 2 * nall;
        oE2 = oSX + nthreads;
        total = oE2 + 4 * nb;
    }
};

// groups of G lanes over the nodes of levels [la, lb) (flattened); body(node or -1, level, r, base)
// is called by every lane the same number of times (it may hold workgroup barriers)
template <class F>
__device__ __forceinline__ void mega_groups(const int* lo, const int* hi, int la, int lb, int G, F body) {
    int tot = 0;
    for (int l = la; l < lb; ++l) tot += hi[l] - lo[l];
    const int per = blockDim.x / G, gl = threadIdx.x / G, r = threadIdx.x - gl * G;
    for (int v0 = 0; v0 < tot; v0 += per) {
        const int v = v0 + gl;
        int node = -1, lvl = la;
        if (gl < per && v < tot) {
            int rem = v;
            for (int l = la; l < lb; ++l) {
                const int c = hi[l] - lo[l];
                if (rem < c) {
                    node = lo[l] + rem;
                    lvl = l;
                    break;
                }
                rem -= c;
            }
        }
        body(node, lvl, r, gl * G);
    }
}

__device__ __forceinline__ double wave_max(double v) {
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
    return v;
}

// forward step 1: u_i = K_i x_i + d_i (nodes [b, e) of one level; x_i in XQ rows, d_i in DR rows)
template <int KS, int NXc, int NUc, class INF>
__device__ __forceinline__ void mega_fwd_u(const Dev& p, const ldsd* KM, int cbase, const INF& inf, int b, int e,
                                           const LRows& xq, const LRows& dr, const LRows& ur, glbd* z) {
    const Geo<NXc, NUc> g(p);
    constexpr int cKC = Geo<NXc, NUc>::cKP / KS;
    const int KC = g.KP / KS;
    const int items = (e - b) * g.nu * KS;
    for (int vi = threadIdx.x; vi - (int)threadIdx.x < items; vi += blockDim.x) {
        const bool live = vi < items;
        const int grp = live ? vi / KS : 0, sl = vi - grp * KS;
        const int i = b + grp / g.nu, r = grp - (grp / g.nu) * g.nu;
        double acc = 0.0;
        if (live) {
            const Rec ni = inf.nonleaf(i);
            const ldsd* km = KM + ((size_t)(ni.z - cbase) * g.nu + r) * g.SKP + sl * KC;
            acc = dot_slice<cKC>(km, xq(i) + sl * KC, KC);
        }
        acc = ks_reduce<KS>(acc);
        if (live && sl == 0) {
            const double u = acc + dr(i)[r];
            z[p.U0 + (size_t)i * g.nu + r] = u;
            ur(i)[r] = u;
        }
    }
}

// forward step 2: x_j = A_j x_i + B_j u_i for children [cb, ce) (parent rows xq(i), ur(i)),
// W = [B'; A'] rows of the child's kind: A[r][k] = W[nu + k][r], B[r][k] = W[k][r].
// The child's row goes to xq(j) and, when ZOUT, to z.
template <int KS, int NXc, int NUc, class INF>
__device__ __forceinline__ void mega_fwd_x(const Dev& p, const ldsd* W, const INF& inf, int cb, int ce,
                                           const LRows& xq_p, const LRows& ur, const LRows& xq_c, glbd* z, bool zout) {
    const Geo<NXc, NUc> g(p);
    const int R = g.R;
    const int KC = (R + KS - 1) / KS;
    const int items = (ce - cb) * g.nx * KS;
    for (int vi = threadIdx.x; vi - (int)threadIdx.x < items; vi += blockDim.x) {
        const bool live = vi < items;
        const int grp = live ? vi / KS : 0, sl = vi - grp * KS;
        const int j = cb + grp / g.nx, r = grp - (grp / g.nx) * g.nx;
        double acc = 0.0;
        if (live) {
            const Rec cj = inf.child(j);
            const ldsd* wk = W + (size_t)cj.x * R * g.SKP + r;  // column r of the kind's rows
            const ldsd* xi = xq_p(cj.z);
            const ldsd* ui = ur(cj.z);
            const int k0 = sl * KC, k1 = min(R, k0 + KC);
            double s0 = 0.0, s1 = 0.0;
            int k = k0;
            for (; k + 1 < k1; k += 2) {
                const double v0 = k < g.nx ? xi[k] : ui[k - g.nx];
                const double v1 = k + 1 < g.nx ? xi[k + 1] : ui[k + 1 - g.nx];
                const int w0 = k < g.nx ? g.nu + k : k - g.nx, w1 = k + 1 < g.nx ? g.nu + k + 1 : k + 1 - g.nx;
                s0 = fma(wk[(size_t)w0 * g.SKP], v0, s0);
                s1 = fma(wk[(size_t)w1 * g.SKP], v1, s1);
            }
            if (k < k1) {
                const double v0 = k < g.nx ? xi[k] : ui[k - g.nx];
                const int w0 = k < g.nx ? g.nu + k : k - g.nx;
                s0 = fma(wk[(size_t)w0 * g.SKP], v0, s0);
            }
            acc = s0 + s1;
        }
        acc = ks_reduce<KS>(acc);
        if (live && sl == 0) {
            xq_c(j)[r] = acc;
            if (zout) z[p.X0 + (size_t)j * g.nx + r] = acc;
        }
    }
}

template <int NXc, int NUc, class INF>
__device__ __forceinline__ void mega_fwd_level(const Dev& p, const ldsd* W, const ldsd* KM, int cbase,
                                               const INF& inf, int b, int e, int cb, int ce, const LRows& xq_p,
                                               const LRows& dr, const LRows& ur, const LRows& xq_c, glbd* z,
                                               bool zout) {
    const int nx = NXc ? NXc : p.nx, nu = NUc ? NUc : p.nu;
    const int nthr = blockDim.x;
    const int iu = (e - b) * nu;
    if (iu * 4 <= nthr) mega_fwd_u<4, NXc, NUc>(p, KM, cbase, inf, b, e, xq_p, dr, ur, z);
    else if (iu * 2 <= nthr) mega_fwd_u<2, NXc, NUc>(p, KM, cbase, inf, b, e, xq_p, dr, ur, z);
    else mega_fwd_u<1, NXc, NUc>(p, KM, cbase, inf, b, e, xq_p, dr, ur, z);
    lds_sync();
    const int ix = (ce - cb) * nx;
    if (ix * 4 <= nthr) mega_fwd_x<4, NXc, NUc>(p, W, inf, cb, ce, xq_p, ur, xq_c, z, zout);
    else if (ix * 2 <= nthr) mega_fwd_x<2, NXc, NUc>(p, W, inf, cb, ce, xq_p, ur, xq_c, z, zout);
    else mega_fwd_x<1, NXc, NUc>(p, W, inf, cb, ce, xq_p, ur, xq_c, z, zout);
    lds_sync();
}

// DYN: the dynamics projection only (cache.py:259-288) of the half step a.Z[1], one launch per
// projection inside the captured CP iteration: the backward / forward sweeps and the two
// hand-offs, no dual / primal phases; tags continue from *a.epoch.
template <int NXc, int NUc, bool DYN>
__global__ void __launch_bounds__(DYN ? kMegaDynThreads : kMegaThreads) k_mega(Dev p, MegaArg a, const Ctl* dctl) {
    constexpr int NT = DYN ? kMegaDynThreads : kMegaThreads;
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ int s_lo[kMegaLev + 1], s_hi[kMegaLev + 1], s_off[kMegaLev + 1];
    __shared__ int s_L, s_ok, s_stop;
    __shared__ double s_red[NT / 64][8];
    __shared__ double s_sr[2];  // subtree: s_r of z+ and of p
    __shared__ int s_sg[kMegaLev + 1][8];  // LDS offsets of the staged operands, per level
    const int wg = blockIdx.x, tid = threadIdx.x, nthr = blockDim.x;
    const bool top = wg == 0;
    const int sub = wg - 1;
    const Geo<NXc, NUc> g(p);
    const TabSize<NXc, NUc> ts(g);
    const int nx = g.nx, nu = g.nu;
    const double alpha = a.alpha;
    unsigned long long* stp = a.stamps ? a.stamps + (size_t)wg * 64 : nullptr;
    int nst = 0;
    auto stamp_ = [&]() {
        if (stp && tid == 0 && nst < 64) stp[nst] = __builtin_amdgcn_s_memrealtime();
        ++nst;
    };
    stamp_();
    // the dynamics-only engine inside a captured batch: iterations past the stopping test
    // do nothing (every workgroup reads the same word, so none waits on another)
    if (DYN && dctl && dctl->done) return;
    const unsigned ep = DYN ? *(const glbd32*)a.epoch : 0u;
    if (tid <= kMegaLev) {
        const Rec r = a.lv[(size_t)wg * (kMegaLev + 1) + tid];
        s_lo[tid] = r.x;
        s_hi[tid] = r.y;
        s_off[tid] = r.z;
    }
    if (tid == 0) {
        s_L = a.wl[wg];
        s_ok = 1;
        s_stop = 0;
        s_sr[0] = s_sr[1] = 0.0;
    }
    __syncthreads();
    const int L = s_L;
    const int nall = s_off[L] + (s_hi[L] - s_lo[L]), nnl = s_off[L];
    const int c0 = top ? 0 : a.c_sub0, c1 = top ? a.c_top1 : a.c_sub1;
    const int nQ = p.nSQ * nx * nx, nR = p.nSR * nu * nu, nP = p.nSP * nx * nx;
    const MegaLds ml(p.nkind, c1 - c0, nall, nnl, a.maxch, top ? a.nsub : 0, nx, nu, DYN ? 0 : nQ + nR + nP,
                     DYN ? 0 : a.stage_cap, NT);
    ldsd* sm = (ldsd*)smem_;
    ldsd* W = sm + ml.oW;
    ldsd* RG = sm + ml.oRG;
    ldsd* KM = sm + ml.oKM;
    ldsd* XQ = sm + ml.oXQ;
    ldsd* U = sm + ml.oU;
    ldsd* DR = sm + ml.oDR;
    ldsd* PB = sm + ml.oP;
    ldsd* NLd = sm + ml.oNL;
    ldsd* CHd = sm + ml.oCH;
    double* SX = (double*)(sm + ml.oSX);  // group-reduction scratch (generic: kernel_proj_group)
    ldsd* E2T = sm + ml.oE2;              // top: per root {eta+, d, xi2} of eta2_r
    ldsd* STG = sm + ml.oXQ;              // phase stage (aliases the dynamics rows)
    const ldsd* SQl = sm + ml.oMAT;       // L weights, column-major (M[k n + r])
    const ldsd* SRl = SQl + nQ;
    const ldsd* SPl = SRl + nR;
    // stage `count` doubles from src at the next free offset; returns where the data starts
    auto stage = [&](int& off, int& rot, const glbd* src, int count) {
        const int sh = dma_any(STG + off, src, count * 8, &rot);
        const int at = off + sh;
        off += rup(count, 2) + 4;
        return at;
    };
    auto stage_rec = [&](int& off, int& rot, const Rec* src, int count) {
        dma_any(STG + off, (const glbd*)src, count * 16, &rot);
        const int at = off;
        off += 2 * count + 4;
        return at;
    };
    // ---- tables, once: W (all kinds), RG / KM (the workgroup's classes), node records
    {
        const int nW = p.nkind * ts.W1, nRG = (c1 - c0) * ts.RG1, nKM = (c1 - c0) * ts.KM1;
        const glbd* gW = (const glbd*)p.dW;
        const glbd* gRG = (const glbd*)p.dRG + (size_t)c0 * ts.RG1;
        const glbd* gKM = (const glbd*)p.dKM + (size_t)c0 * ts.KM1;
        for (int e = tid; e < nW; e += nthr) W[e] = gW[e];
        for (int e = tid; e < nRG; e += nthr) RG[e] = gRG[e];
        for (int e = tid; e < nKM; e += nthr) KM[e] = gKM[e];
        if (!DYN) {
            ldsd* MAT = sm + ml.oMAT;
            for (int e = tid; e < nQ; e += nthr) MAT[e] = ((const glbd*)p.SQ)[e];
            for (int e = tid; e < nR; e += nthr) MAT[nQ + e] = ((const glbd*)p.SR)[e];
            for (int e = tid; e < nP; e += nthr) MAT[nQ + nR + e] = ((const glbd*)p.SP)[e];
        }
        ldsrec* NL = (ldsrec*)NLd;
        ldsrec* CH = (ldsrec*)CHd;
        for (int l = 0; l <= L; ++l) {
            const int lo = s_lo[l], cnt = s_hi[l] - s_lo[l], off = s_off[l];
            for (int q = tid; q < cnt; q += nthr) {
                if (l < L) NL[off + q] = ((const glbrec*)p.ninfo)[lo + q];
                CH[off + q] = ((const glbrec*)p.cinfo)[lo + q];
            }
        }
        for (int e = tid; e < nall * g.KP; e += nthr) XQ[e] = 0.0;
        for (int e = tid; e < nnl * g.NUP; e += nthr) {
            U[e] = 0.0;
            DR[e] = 0.0;
        }
    }
    __syncthreads();
    const ldsrec* NL = (const ldsrec*)NLd;
    const ldsrec* CH = (const ldsrec*)CHd;
    const TabsT<const ldsd*, const ldsd*> tb{W, RG, KM, nullptr, c0, 0};
    auto inf = [&](int l) {
        return InfoT<const ldsrec*>{NL + s_off[l], s_lo[l], CH + s_off[l + 1], s_lo[l + 1]};
    };
    auto rows = [&](ldsd* base, int l, int w) { return LRows{base + (size_t)s_off[l] * w, s_lo[l], w}; };
    const int root = top ? 0 : s_lo[0];
    const int rb = top ? s_lo[L] : 0;  // first root id (top: the boundary level)

    double m0 = 0, m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0;  // this lane's residual maxima (iteration in flight)
    int nan_local = 0;
    const double* x0 = a.x0;
    stamp_();

    for (int it = 0;; ++it) {
        const glbd* Zp = (const glbd*)a.Z[it % 3];
        glbd* Zc = (glbd*)a.Z[(it + 1) % 3];
        glbd* Zn = (glbd*)a.Z[(it + 2) % 3];
        glbd* Ed = (glbd*)a.E[it % 2];
        glbd* Ee = (glbd*)a.E[(it + 1) % 2];
        glbd* X2 = (glbd*)a.xi2;
        const unsigned tag = ep + (unsigned)(it + 1);

        // ================= backward sweep: x, u rows of the half step -> q, d ==================
        if (top) {
            // wait for every subtree's UP[it]
            if (tid < 64) {
                const long long t0 = __builtin_amdgcn_s_memrealtime();
                bool ok = true;
                for (;;) {
                    bool mine = true;
                    for (int k = tid; k < a.nsub; k += 64) mine = mine && ld_flag(a.up_flag + k) >= tag;
                    if (__all(mine)) break;
                    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (tid == 0 && !ok) s_ok = 0;
            }
            __syncthreads();
            if (!s_ok) break;
            stamp_();
            // boundary rows: q_r from UP; eta2_r triples; the subtrees' maxima
            for (int e = tid; e < a.nsub * g.KP; e += nthr) {
                const int k = e / g.KP, c = e - k * g.KP;
                XQ[(size_t)(s_off[L] + k) * g.KP + c] = c < nx ? ld_sc1(a.up + (size_t)k * a.ups + c) : 0.0;
            }
            for (int e = tid; e < a.nsub * 3; e += nthr) {
                const int k = e / 3, c = e - k * 3;
                E2T[4 * k + c] = ld_sc1(a.up + (size_t)k * a.ups + g.KP + c);
            }
            if (it > 0) {
                for (int k = tid; k < a.nsub; k += nthr) {
                    const double* rec = a.up + (size_t)k * a.ups + g.KP + 3;
                    m0 = fmax(m0, ld_sc1(rec + 0)); m1 = fmax(m1, ld_sc1(rec + 1)); m2 = fmax(m2, ld_sc1(rec + 2));
                    m3 = fmax(m3, ld_sc1(rec + 3)); m4 = fmax(m4, ld_sc1(rec + 4)); m5 = fmax(m5, ld_sc1(rec + 5));
                    if (ld_sc1(rec + 6) != 0.0) nan_local = 1;
                }
            }
            __syncthreads();
            // deferred rows of iteration it-1: y_P, tau_r, s_r of the stage s-1 families (their
            // L^T needs the subtrees' eta2_r) and the kernel projection at P
            if (it > 0) {
                const glbd* pP = (const glbd*)a.Z[(it + 2) % 3];  // p of it-1
                const glbd* pZ = (const glbd*)a.Z[it % 3];        // z+ of it-1
                glbd* pO = (glbd*)a.Z[(it + 1) % 3];              // its next half step (this z+)
                const glbd* dA = (const glbd*)a.E[it % 2];        // eta+ of it-1
                const glbd* dP = (const glbd*)a.E[(it + 1) % 2];  // d of it-1
                const int G = nx + nu + p.cmax + 1;
                mega_groups(s_lo, s_hi, L - 1, L, G, [&](int i, int, int r, int base) {
                    const bool live = i >= 0;
                    const int rk = r - (nx + nu);
                    int c = 0, cs = 0, yo = 0;
                    if (live) {
                        const Rec fr = ((const glbrec*)p.frec)[i];  // {yrel, nch, ch_start, e7off}
                        yo = fr.x;
                        c = fr.y;
                        cs = fr.z;
                    }
                    auto account = [&](int e, double w, double cc) {
                        const double pp = pP[e], zz = pZ[e];
                        const double x1 = (pp - zz) / alpha - w, x0v = x1 + cc, dl1 = zz - pp, dl0 = dl1 + w;
                        m0 = fmax(m0, fabs(x0v)); m1 = fmax(m1, fabs(x1));
                        m3 = fmax(m3, fabs(dl0)); m4 = fmax(m4, fabs(dl1));
                    };
                    double vals[4] = {0, 0, 0, 0};
                    double y2c = 0.0;
                    const double e2A = live ? dA[p.E2 + i] : 0.0;
                    const double e2W = live ? dP[p.E2 + i] - dA[p.E2 + i] : 0.0;
                    const double e2C = live ? X2[p.E2 + i] : 0.0;
                    if (live && rk >= 0 && rk < c) {
                        const int j = cs + rk;
                        const double b = p.cond[j];
                        const int ey0 = p.Y0 + yo + rk, ey1 = p.Y0 + yo + c + rk;
                        const int f0 = p.E1 + yo + rk, f1 = p.E1 + yo + c + rk;
                        vals[0] = pZ[ey0] - alpha * (dA[f0] - b * e2A);
                        vals[1] = pZ[ey1] - alpha * (dA[f1] - 0.0 * e2A);
                        vals[2] = pZ[p.T0 + j] - alpha * (0.5 * (dA[p.E5 + j] + dA[p.E6 + j]));
                        const ldsd* t3 = E2T + 4 * (j - rb);  // {eta+, d, xi2} at eta2_j
                        vals[3] = pZ[p.S0 + j] - alpha * t3[0];
                        account(ey0, (dP[f0] - dA[f0]) - b * e2W, X2[f0] - b * e2C);
                        account(ey1, (dP[f1] - dA[f1]) - 0.0 * e2W, X2[f1] - 0.0 * e2C);
                        account(p.T0 + j, 0.5 * ((dP[p.E5 + j] - dA[p.E5 + j]) + (dP[p.E6 + j] - dA[p.E6 + j])),
                                0.5 * (X2[p.E5 + j] + X2[p.E6 + j]));
                        account(p.S0 + j, t3[1] - t3[0], t3[2]);
                    }
                    if (live && rk == p.cmax) {
                        const int f2 = p.E1 + yo + 2 * c, ey2 = p.Y0 + yo + 2 * c;
                        y2c = pZ[ey2] - alpha * (dA[f2] - 1.0 * e2A);
                        account(ey2, (dP[f2] - dA[f2]) - 1.0 * e2W, X2[f2] - 1.0 * e2C);
                        if (i == 0) {
                            pO[p.S0] = (pZ[p.S0] - alpha * e2A) - alpha;
                            account(p.S0, e2W, e2C);
                        }
                    }
                    kernel_proj_group(p, live ? i : 0, c, cs, rk, live && rk >= 0, base + nx + nu, SX, vals, y2c);
                    if (live && rk >= 0 && rk < c) {
                        const int j = cs + rk;
                        pO[p.Y0 + yo + rk] = vals[0];
                        pO[p.Y0 + yo + c + rk] = vals[1];
                        pO[p.T0 + j] = vals[2];
                        pO[p.S0 + j] = vals[3];
                    }
                    if (live && rk == p.cmax) pO[p.Y0 + yo + 2 * c] = y2c;
                    __syncthreads();
                });
                // residual maxima of it-1 -> history row, stopping test (ctl, k_cp_check)
                const int wv = tid >> 6;
                {
                    const double mv[6] = {wave_max(m0), wave_max(m1), wave_max(m2), wave_max(m3), wave_max(m4),
                                          wave_max(m5)};
                    if ((tid & 63) == 0) _Pragma("unroll") for (int q = 0; q < 6; ++q) s_red[wv][q] = mv[q];
                }
                const int nanw = __any(nan_local);
                if ((tid & 63) == 0) s_red[wv][6] = nanw ? 1.0 : 0.0;
                __syncthreads();
                if (tid == 0) {
                    double mm[7] = {0, 0, 0, 0, 0, 0, 0};
                    for (int w2 = 0; w2 < nthr / 64; ++w2)
                        for (int q = 0; q < 7; ++q) mm[q] = fmax(mm[q], s_red[w2][q]);
                    const int k = it - 1;
                    for (int q = 0; q < 6; ++q) a.hist[(size_t)k * 6 + q] = mm[q];
                    const double err = fmax(fmax(mm[0], mm[1]), mm[2]);
                    const bool nanf = mm[6] != 0.0;
                    if (k >= a.max_iters || err <= a.tol || nanf) {
                        s_stop = 1;
                        a.ctl->done = 1;
                        a.ctl->final_k = k;
                        a.ctl->k = k;
                        if (nanf) atomicOr(&a.ctl->flags, 1);
                    }
                }
                m0 = m1 = m2 = m3 = m4 = m5 = 0.0;
                nan_local = 0;
                __syncthreads();
                if (s_stop) {
                    mega_publish(a.dn_flag, 2u * tag + 1u);
                    break;
                }
            }
            stamp_();
            // top x, u rows of the half step
            for (int l = 0; l < L; ++l) {
                const int lo = s_lo[l], cnt = s_hi[l] - lo, off = s_off[l];
                for (int e = tid; e < cnt * g.KP; e += nthr) {
                    const int q = e / g.KP, c = e - q * g.KP;
                    XQ[(size_t)(off + q) * g.KP + c] = c < nx ? (double)Zc[p.X0 + (size_t)(lo + q) * nx + c] : 0.0;
                }
                for (int e = tid; e < cnt * g.NUP; e += nthr) {
                    const int q = e / g.NUP, c = e - q * g.NUP;
                    U[(size_t)(off + q) * g.NUP + c] = c < nu ? (double)Zc[p.U0 + (size_t)(lo + q) * nu + c] : 0.0;
                }
            }
            lds_sync();
            for (int l = L - 1; l >= 0; --l) {
                const auto nf = inf(l);
                const LRows pr{PB, s_lo[l + 1], g.PS};
                back_phase_a<NXc, NUc>(p, tb, nf, s_lo[l + 1], s_hi[l + 1], rows(XQ, l + 1, g.KP), 1.0, pr, tid, nthr);
                lds_sync();
                back_phase_b<NXc, NUc>(p, tb, nf, s_lo[l], s_hi[l], pr, rows(XQ, l, g.KP), rows(U, l, g.NUP),
                                       rows(XQ, l, g.KP), rows(DR, l, g.NUP), tid, nthr);
                lds_sync();
            }
            stamp_();
            // forward: x_0 = x0bar, then u_i, x_j level by level; the roots' x go to DOWN
            if (tid < nx) {
                const double v = ((const glbd*)x0)[tid];
                XQ[tid] = v;
                Zc[p.X0 + tid] = v;
            }
            lds_sync();
            for (int l = 0; l < L; ++l)
                mega_fwd_level<NXc, NUc>(p, W, KM, c0, inf(l), s_lo[l], s_hi[l], s_lo[l + 1], s_hi[l + 1],
                                         rows(XQ, l, g.KP), rows(DR, l, g.NUP), rows(U, l, g.NUP),
                                         rows(XQ, l + 1, g.KP), Zc, l + 1 < L);
            stamp_();
            // DOWN[it]: x_r and s_r of z+ for every root
            for (int e = tid; e < a.nsub * (nx + 1); e += nthr) {
                const int k = e / (nx + 1), c = e - k * (nx + 1);
                const double v = c < nx ? (double)XQ[(size_t)(s_off[L] + k) * g.KP + c] : (double)Zc[p.S0 + rb + k];
                st_sc1(a.dn + (size_t)k * a.dns + c, v);
            }
            mega_publish(a.dn_flag, 2u * tag);
            stamp_();
            if (DYN) {
                // every subtree has read the epoch (its UP arrived): the next launch's tags follow
                if (tid == 0) *(glbd32*)a.epoch = ep + 1u;
                break;
            }
        } else {
            // subtree: x, u rows of the half step (leaves too: their q = -x)
            for (int l = 0; l <= L; ++l) {
                const int lo = s_lo[l], cnt = s_hi[l] - lo, off = s_off[l];
                for (int e = tid; e < cnt * g.KP; e += nthr) {
                    const int q = e / g.KP, c = e - q * g.KP;
                    XQ[(size_t)(off + q) * g.KP + c] = c < nx ? (double)Zc[p.X0 + (size_t)(lo + q) * nx + c] : 0.0;
                }
                if (l < L)
                    for (int e = tid; e < cnt * g.NUP; e += nthr) {
                        const int q = e / g.NUP, c = e - q * g.NUP;
                        U[(size_t)(off + q) * g.NUP + c] = c < nu ? (double)Zc[p.U0 + (size_t)(lo + q) * nu + c] : 0.0;
                    }
            }
            lds_sync();
            for (int l = L - 1; l >= 0; --l) {
                const auto nf = inf(l);
                const LRows pr{PB, s_lo[l + 1], g.PS};
                back_phase_a<NXc, NUc>(p, tb, nf, s_lo[l + 1], s_hi[l + 1], rows(XQ, l + 1, g.KP),
                                       l + 1 == L ? -1.0 : 1.0, pr, tid, nthr);
                lds_sync();
                back_phase_b<NXc, NUc>(p, tb, nf, s_lo[l], s_hi[l], pr, rows(XQ, l, g.KP), rows(U, l, g.NUP),
                                       rows(XQ, l, g.KP), rows(DR, l, g.NUP), tid, nthr);
                lds_sync();
            }
            stamp_();
            // UP[it]: q_r | eta2_r of (eta+, d, xi2) of it-1 | maxima of it-1 | NaN flag
            {
                double* rec = a.up + (size_t)sub * a.ups;
                if (tid < nx) st_sc1(rec + tid, XQ[tid]);
                if (it > 0 && tid == 64) {
                    st_sc1(rec + g.KP + 0, a.E[it % 2][p.E2 + root]);
                    st_sc1(rec + g.KP + 1, a.E[(it + 1) % 2][p.E2 + root]);
                    st_sc1(rec + g.KP + 2, a.xi2[p.E2 + root]);
                }
                if (it > 0) {
                    const int wv = tid >> 6;
                    {
                        const double mv[6] = {wave_max(m0), wave_max(m1), wave_max(m2), wave_max(m3), wave_max(m4),
                                              wave_max(m5)};
                        if ((tid & 63) == 0) _Pragma("unroll") for (int q = 0; q < 6; ++q) s_red[wv][q] = mv[q];
                    }
                    const int nanw = __any(nan_local);
                    if ((tid & 63) == 0) s_red[wv][6] = nanw ? 1.0 : 0.0;
                    __syncthreads();
                    if (tid < 7) {
                        double v = 0.0;
                        for (int w2 = 0; w2 < nthr / 64; ++w2) v = fmax(v, s_red[w2][tid]);
                        st_sc1(rec + g.KP + 3 + tid, v);
                    }
                    m0 = m1 = m2 = m3 = m4 = m5 = 0.0;
                    nan_local = 0;
                }
                mega_publish(a.up_flag + sub, tag);
            }
            stamp_();
            // wait for DOWN[it]
            if (tid == 0) {
                const long long t0 = __builtin_amdgcn_s_memrealtime();
                unsigned f;
                for (;;) {
                    f = ld_flag(a.dn_flag);
                    if (f >= 2u * tag) break;
                    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
                        s_ok = 0;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (s_ok && (f & 1u)) s_stop = 1;
            }
            __syncthreads();
            if (!s_ok || s_stop) break;
            stamp_();
            const double* drec = a.dn + (size_t)sub * a.dns;
            if (tid < nx) {
                const double v = ld_sc1(drec + tid);
                XQ[tid] = v;
                Zc[p.X0 + (size_t)root * nx + tid] = v;
            }
            if (!DYN && tid == 64) {  // s_r of z+ and p (the dual's eta2_r row)
                s_sr[1] = it == 0 ? (double)Zp[p.S0 + root] : s_sr[0];
                s_sr[0] = ld_sc1(drec + nx);
            }
            lds_sync();
            for (int l = 0; l < L; ++l)
                mega_fwd_level<NXc, NUc>(p, W, KM, c0, inf(l), s_lo[l], s_hi[l], s_lo[l + 1], s_hi[l + 1],
                                         rows(XQ, l, g.KP), rows(DR, l, g.NUP), rows(U, l, g.NUP),
                                         rows(XQ, l + 1, g.KP), Zc, true);
            stamp_();
            if (DYN) break;
        }

        if constexpr (!DYN) {
        // ================= dual: eta+ = prox_{alpha g*}(d + alpha L(2z+ - p)), xi2, delta2 =====
        // Operands read by several lanes (the parents' x, u rows of z+ and p, the child / node
        // records) are staged into LDS by LDS-DMA, a batch of levels at a time (one memory round
        // trip per batch); per-lane operands are plain loads.
        __syncthreads();  // the forward sweep's z+ stores (other waves) before they are read
        {
            const glbd* pz = Zp;
            const glbd* zp = Zc;
            auto finish = [&](int e, double dv, double v, double pv, double bb) {
                const double ep = alpha * (v - pv);
                Ee[e] = ep;
                const double x2 = (dv - ep) / alpha + bb;
                X2[e] = x2;
                m2 = fmax(m2, fabs(x2));
                m5 = fmax(m5, fabs(ep - dv));
            };
            auto box = [&](double v, double lo, double hi) {
                if (lo <= v && v <= hi) return v;
                if (v <= lo) return lo;
                if (v >= hi) return hi;
                nan_local = 1;
                return v;
            };
            for (int la = 0; la < L;) {
                // batch [la, lb): parent levels whose x / u rows (z+, p) and records fit the stage
                int lb = la, need = 0;
                while (lb < L) {
                    const int cp = s_hi[lb] - s_lo[lb], cc = s_hi[lb + 1] - s_lo[lb + 1];
                    const int nd = 2 * (rup(cp * nx, 2) + 4) + 2 * (rup(cp * nu, 2) + 4) + 2 * cp + 4 + 2 * cc + 4;
                    if (lb > la && need + nd > a.stage_cap) break;
                    need += nd;
                    ++lb;
                }
                int off = 0, rot = 0;
                for (int l = la; l < lb; ++l) {
                    const int lo = s_lo[l], cp = s_hi[l] - lo, lo1 = s_lo[l + 1], cc = s_hi[l + 1] - lo1;
                    const int o0 = stage(off, rot, zp + p.X0 + (size_t)lo * nx, cp * nx);
                    const int o1 = stage(off, rot, pz + p.X0 + (size_t)lo * nx, cp * nx);
                    const int o2 = stage(off, rot, zp + p.U0 + (size_t)lo * nu, cp * nu);
                    const int o3 = stage(off, rot, pz + p.U0 + (size_t)lo * nu, cp * nu);
                    const int o4 = stage_rec(off, rot, p.frec + lo, cp);
                    const int o5 = stage_rec(off, rot, p.crec + lo1, cc);
                    if (tid == 0) {
                        s_sg[l][0] = o0; s_sg[l][1] = o1; s_sg[l][2] = o2; s_sg[l][3] = o3;
                        s_sg[l][4] = o4; s_sg[l + 1][5] = o5;
                    }
                }
                dma_wait();
                __syncthreads();
                // children of the batch (levels la+1 .. lb): SOC on (eta3, eta4, eta5 | eta6)
                {
                    const int G = nx + nu + 2;
                    mega_groups(s_lo, s_hi, la + 1, lb + 1, G, [&](int j, int lj, int r, int base) {
                        const bool live = j >= 0;
                        double v = 0.0, bb = 0.0, dv = 0.0;
                        int e = -1;
                        if (live) {
                            const Rec cr = ((const ldsrec*)(STG + s_sg[lj][5]))[j - s_lo[lj]];  // {anc, iSQ, iSR}
                            const int pr = cr.x - s_lo[lj - 1];
                            double av = 0.0;
                            if (r < nx) {
                                e = e3(p, j) + r;
                                dot_zp<NXc>(SQl + (size_t)cr.y * nx * nx + r, nx, STG + s_sg[lj - 1][0] + pr * nx,
                                            STG + s_sg[lj - 1][1] + pr * nx, nx, av, bb);
                            } else if (r < nx + nu) {
                                const int rr = r - nx;
                                e = e4(p, j) + rr;
                                dot_zp<NUc>(SRl + (size_t)cr.z * nu * nu + rr, nu, STG + s_sg[lj - 1][2] + pr * nu,
                                            STG + s_sg[lj - 1][3] + pr * nu, nu, av, bb);
                            } else {
                                e = (r == nx + nu ? p.E5 : p.E6) + j;
                                const double zt = zp[p.T0 + j], pt = pz[p.T0 + j];
                                av = 0.5 * (2.0 * zt - pt);
                                bb = 0.5 * (zt - pt);
                            }
                            dv = Ed[e];
                            v = (dv + alpha * av) / alpha;
                            if (r == nx + nu) v += -0.5;
                            if (r == nx + nu + 1) v += 0.5;
                        }
                        SX[threadIdx.x] = (live && r < G - 1) ? v * v : 0.0;
                        if (live && r == G - 1) SX[threadIdx.x] = v;
                        __syncthreads();
                        if (live) {
                            double ss = 0.0;
                            for (int q = 0; q < G - 1; ++q) ss += SX[base + q];
                            finish(e, dv, v, soc_apply(v, r == G - 1, sqrt(ss), SX[base + G - 1]), bb);
                        }
                        __syncthreads();
                    });
                }
                // nonleaf nodes of the batch: eta1 (2c+1), eta2, eta7 (nx+nu)
                {
                    const int G = 2 * p.cmax + 2 + nx + nu;
                    mega_groups(s_lo, s_hi, la, lb, G, [&](int i, int li, int r, int) {
                        if (i < 0) return;
                        const int row = i - s_lo[li];
                        const Rec fr = ((const ldsrec*)(STG + s_sg[li][4]))[row];  // {yrel, nch, ch_start, e7off}
                        const int yo = fr.x, c = fr.y, cs = fr.z;
                        if (r < 2 * c + 1) {
                            const int e = p.E1 + yo + r;
                            const double zy = zp[p.Y0 + yo + r], py = pz[p.Y0 + yo + r];
                            const double dv = Ed[e];
                            const double v = (dv + alpha * (2.0 * zy - py)) / alpha;
                            finish(e, dv, v, r < 2 * c ? fmax(v, 0.0) : v, zy - py);
                        } else if (r == 2 * p.cmax + 1) {
                            const int e = p.E2 + i;
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
                            double zs, ps;
                            if (!top && i == root) {
                                zs = s_sr[0];
                                ps = s_sr[1];
                            } else {
                                zs = zp[p.S0 + i];
                                ps = pz[p.S0 + i];
                            }
                            const double dv = Ed[e];
                            const double v = (dv + alpha * ((2.0 * zs - ps) - bya)) / alpha;
                            finish(e, dv, v, fmax(v, 0.0), (zs - ps) - byb);
                        } else if (r >= 2 * p.cmax + 2 && fr.w >= 0) {
                            const int rr = r - (2 * p.cmax + 2);
                            const int e = fr.w + rr;
                            const double zv = rr < nx ? (double)STG[s_sg[li][0] + row * nx + rr]
                                                      : (double)STG[s_sg[li][2] + row * nu + rr - nx];
                            const double pv_ = rr < nx ? (double)STG[s_sg[li][1] + row * nx + rr]
                                                       : (double)STG[s_sg[li][3] + row * nu + rr - nx];
                            const double dv = Ed[e];
                            const double v = (dv + alpha * (2.0 * zv - pv_)) / alpha;
                            const int bi = p.iBnl[i];
                            finish(e, dv, v,
                                   box(v, p.blo_nl[(size_t)bi * (nx + nu) + rr], p.bhi_nl[(size_t)bi * (nx + nu) + rr]),
                                   zv - pv_);
                        }
                    });
                }
                __syncthreads();  // the stage is reused by the next batch
                la = lb;
            }
            // leaves (subtree level L): SOC on (eta11, eta12 | eta13), eta14 box
            if (!top) {
                {
                    const int lo = s_lo[L], cl = s_hi[L] - lo;
                    int off = 0, rot = 0;
                    const int o0 = stage(off, rot, zp + p.X0 + (size_t)lo * nx, cl * nx);
                    const int o1 = stage(off, rot, pz + p.X0 + (size_t)lo * nx, cl * nx);
                    const int o4 = stage_rec(off, rot, p.lrec + (lo - p.m), cl);  // {iSP, iBl, e14off}
                    if (tid == 0) { s_sg[L][0] = o0; s_sg[L][1] = o1; s_sg[L][4] = o4; }
                    dma_wait();
                    __syncthreads();
                }
                const int G = 2 * nx + 2;
                mega_groups(s_lo, s_hi, L, L + 1, G, [&](int l, int, int r, int base) {
                    const bool live = l >= 0;
                    double v = 0.0, bb = 0.0, dv = 0.0;
                    int e = -1;
                    Rec lr = {0, 0, -1, 0};
                    if (live) {
                        const int row = l - s_lo[L];
                        lr = ((const ldsrec*)(STG + s_sg[L][4]))[row];
                        const ldsd* xz = STG + s_sg[L][0] + row * nx;
                        const ldsd* xp = STG + s_sg[L][1] + row * nx;
                        double av = 0.0;
                        if (r < nx) {
                            e = e11(p, l) + r;
                            dot_zp<NXc>(SPl + (size_t)lr.x * nx * nx + r, nx, xz, xp, nx, av, bb);
                        } else if (r < nx + 2) {
                            e = (r == nx ? p.E12 : p.E13) + l;
                            const double zs = zp[p.S0 + l], ps = pz[p.S0 + l];
                            av = 0.5 * (2.0 * zs - ps);
                            bb = 0.5 * (zs - ps);
                        } else if (lr.z >= 0) {
                            const int rr = r - nx - 2;
                            e = lr.z + rr;
                            av = 2.0 * xz[rr] - xp[rr];
                            bb = xz[rr] - xp[rr];
                        }
                        if (e >= 0) {
                            dv = Ed[e];
                            v = (dv + alpha * av) / alpha;
                            if (r == nx) v += -0.5;
                            if (r == nx + 1) v += 0.5;
                        }
                    }
                    SX[threadIdx.x] = (live && r < nx + 1) ? v * v : 0.0;
                    if (live && r == nx + 1) SX[threadIdx.x] = v;
                    __syncthreads();
                    if (live && e >= 0) {
                        if (r < nx + 2) {
                            double ss = 0.0;
                            for (int q = 0; q < nx + 1; ++q) ss += SX[base + q];
                            finish(e, dv, v, soc_apply(v, r == nx + 1, sqrt(ss), SX[base + nx + 1]), bb);
                        } else {
                            const int rr = r - nx - 2;
                            finish(e, dv, v, box(v, p.blo_l[(size_t)lr.y * nx + rr], p.bhi_l[(size_t)lr.y * nx + rr]),
                                   bb);
                        }
                    }
                    __syncthreads();
                });
            }
        }
        __syncthreads();
        stamp_();

        // ================= next primal half step + kernel projection + residual terms ===========
        // The children's eta3 / eta4 rows (and the leaves' eta11) of the three duals eta+, d, xi2
        // are what several lanes read: staged per batch of parent levels.
        {
            const glbd* pz = Zp;   // p
            const glbd* zp = Zc;   // z+
            glbd* out = Zn;
            const glbd* dA = Ee;   // eta+
            const glbd* dP = Ed;   // d
            const glbd* dC = X2;   // xi2
            auto account = [&](int e, double w, double cc) {
                const double pp = pz[e], zz = zp[e];
                const double x1 = (pp - zz) / alpha - w, x0v = x1 + cc, dl1 = zz - pp, dl0 = dl1 + w;
                m0 = fmax(m0, fabs(x0v)); m1 = fmax(m1, fabs(x1));
                m3 = fmax(m3, fabs(dl0)); m4 = fmax(m4, fabs(dl1));
            };
            const int G = nx + nu + p.cmax + 1;
            for (int la = 0; la < L;) {
                int lb = la, need = 0;
                while (lb < L) {
                    const int cp = s_hi[lb] - s_lo[lb], cc = s_hi[lb + 1] - s_lo[lb + 1];
                    const int nd = 3 * (rup(cc * nx, 2) + 4) + 3 * (rup(cc * nu, 2) + 4) + 2 * cc + 4 + 2 * cp + 4;
                    if (lb > la && need + nd > a.stage_cap) break;
                    need += nd;
                    ++lb;
                }
                int off = 0, rot = 0;
                for (int l = la; l < lb; ++l) {
                    const int lo = s_lo[l], cp = s_hi[l] - lo, lo1 = s_lo[l + 1], cc = s_hi[l + 1] - lo1;
                    const int o0 = stage(off, rot, dA + e3(p, lo1), cc * nx);
                    const int o1 = stage(off, rot, dP + e3(p, lo1), cc * nx);
                    const int o2 = stage(off, rot, dC + e3(p, lo1), cc * nx);
                    const int o3 = stage(off, rot, dA + e4(p, lo1), cc * nu);
                    const int o4 = stage(off, rot, dP + e4(p, lo1), cc * nu);
                    const int o5 = stage(off, rot, dC + e4(p, lo1), cc * nu);
                    const int o6 = stage_rec(off, rot, p.crec + lo1, cc);
                    const int o7 = stage_rec(off, rot, p.frec + lo, cp);
                    if (tid == 0) {
                        s_sg[l + 1][0] = o0; s_sg[l + 1][1] = o1; s_sg[l + 1][2] = o2;
                        s_sg[l + 1][3] = o3; s_sg[l + 1][4] = o4; s_sg[l + 1][5] = o5;
                        s_sg[l + 1][6] = o6; s_sg[l][7] = o7;
                    }
                }
                dma_wait();
                __syncthreads();
                // families whose kernel projection waits for the next UP (the top's last level)
                const int lf = top ? min(lb, L - 1) : lb;
                for (int part = 0; part < 2; ++part) {
                    const int pa = part == 0 ? la : max(la, lf), pb = part == 0 ? lf : lb;
                    const bool full = part == 0;
                    if (pa >= pb) continue;
                    mega_groups(s_lo, s_hi, pa, pb, G, [&](int i, int li, int r, int base) {
                        const bool live = i >= 0;
                        int c = 0, cs = 0, yo = 0, o7 = -1;
                        if (live) {
                            const Rec fr = ((const ldsrec*)(STG + s_sg[li][7]))[i - s_lo[li]];
                            yo = fr.x;
                            c = fr.y;
                            cs = fr.z;
                            o7 = fr.w;
                        }
                        if (live && r < nx + nu) {
                            const bool isx = r < nx;
                            const int rr = isx ? r : r - nx;
                            double accA = 0.0, accW = 0.0, accC = 0.0;
                            if (o7 >= 0) {
                                const int e = o7 + (isx ? rr : nx + rr);
                                accA = dA[e];
                                accW = dP[e] - dA[e];
                                accC = dC[e];
                            }
                            const int lc = li + 1, c0r = cs - s_lo[lc];
                            const ldsrec* CR = (const ldsrec*)(STG + s_sg[lc][6]);
                            for (int q = 0; q < c; ++q) {
                                const int jr = c0r + q;
                                const Rec cr = CR[jr];
                                double sA, sW, sC;
                                if (isx)
                                    dot_lt3<NXc, true>(SQl + (size_t)cr.y * nx * nx + rr, nx, STG + s_sg[lc][0] + jr * nx,
                                                       STG + s_sg[lc][1] + jr * nx, STG + s_sg[lc][2] + jr * nx, nx, sA,
                                                       sW, sC);
                                else
                                    dot_lt3<NUc, true>(SRl + (size_t)cr.z * nu * nu + rr, nu, STG + s_sg[lc][3] + jr * nu,
                                                       STG + s_sg[lc][4] + jr * nu, STG + s_sg[lc][5] + jr * nu, nu, sA,
                                                       sW, sC);
                                accA += sA;
                                accW += sW;
                                accC += sC;
                            }
                            const int e = isx ? p.X0 + i * nx + rr : p.U0 + i * nu + rr;
                            out[e] = zp[e] - alpha * accA;
                            account(e, accW, accC);
                        }
                        if (!full) return;  // uniform per call: no lane reaches the barriers below
                        const int rk = r - (nx + nu);
                        double vals[4] = {0, 0, 0, 0};
                        double y2c = 0.0;
                        const double e2A = live ? dA[p.E2 + i] : 0.0;
                        const double e2W = live ? dP[p.E2 + i] - dA[p.E2 + i] : 0.0;
                        const double e2C = live ? dC[p.E2 + i] : 0.0;
                        if (live && rk >= 0 && rk < c) {
                            const int j = cs + rk;
                            const double b = p.cond[j];
                            const int ey0 = p.Y0 + yo + rk, ey1 = p.Y0 + yo + c + rk;
                            const int f0 = p.E1 + yo + rk, f1 = p.E1 + yo + c + rk;
                            vals[0] = zp[ey0] - alpha * (dA[f0] - b * e2A);
                            vals[1] = zp[ey1] - alpha * (dA[f1] - 0.0 * e2A);
                            vals[2] = zp[p.T0 + j] - alpha * (0.5 * (dA[p.E5 + j] + dA[p.E6 + j]));
                            const double lts = j < p.m ? dA[p.E2 + j] : 0.5 * (dA[p.E12 + j] + dA[p.E13 + j]);
                            vals[3] = zp[p.S0 + j] - alpha * lts;
                            account(ey0, (dP[f0] - dA[f0]) - b * e2W, dC[f0] - b * e2C);
                            account(ey1, (dP[f1] - dA[f1]) - 0.0 * e2W, dC[f1] - 0.0 * e2C);
                            account(p.T0 + j, 0.5 * ((dP[p.E5 + j] - dA[p.E5 + j]) + (dP[p.E6 + j] - dA[p.E6 + j])),
                                    0.5 * (dC[p.E5 + j] + dC[p.E6 + j]));
                            double ws, cs2;
                            if (j < p.m) {
                                ws = dP[p.E2 + j] - dA[p.E2 + j];
                                cs2 = dC[p.E2 + j];
                            } else {
                                ws = 0.5 * ((dP[p.E12 + j] - dA[p.E12 + j]) + (dP[p.E13 + j] - dA[p.E13 + j]));
                                cs2 = 0.5 * (dC[p.E12 + j] + dC[p.E13 + j]);
                            }
                            account(p.S0 + j, ws, cs2);
                        }
                        if (live && rk == p.cmax) {
                            const int f2 = p.E1 + yo + 2 * c, ey2 = p.Y0 + yo + 2 * c;
                            y2c = zp[ey2] - alpha * (dA[f2] - 1.0 * e2A);
                            account(ey2, (dP[f2] - dA[f2]) - 1.0 * e2W, dC[f2] - 1.0 * e2C);
                            if (i == 0) {
                                out[p.S0] = (zp[p.S0] - alpha * e2A) - alpha;
                                account(p.S0, e2W, e2C);
                            }
                        }
                        kernel_proj_group(p, live ? i : 0, c, cs, rk, live && rk >= 0, base + nx + nu, SX, vals, y2c);
                        if (live && rk >= 0 && rk < c) {
                            const int j = cs + rk;
                            out[p.Y0 + yo + rk] = vals[0];
                            out[p.Y0 + yo + c + rk] = vals[1];
                            out[p.T0 + j] = vals[2];
                            out[p.S0 + j] = vals[3];
                        }
                        if (live && rk == p.cmax) out[p.Y0 + yo + 2 * c] = y2c;
                        __syncthreads();
                    });
                }
                __syncthreads();  // the stage is reused by the next batch
                la = lb;
            }
            // leaves: x = sqrtPf eta11 + eta14
            if (!top) {
                {
                    const int lo = s_lo[L], cl = s_hi[L] - lo;
                    int off = 0, rot = 0;
                    const int o0 = stage(off, rot, dA + e11(p, lo), cl * nx);
                    const int o1 = stage(off, rot, dP + e11(p, lo), cl * nx);
                    const int o2 = stage(off, rot, dC + e11(p, lo), cl * nx);
                    const int o4 = stage_rec(off, rot, p.lrec + (lo - p.m), cl);
                    if (tid == 0) { s_sg[L][0] = o0; s_sg[L][1] = o1; s_sg[L][2] = o2; s_sg[L][4] = o4; }
                    dma_wait();
                    __syncthreads();
                }
                mega_groups(s_lo, s_hi, L, L + 1, nx, [&](int l, int, int r, int) {
                    if (l < 0) return;
                    const int row = l - s_lo[L];
                    const Rec lr = ((const ldsrec*)(STG + s_sg[L][4]))[row];
                    double sA, sW, sC;
                    dot_lt3<NXc, true>(SPl + (size_t)lr.x * nx * nx + r, nx, STG + s_sg[L][0] + row * nx,
                                       STG + s_sg[L][1] + row * nx, STG + s_sg[L][2] + row * nx, nx, sA, sW, sC);
                    const int o14 = lr.z;
                    if (o14 >= 0) {
                        sA += dA[o14 + r];
                        sW += dP[o14 + r] - dA[o14 + r];
                        sC += dC[o14 + r];
                    }
                    const int e = p.X0 + l * nx + r;
                    out[e] = zp[e] - alpha * sA;
                    account(e, sW, sC);
                });
            }
        }
        __syncthreads();
        stamp_();
        }  // !DYN
    }
    if (!s_ok && tid == 0) atomicOr(&a.ctl->flags, 2);
}
