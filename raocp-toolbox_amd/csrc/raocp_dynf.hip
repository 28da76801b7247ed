// raocp_dynf.hip — the tiered dynamics projection (raocp_dyn.hip) in TWO launches: the
// split sweep k_dyn_up / k_dyn_down. Included by raocp_kernels.hip after raocp_dyn.hip
// (inside namespace raocp). The fallback of trees the regular-tree sweep (raocp_dynr.hip)
// does not take but whose tier plan is regular (every subtree of a tier the same shape, ids
// consecutive): e.g. Markov trees with uniform branching (BASELINE configs[2]).
//
// Same recursion and level routines as the tier kernels (cache.py:259-288; header of
// raocp_dyn.hip), same cut into the top (stages [0, s)) and tiers t[0] .. t[K-1] below it,
// one workgroup per subtree of every tier plus one for the top, each with ONE role fixed by
// its block index, so every workgroup stages its tables and vectors at its start and only
// the dependent rows (the children's q, the parent's x) wait for a hand-off (below).
//
// Hand-offs across workgroups (MI355X: per-XCD L2s are not coherent): the roots' q rows
// and the boundary x rows are stored write-through (st_sc1) and read with ld_sc1; after a
// barrier one lane arrives / stores the flag with agent-scope release, the waiter polls
// relaxed and takes an agent-scope acquire before the barrier that frees its readers. The
// host launches the sweep only where the whole grid is co-resident
// (hipOccupancyMaxActiveBlocksPerMultiprocessor), so no wait depends on the dispatch order;
// every wait is bounded (FuseArg::timeout) and a timed-out workgroup sets the error word,
// which every workgroup of a later launch reads at its start and then leaves at once.

constexpr int kFuseTiers = 4;
// workgroup size of the fused sweep: at most 512 lanes leaves 256 VGPRs per lane (the tier,
// top and forward routines inlined into one kernel spill at 1024 lanes' 128)
constexpr int kFuseBlock = 512;

struct FuseTier {
    int s0, s1;        // roots at stage s0, levels s0 .. s1-1, boundary nodes at s1
    int r;             // subtrees of this tier under one subtree of the tier above (or the top)
    int c0, c1, p0, p1;
    int maxch;         // widest child level of one subtree (P rows)
    int fm;            // F rows in the forward sweep: 1 every pair of the tier, 2 per level
    int fold;          // one-phase backward levels (per-pair WT tables, back_fold)
    int nnl;           // nonleaf nodes of one subtree (levels 0 .. L-1)
    int ngroups;       // subtrees of the tier above (tickets / flags)
    TierArg ta;        // regular tier: level sizes and first nodes
    unsigned* cnt;     // [ngroups] tickets
    unsigned* flag;    // [ngroups] forward released by the tier above
};

struct FuseArg {
    int K;                          // tiers below the top
    FuseTier t[kFuseTiers];
    int s, T, nb, c1, p1, maxch_top; // the top: stages [0, s), nodes [0, T), nb boundary roots
    int fold_top;                   // the top's backward levels in one phase
    unsigned* epoch;
    int* err;                       // set to 1 by a workgroup whose wait timed out
    long long timeout;              // per wait, 100 MHz ticks
    ChkArg ck;                      // the previous CP iteration's stopping test
};

// diagnostics: thread 0 stamps the next slot of this workgroup's path (p.stamps != nullptr)
__device__ __forceinline__ void fz_stamp(const Dev& p, Prologue& pl) {
    if (kDiag && p.stamps && threadIdx.x == 0) pl.ts[pl.nts++ & 63] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ unsigned ld_u32_sc1(const unsigned* p) {
    return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_u32_sc1(unsigned* p, unsigned v) {
    __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// level l of subtree `sub` of a regular tier: first node and count
__device__ __forceinline__ int fz_lo(const TierArg& ta, int l, int sub) { return ta.lo0[l] + sub * ta.cnt[l]; }

__device__ __forceinline__ void fz_levels(Prologue& pl, const TierArg& ta, int L, int sub) {
    const int l = threadIdx.x;
    if (l > L) return;
    int off = 0;
    for (int k = 0; k < l; ++k) off += ta.cnt[k];
    pl.lo[l] = fz_lo(ta, l, sub);
    pl.hi[l] = pl.lo[l] + ta.cnt[l];
    pl.off[l] = off;
}

// backward sweep of subtree `sub` of tier tt in two parts: fz_back_stage issues the copies
// of everything the subtree's own data holds (tables, x / u rows, records), so a workgroup
// can prefetch a subtree before it knows whether it will sweep it; fz_back_wait copies the
// boundary q rows other workgroups published (not for the deepest tier, whose boundary is
// the leaves' x) and waits for every copy in flight; fz_back_levels runs the levels and
// publishes the root's q row (padded) to qbuf. A prefetch issued between the two overlaps
// the levels (the waits are vmcnt(0): a prefetch issued before a wait is waited for).
// region: [W (all kinds) | RG (c0..c1) | XQ (nall, KP) | U (nnl, NUP) | P | NL | CH];
// fold: W -> WT (pairs p0..p1), no P rows
template <int NXc, int NUc>
struct BackLds {
    ldsd *W, *RG, *XQ, *U, *PB, *NL, *CH;
    int nall;
    __device__ __forceinline__ BackLds(const Dev& p, const FuseTier& tt, ldsd* scr) {
        const Geo<NXc, NUc> g(p);
        const TabSize<NXc, NUc> ts(g);
        const int L = tt.s1 - tt.s0;
        nall = tt.nnl + tt.ta.cnt[L];
        W = scr;
        RG = W + (tt.fold ? tt.p1 - tt.p0 : p.nkind) * ts.W1;
        XQ = RG + (tt.c1 - tt.c0) * ts.RG1;
        U = XQ + (size_t)nall * g.KP;
        PB = U + (size_t)tt.nnl * g.NUP;
        NL = PB + (tt.fold ? 0 : rup(tt.maxch * g.PS, 2));
        CH = NL + 2 * tt.nnl;
    }
};

template <int NXc, int NUc>
__device__ void fz_back_stage(const Dev& p, const glbd* z, const FuseTier& tt, int sub, bool leaves, ldsd* scr) {
    const Geo<NXc, NUc> g(p);
    const TabSize<NXc, NUc> ts(g);
    const bool dmaok = (g.nx % 2 == 0) && (g.nu % 2 == 0);
    const int tid = threadIdx.x, nthr = blockDim.x;
    const TierArg& ta = tt.ta;
    const int L = tt.s1 - tt.s0;
    const BackLds<NXc, NUc> ly(p, tt, scr);
    int rot = p.dyn_rot ? 0 : -1;
    if (tt.fold) dma_r(ly.W, p.dWT + (size_t)tt.p0 * ts.W1, (tt.p1 - tt.p0) * ts.W1, rot);
    else dma_r(ly.W, p.dW, p.nkind * ts.W1, rot);
    dma_r(ly.RG, p.dRG + (size_t)tt.c0 * ts.RG1, (tt.c1 - tt.c0) * ts.RG1, rot);
    for (int l = 0, off = 0; l <= L; ++l) {
        const int lo = fz_lo(ta, l, sub), cnt = ta.cnt[l];
        if (l < L || leaves)
            rows_in_r(dmaok, ly.XQ + (size_t)off * g.KP, g.KP, (const double*)z + p.X0 + (size_t)lo * g.nx, g.nx, g.nx,
                      cnt, p.zpage, tid, nthr, rot);
        if (l < L) {
            rows_in_r(dmaok, ly.U + (size_t)off * g.NUP, g.NUP, (const double*)z + p.U0 + (size_t)lo * g.nu, g.nu, g.nu,
                      cnt, p.zpage, tid, nthr, rot);
            dma_r(ly.NL + 2 * off, (const double*)(p.ninfo + lo), 2 * cnt, rot);
        }
        if (l > 0) dma_r(ly.CH + 2 * (off - 1), (const double*)(p.cinfo + lo), 2 * cnt, rot);
        off += cnt;
    }
}

template <int NXc, int NUc>
__device__ void fz_back_wait(const Dev& p, const double* qbuf_, const FuseTier& tt, int sub, bool leaves, ldsd* scr,
                             Prologue& pl) {
    const Geo<NXc, NUc> g(p);
    const int tid = threadIdx.x, nthr = blockDim.x;
    const TierArg& ta = tt.ta;
    const BackLds<NXc, NUc> ly(p, tt, scr);
    const int L = tt.s1 - tt.s0;
    fz_levels(pl, ta, L, sub);
    // (LDS stores here, not in the stage: a store into a region with LDS-DMA copies in
    // flight waits for them)
    if (!tt.fold) zero_fill(ly.PB, tt.maxch * g.PS, tid, nthr);
    if (!leaves) {  // q rows of the tier below's roots, published by other workgroups (issued last:
                    // their wait covers the staging copies still in flight)
        const int lo = fz_lo(ta, L, sub), cnt = ta.cnt[L];
        for (int e = tid; e < cnt * g.KP; e += nthr)
            ly.XQ[(size_t)tt.nnl * g.KP + e] = ld_sc1(qbuf_ + (size_t)lo * g.KP + e);
    }
    dma_wait();
    lds_sync();
    fz_stamp(p, pl);
}

// d_i goes to the tier's XD rows in LDS (XD; the fused sweep's forward reads them there) or,
// with dglob, to global rows (the split sweep's forward is the next launch)
template <int NXc, int NUc>
__device__ void fz_back_levels(const Dev& p, double* qbuf_, const FuseTier& tt, int sub, bool leaves, ldsd* XD,
                               ldsd* scr, Prologue& pl, glbd* dglob = nullptr) {
    const Geo<NXc, NUc> g(p);
    const int tid = threadIdx.x, nthr = blockDim.x;
    const TierArg& ta = tt.ta;
    const int L = tt.s1 - tt.s0;
    const BackLds<NXc, NUc> ly(p, tt, scr);
    const ldsrec* NL = (const ldsrec*)ly.NL;
    const ldsrec* CH = (const ldsrec*)ly.CH;
    const TabsT<const ldsd*, const ldsd*> tb{ly.W, ly.RG, nullptr, nullptr, tt.c0, tt.fold ? tt.p0 : 0};
    const GRows dg{dglob, 0, g.nu};
    for (int l = L - 1; l >= 0; --l) {
        const InfoT<const ldsrec*> inf{NL + pl.off[l], pl.lo[l], CH + pl.off[l + 1] - 1, pl.lo[l + 1]};
        const LRows xq_l{ly.XQ + (size_t)pl.off[l] * g.KP, pl.lo[l], g.KP};
        const LRows xq_c{ly.XQ + (size_t)pl.off[l + 1] * g.KP, pl.lo[l + 1], g.KP};
        const LRows ur{ly.U + (size_t)pl.off[l] * g.NUP, pl.lo[l], g.NUP};
        const LRows dl{XD + (size_t)pl.off[l] * g.KF + g.nx, pl.lo[l], g.KF};  // d_i into XD row i, cols nx..
        const double sign = (l + 1 == L && leaves) ? -1.0 : 1.0;
        if (tt.fold) {
            if (dglob) back_fold<NXc, NUc>(p, tb, inf, pl.lo[l], pl.hi[l], xq_c, sign, xq_l, ur, xq_l, dg, tid, nthr);
            else back_fold<NXc, NUc>(p, tb, inf, pl.lo[l], pl.hi[l], xq_c, sign, xq_l, ur, xq_l, dl, tid, nthr);
            lds_sync();
            continue;
        }
        const LRows pr{ly.PB, pl.lo[l + 1], g.PS};
        back_phase_a<NXc, NUc>(p, tb, inf, pl.lo[l + 1], pl.hi[l + 1], xq_c, sign, pr, tid, nthr);
        lds_sync();
        if (dglob) back_phase_b<NXc, NUc>(p, tb, inf, pl.lo[l], pl.hi[l], pr, xq_l, ur, xq_l, dg, tid, nthr);
        else back_phase_b<NXc, NUc>(p, tb, inf, pl.lo[l], pl.hi[l], pr, xq_l, ur, xq_l, dl, tid, nthr);
        lds_sync();
    }
    // the root's q row (XQ row 0, zero tail) for the tier above
    const int root = fz_lo(ta, 0, sub);
    if (tid < g.KP) st_sc1(qbuf_ + (size_t)root * g.KP + tid, ly.XQ[tid]);
}

// forward sweep of subtree `sub` of tier tt, in two parts: fz_fwd_stage issues the table
// and record copies (a waiting workgroup issues them before its wait), fz_fwd_run takes the
// root's x row published by the tier above (or the top) and runs the levels. sc: the
// boundary children's x rows are published (every tier but the deepest).
// scratch: [KM (c0..c1) | F (fm 1: pairs p0..p1; 2: one level's pairs) | NL | CH]
template <int NXc, int NUc>
struct FwdLds {
    ldsd *KM, *F, *NL, *CH;
    __device__ __forceinline__ FwdLds(const Dev& p, const FuseTier& tt, ldsd* scr) {
        const Geo<NXc, NUc> g(p);
        const TabSize<NXc, NUc> ts(g);
        const int L = tt.s1 - tt.s0;
        int npl = tt.p1 - tt.p0;
        if (tt.fm == 2) {
            npl = 0;
            for (int l = 0; l < L; ++l) npl = max(npl, tt.ta.pl0[l + 1] - tt.ta.pl0[l]);
        }
        KM = scr;
        F = KM + (tt.c1 - tt.c0) * ts.KM1;
        NL = F + npl * ts.F1;
        CH = NL + 2 * tt.nnl;
    }
};

template <int NXc, int NUc>
__device__ void fz_fwd_stage(const Dev& p, const FuseTier& tt, int sub, ldsd* scr) {
    const Geo<NXc, NUc> g(p);
    const TabSize<NXc, NUc> ts(g);
    const TierArg& ta = tt.ta;
    const int L = tt.s1 - tt.s0;
    const FwdLds<NXc, NUc> ly(p, tt, scr);
    int rot = p.dyn_rot ? 0 : -1;
    dma_r(ly.KM, p.dKM + (size_t)tt.c0 * ts.KM1, (tt.c1 - tt.c0) * ts.KM1, rot);
    if (tt.fm == 1) dma_r(ly.F, p.dF + (size_t)tt.p0 * ts.F1, (tt.p1 - tt.p0) * ts.F1, rot);
    else dma_r(ly.F, p.dF + (size_t)ta.pl0[0] * ts.F1, (ta.pl0[1] - ta.pl0[0]) * ts.F1, rot);
    for (int l = 0, off = 0; l <= L; ++l) {
        const int lo = fz_lo(ta, l, sub), cnt = ta.cnt[l];
        if (l < L) dma_r(ly.NL + 2 * off, (const double*)(p.ninfo + lo), 2 * cnt, rot);
        if (l > 0) dma_r(ly.CH + 2 * (off - 1), (const double*)(p.cinfo + lo), 2 * cnt, rot);
        off += cnt;
    }
    (void)g;
}

template <int NXc, int NUc>
__device__ void fz_fwd_run(const Dev& p, glbd* z, const FuseTier& tt, int sub, bool sc, ldsd* XD, ldsd* scr,
                           Prologue& pl) {
    const Geo<NXc, NUc> g(p);
    const TabSize<NXc, NUc> ts(g);
    const int tid = threadIdx.x, nthr = blockDim.x;
    const TierArg& ta = tt.ta;
    const int L = tt.s1 - tt.s0;
    const FwdLds<NXc, NUc> ly(p, tt, scr);
    const int root = fz_lo(ta, 0, sub);
    fz_levels(pl, ta, L, sub);
    if (tid < g.nx) XD[tid] = ld_sc1((const double*)z + p.X0 + (size_t)root * g.nx + tid);
    dma_wait();
    lds_sync();
    fz_stamp(p, pl);
    const ldsrec* NL = (const ldsrec*)ly.NL;
    const ldsrec* CH = (const ldsrec*)ly.CH;
    TabsT<const ldsd*, const ldsd*> tb{nullptr, nullptr, ly.KM, ly.F, tt.c0, tt.fm == 1 ? tt.p0 : ta.pl0[0]};
    for (int l = 0; l < L; ++l) {
        if (tt.fm == 2 && l > 0) {  // level l-1's products are done (the barrier that ended it)
            tb.p0 = ta.pl0[l];
            dma(ly.F, p.dF + (size_t)ta.pl0[l] * ts.F1, (ta.pl0[l + 1] - ta.pl0[l]) * ts.F1);
            dma_wait();
            lds_sync();
        }
        const InfoT<const ldsrec*> inf{NL + pl.off[l], pl.lo[l], CH + pl.off[l + 1] - 1, pl.lo[l + 1]};
        const LRows xd_l{XD + (size_t)pl.off[l] * g.KF, pl.lo[l], g.KF};
        if (l + 1 < L) {
            const LRows xd_c{XD + (size_t)pl.off[l + 1] * g.KF, pl.lo[l + 1], g.KF};
            fwd_phase<NXc, NUc, true>(p, tb, inf, pl.lo[l], pl.hi[l], xd_l, z, xd_c, tid, nthr);
        } else if (sc) {
            fwd_phase<NXc, NUc, false, true>(p, tb, inf, pl.lo[l], pl.hi[l], xd_l, z, xd_l, tid, nthr);
        } else {
            fwd_phase<NXc, NUc, false>(p, tb, inf, pl.lo[l], pl.hi[l], xd_l, z, xd_l, tid, nthr);
        }
        lds_sync();
    }
}

// the top (stages [0, s), nodes [0, T)), backward then forward, as k_dyn_top: the boundary
// q rows come from tier t[0]'s roots (ld_sc1), the boundary x rows are published
// [W | RG | KM | F (FL) | XQ (T, KP) | QB (nb, KP) | U (T, NUP) | XD (T, KF) | P | NL | CH]
// The top's layout: [W | RG | KM | F (FL) | XQ (T, KP) | QB (nb, KP) | U (T, NUP) | XD (T, KF) | P | NL | CH];
// bwd (split sweep): backward only (no KM / F), d_i of the top's nodes also stored to
// global rows for the next launch's forward sweep
template <int NXc, int NUc, bool FL>
struct TopLds {
    int oW, oRG, oKM, oF, oXQ, oQB, oU, oXD, oP, oNL, oCH;
    __device__ __forceinline__ TopLds(const Dev& p, const FuseArg& fa, bool bwd) {
        const Geo<NXc, NUc> g(p);
        const TabSize<NXc, NUc> ts(g);
        const int T = fa.T, nb = fa.nb, c1 = fa.c1, p1 = fa.p1;
        const bool fold = fa.fold_top;
        oW = 0;
        oRG = oW + (fold ? p1 : p.nkind) * ts.W1;
        oKM = oRG + c1 * ts.RG1;
        oF = oKM + (bwd ? 0 : c1 * ts.KM1);
        oXQ = oF + (FL && !bwd ? p1 * ts.F1 : 0);
        oQB = oXQ + T * g.KP;
        oU = oQB + nb * g.KP;
        oXD = oU + T * g.NUP;
        oP = oXD + T * g.KF;
        oNL = oP + (fold ? 0 : rup(fa.maxch_top * g.PS, 2));
        oCH = oNL + 2 * T;
    }
};

// everything but the boundary q rows (issued before a wait for them)
template <int NXc, int NUc, bool FL>
__device__ void fz_top_stage(const Dev& p, const glbd* z, const FuseArg& fa, ldsd* scr, Prologue& pl, bool bwd) {
    const Geo<NXc, NUc> g(p);
    const TabSize<NXc, NUc> ts(g);
    const bool dmaok = (g.nx % 2 == 0) && (g.nu % 2 == 0);
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int s = fa.s, T = fa.T, nb = fa.nb, c1 = fa.c1, p1 = fa.p1;
    const bool fold = fa.fold_top;
    const TopLds<NXc, NUc, FL> o(p, fa, bwd);
    int rot = p.dyn_rot ? 0 : -1;
    dma_r(scr + o.oW, fold ? p.dWT : p.dW, (fold ? p1 : p.nkind) * ts.W1, rot);
    dma_r(scr + o.oRG, p.dRG, c1 * ts.RG1, rot);
    if (!bwd) dma_r(scr + o.oKM, p.dKM, c1 * ts.KM1, rot);
    if (FL && !bwd) dma_r(scr + o.oF, p.dF, p1 * ts.F1, rot);
    dma_r(scr + o.oNL, (const double*)p.ninfo, 2 * T, rot);
    dma_r(scr + o.oCH, (const double*)(p.cinfo + 1), 2 * (T + nb - 1), rot);
    if (tid <= s + 1) pl.sp[tid] = p.stage_ptr[tid];
    rows_in_r(dmaok, scr + o.oXQ, g.KP, (const double*)z + p.X0, g.nx, g.nx, T, p.zpage, tid, nthr, rot);
    rows_in_r(dmaok, scr + o.oU, g.NUP, (const double*)z + p.U0, g.nu, g.nu, T, p.zpage, tid, nthr, rot);
}

template <int NXc, int NUc, bool FL>
__device__ void fz_top_run(const Dev& p, glbd* z, const double* qbuf_, const double* x0_, const FuseArg& fa, ldsd* scr,
                           Prologue& pl, glbd* dglob) {
    const Geo<NXc, NUc> g(p);
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int s = fa.s, T = fa.T, nb = fa.nb;
    const bool fold = fa.fold_top;
    const bool bwd = dglob != nullptr;
    const TopLds<NXc, NUc, FL> o(p, fa, bwd);
    zero_fill(scr + o.oXD, T * g.KF, tid, nthr);
    if (!fold) zero_fill(scr + o.oP, fa.maxch_top * g.PS, tid, nthr);
    // the boundary q rows last: their wait covers the copies still in flight
    for (int e = tid; e < nb * g.KP; e += nthr) scr[o.oQB + e] = ld_sc1(qbuf_ + (size_t)T * g.KP + e);
    dma_wait();
    lds_sync();
    fz_stamp(p, pl);
    typedef typename std::conditional<FL, const ldsd*, const glbd*>::type PF;
    const TabsT<const ldsd*, PF> tb{scr + o.oW, scr + o.oRG, scr + o.oKM,
                                    FL ? (PF)(scr + o.oF) : (PF)((const glbd*)p.dF), 0, 0};
    const InfoT<const ldsrec*> inf{(const ldsrec*)(scr + o.oNL), 0, (const ldsrec*)(scr + o.oCH), 1};
    ldsd* XD = scr + o.oXD;
    const LRows xq{scr + o.oXQ, 0, g.KP}, qb{scr + o.oQB, T, g.KP}, ur{scr + o.oU, 0, g.NUP}, xd{XD, 0, g.KF};
    const LRows dlds{XD + g.nx, 0, g.KF};
    for (int t = s - 1; t >= 0; --t) {
        const int b = pl.sp[t], e = pl.sp[t + 1];
        const int cb = e, ce = pl.sp[t + 2];
        if (fold) {
            if (t + 1 < s) back_fold<NXc, NUc>(p, tb, inf, b, e, xq, 1.0, xq, ur, xq, dlds, tid, nthr);
            else back_fold<NXc, NUc>(p, tb, inf, b, e, qb, 1.0, xq, ur, xq, dlds, tid, nthr);
            lds_sync();
            continue;
        }
        const LRows pr{scr + o.oP, cb, g.PS};
        if (t + 1 < s) back_phase_a<NXc, NUc>(p, tb, inf, cb, ce, xq, 1.0, pr, tid, nthr);
        else back_phase_a<NXc, NUc>(p, tb, inf, cb, ce, qb, 1.0, pr, tid, nthr);
        lds_sync();
        back_phase_b<NXc, NUc>(p, tb, inf, b, e, pr, xq, ur, xq, dlds, tid, nthr);
        lds_sync();
    }
    fz_stamp(p, pl);
    if (bwd) {  // d of the top's nodes for the next launch's forward sweep
        for (int e = tid; e < T * g.nu; e += nthr) {
            const int i = e / g.nu, c = e - i * g.nu;
            dglob[(size_t)i * g.nu + c] = XD[(size_t)i * g.KF + g.nx + c];
        }
        return;
    }
    if (tid < g.nx) {
        const double v = ((const glbd*)x0_)[tid];
        XD[tid] = v;
        z[p.X0 + tid] = v;  // x_0 = x0bar (cache.py:282)
    }
    lds_sync();
    for (int t = 0; t < s; ++t) {
        const int b = pl.sp[t], e = pl.sp[t + 1];
        if (t + 1 < s) fwd_phase<NXc, NUc, true>(p, tb, inf, b, e, xd, z, xd, tid, nthr);
        else fwd_phase<NXc, NUc, false, true>(p, tb, inf, b, e, xd, z, xd, tid, nthr);
        lds_sync();
    }
}

// hand-off publish: the workgroup's payload stores (write-through) happen before the barrier,
// then one lane releases at agent scope (HIP memory model: the barrier orders every lane's
// stores before lane 0's release; the waiter's acquire after its poll orders the payload
// reads after it)
__device__ __forceinline__ void fz_release_add(unsigned* c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores have reached the L2
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add((gu32*)c, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fz_release_store(unsigned* f, unsigned v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores have reached the L2
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store((gu32*)f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// ==============================================================================
// The split sweep:
//   k_dyn_up:   [deferred stopping test] [deepest subtrees] [tier D-1] .. [tier 0] [top]
//               a tier-k workgroup waits until its r children subtrees have published
//               their q rows (a counter of arrivals), sweeps backward, publishes its
//               root's q row and arrives at its parent's counter; the top sweeps backward
//               and bumps the epoch. d_i goes to global rows.
//   k_dyn_down: [top] [tier 0] .. [deepest]: the top sweeps forward and releases tier 0;
//               a tier-k workgroup waits for its parent's flag (the launch's epoch),
//               sweeps forward, publishes its boundary x rows and releases its children.
// Counters are reset by their one consumer after its wait; flags carry the epoch, which
// k_dyn_up's top advances once per projection.

// spin (one lane, relaxed polls) until *f == v, bounded, then an agent-scope acquire; false
// on a timeout (error word set)
__device__ __forceinline__ bool fz_wait_eq(const unsigned* f, unsigned v, const FuseArg& fa, int& ok) {
    if (threadIdx.x == 0) {
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        while (ld_u32_sc1(f) != v) {
            if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > fa.timeout) {
                ok = 0;
                __hip_atomic_store(fa.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return ok != 0;
}

template <int NXc, int NUc>
__global__ void __launch_bounds__(kFuseBlock) k_dyn_up(Dev p, Bufs bf, const Ctl* ctl, int zsel,
                                                       double* qbuf_, double* dbuf_, FuseArg fa) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ Prologue pl;
    __shared__ int s_ok;
    const int tid = threadIdx.x;
    if (fa.ck.on && blockIdx.x == 0) {  // the previous CP iteration's stopping test
        if (tid < 64) cp_check_wave(fa.ck);
        return;
    }
    if (ld_u32_sc1((const unsigned*)fa.err)) return;  // an earlier hand-off timed out: the host resets
    ldsd* smem = (ldsd*)smem_;
    glbd* z = dyn_z(bf, zsel, ctl);
    if (tid == 0) {
        pl.nts = 0;
        s_ok = 1;
    }
    fz_stamp(p, pl);
    const int D = fa.K - 1;
    int b = (int)blockIdx.x - (fa.ck.on ? 1 : 0), k = D;
    for (; k >= 0 && b >= fa.t[k].ngroups * fa.t[k].r; --k) b -= fa.t[k].ngroups * fa.t[k].r;
    if (k >= 0) {  // subtree b of tier k
        const FuseTier& tt = fa.t[k];
        fz_back_stage<NXc, NUc>(p, z, tt, b, k == D, smem);
        const bool work = !ctl_done(ctl);
        if (k < D && !fz_wait_eq(fa.t[k + 1].cnt + b, (unsigned)fa.t[k + 1].r, fa, s_ok)) return;
        if (k < D && tid == 0) st_u32_sc1(fa.t[k + 1].cnt + b, 0u);
        fz_stamp(p, pl);
        if (work) {
            fz_back_wait<NXc, NUc>(p, qbuf_, tt, b, k == D, smem, pl);
            fz_back_levels<NXc, NUc>(p, qbuf_, tt, b, k == D, nullptr, smem, pl, (glbd*)dbuf_);
        }
        fz_stamp(p, pl);
        fz_release_add(tt.cnt + b / tt.r);
        fz_stamp(p, pl);
        if (kDiag && p.stamps && tid == 0 && b == 0 && (k == 0 || k == D))  // diagnostics: tier 0 / deepest, subtree 0
            for (int q = 0; q < pl.nts && q < 64; ++q) p.stamps[(k == 0 ? 64 : 128) + q] = pl.ts[q];
    } else {  // the top
        fz_top_stage<NXc, NUc, false>(p, z, fa, smem, pl, true);
        const unsigned e = ld_u32_sc1(fa.epoch);
        const bool work = !ctl_done(ctl);
        if (!fz_wait_eq(fa.t[0].cnt, (unsigned)fa.t[0].r, fa, s_ok)) return;
        if (tid == 0) st_u32_sc1(fa.t[0].cnt, 0u);
        fz_stamp(p, pl);
        if (work) fz_top_run<NXc, NUc, false>(p, z, qbuf_, nullptr, fa, smem, pl, (glbd*)dbuf_);
        fz_stamp(p, pl);
        fz_release_store(fa.epoch, e + 1u);
        if (kDiag && p.stamps && tid == 0)
            for (int q = 0; q < pl.nts && q < 64; ++q) p.stamps[q] = pl.ts[q];
    }
}

// the top's forward sweep (k_dyn_down's block 0):
// [KM (0..c1) | F (pairs 0..p1, FL) | XD (T, KF) = [x | d | 0] | NL (T) | CH (T + nb - 1)]
template <int NXc, int NUc, bool FL>
__device__ void fz_top_fwd(const Dev& p, glbd* z, const double* dbuf_, const double* x0_, const FuseArg& fa,
                           ldsd* scr, Prologue& pl) {
    const Geo<NXc, NUc> g(p);
    const TabSize<NXc, NUc> ts(g);
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int s = fa.s, T = fa.T, nb = fa.nb, c1 = fa.c1, p1 = fa.p1;
    const int oKM = 0, oF = oKM + c1 * ts.KM1, oXD = oF + (FL ? p1 * ts.F1 : 0), oNL = oXD + T * g.KF, oCH = oNL + 2 * T;
    int rot = p.dyn_rot ? 0 : -1;
    dma_r(scr + oKM, p.dKM, c1 * ts.KM1, rot);
    if (FL) dma_r(scr + oF, p.dF, p1 * ts.F1, rot);
    dma_r(scr + oNL, (const double*)p.ninfo, 2 * T, rot);
    dma_r(scr + oCH, (const double*)(p.cinfo + 1), 2 * (T + nb - 1), rot);
    if (tid <= s + 1) pl.sp[tid] = p.stage_ptr[tid];
    for (int e = tid; e < T * g.KF; e += nthr) {  // [x0 (row 0) or 0 | d | 0]
        const int i = e / g.KF, c = e - i * g.KF;
        double v = 0.0;
        if (c < g.nx) v = i == 0 ? ((const glbd*)x0_)[c] : 0.0;
        else if (c < g.nx + g.nu) v = ((const glbd*)dbuf_)[(size_t)i * g.nu + c - g.nx];
        scr[oXD + e] = v;
    }
    if (tid < g.nx) z[p.X0 + tid] = ((const glbd*)x0_)[tid];  // x_0 = x0bar (cache.py:282)
    dma_wait();
    lds_sync();
    typedef typename std::conditional<FL, const ldsd*, const glbd*>::type PF;
    const TabsT<const ldsd*, PF> tb{nullptr, nullptr, scr + oKM, FL ? (PF)(scr + oF) : (PF)((const glbd*)p.dF), 0, 0};
    const InfoT<const ldsrec*> inf{(const ldsrec*)(scr + oNL), 0, (const ldsrec*)(scr + oCH), 1};
    const LRows xd{scr + oXD, 0, g.KF};
    for (int t = 0; t < s; ++t) {
        const int b = pl.sp[t], e = pl.sp[t + 1];
        if (t + 1 < s) fwd_phase<NXc, NUc, true>(p, tb, inf, b, e, xd, z, xd, tid, nthr);
        else fwd_phase<NXc, NUc, false, true>(p, tb, inf, b, e, xd, z, xd, tid, nthr);
        lds_sync();
    }
}

// a tier's XD rows for the forward sweep: [0 | d (global rows) | 0]; the root's x arrives later
template <int NXc, int NUc>
__device__ void fz_xd_stage(const Dev& p, const double* dbuf_, const FuseTier& tt, int sub, ldsd* XD) {
    const Geo<NXc, NUc> g(p);
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int L = tt.s1 - tt.s0;
    const bool dmaok = (g.nx % 2 == 0) && (g.nu % 2 == 0);
    const double* zp = p.zpage;
    for (int l = 0, off = 0; l < L; ++l) {
        const int lo = fz_lo(tt.ta, l, sub), cnt = tt.ta.cnt[l];
        ldsd* xd = XD + (size_t)off * g.KF;
        const double* dl = dbuf_ + (size_t)lo * g.nu;
        if (dmaok) {
            const int cpr = g.KF >> 1, cx = g.nx >> 1, cd = (g.nx + g.nu) >> 1;
            dma_gen(xd, cnt * cpr, [=](int ch) {
                const int r = ch / cpr, c = ch - r * cpr;
                return (c >= cx && c < cd) ? dl + (size_t)r * g.nu + 2 * (c - cx) : zp;
            });
        } else {
            for (int e = tid; e < cnt * g.KF; e += nthr) {
                const int r = e / g.KF, c = e - r * g.KF;
                xd[e] = (c >= g.nx && c < g.nx + g.nu) ? ((const glbd*)dl)[(size_t)r * g.nu + c - g.nx] : 0.0;
            }
        }
        off += cnt;
    }
}

template <int NXc, int NUc, bool FL>
__global__ void __launch_bounds__(kFuseBlock) k_dyn_down(Dev p, Bufs bf, const Ctl* ctl, int zsel,
                                                         const double* dbuf_, const double* x0_, FuseArg fa) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ Prologue pl;
    __shared__ int s_ok;
    const int tid = threadIdx.x;
    if (ld_u32_sc1((const unsigned*)fa.err)) return;  // an earlier hand-off timed out: the host resets
    ldsd* smem = (ldsd*)smem_;
    glbd* z = dyn_z(bf, zsel, ctl);
    if (tid == 0) {
        pl.nts = 0;
        s_ok = 1;
    }
    fz_stamp(p, pl);
    const int D = fa.K - 1;
    if (blockIdx.x == 0) {  // the top
        const unsigned tag = ld_u32_sc1(fa.epoch);
        if (!ctl_done(ctl)) fz_top_fwd<NXc, NUc, FL>(p, z, dbuf_, x0_, fa, smem, pl);
        fz_stamp(p, pl);
        fz_release_store(fa.t[0].flag, tag);
        if (kDiag && p.stamps && tid == 0)
            for (int q = 0; q < pl.nts && q < 64; ++q) p.stamps[q] = pl.ts[q];
        return;
    }
    int b = (int)blockIdx.x - 1, k = 0;
    for (; k < D && b >= fa.t[k].ngroups * fa.t[k].r; ++k) b -= fa.t[k].ngroups * fa.t[k].r;
    const FuseTier& tt = fa.t[k];
    // [XD (nnl, KF) | KM | F | NL | CH]
    ldsd* XD = smem;
    ldsd* scr = smem + rup(tt.nnl * Geo<NXc, NUc>(p).KF, 2);
    const bool work = !ctl_done(ctl);
    if (work) {
        fz_fwd_stage<NXc, NUc>(p, tt, b, scr);
        fz_xd_stage<NXc, NUc>(p, dbuf_, tt, b, XD);
    }
    const unsigned tag = ld_u32_sc1(fa.epoch);
    if (!fz_wait_eq(tt.flag + b / tt.r, tag, fa, s_ok)) return;
    fz_stamp(p, pl);
    if (work) fz_fwd_run<NXc, NUc>(p, z, tt, b, k < D, XD, scr, pl);
    fz_stamp(p, pl);
    if (k < D) {
        fz_release_store(fa.t[k + 1].flag + b, tag);
    }
    if (kDiag && p.stamps && tid == 0 && b == 0)  // diagnostics: tier 0 / deepest, subtree 0
        for (int q = 0; q < pl.nts && q < 64; ++q) p.stamps[(k == 0 ? 64 : 128) + q] = pl.ts[q];
}
