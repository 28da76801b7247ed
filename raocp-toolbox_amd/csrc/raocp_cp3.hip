// raocp_cp3.hip — one Chambolle–Pock iteration after the dynamics sweep as ONE streaming
// kernel (included by raocp_kernels.hip after raocp_ell3.hip, namespace raocp):
//
//   dual half step + prox of g*        (solver.py:44-61, cache.py:321-393)
//   next primal half step + s_0 relax + AVaR kernel projection (solver.py:27-39, cache.py:248-317)
//   the finished iteration's residuals xi0, xi1, xi2, delta0, delta1, delta2 (solver.py:63-95)
//
// for trees with one branching factor C (children of parent i: 1 + C i .. C i + C, y_i at
// (2C + 1) i) and one sqrtQ / sqrtR table over the children and one sqrtPf over the leaves
// (host checks, raocp_capi.hip). A FAMILY (parent i and its C children) holds everything
// the iteration couples: L's child rows eta3..eta6 read only x_i, u_i; L^T's x_i, u_i read
// only eta7_i and the children's eta3 / eta4; the kernel projection couples y_i with the
// children's tau / s. So a wave takes tiles of 16 consecutive parents (a grid-stride loop,
// no table, no LDS staging, no block barrier) and finishes the whole iteration on them:
//
//   phase 1  parent rows: L products sqrtQ (2x+ - p), sqrtQ (x+ - p) (and sqrtR on u) as MFMA
//            tiles; eta7 (box), eta1 / eta2 (AVaR cone) and their L^T terms on y
//   phase 2  per child slot k: the SOC of (eta3, eta4, eta5 | eta6), eta+ / xi2 in registers,
//            (eta+, d - eta+, xi2) of the children summed per parent
//   phase 3  eta7 (box) and x_i, u_i of the next half step with their residuals: L^T of the
//            summed child rows (one sqrtQ over the children) as a second MFMA chain
//   phase 4  (parents of leaves, run first) per leaf slot: the leaf SOC (eta11, eta12 | eta13),
//            eta14 box, and the leaf's x row of the next half step (sqrtPf MFMA chains)
//   phase 5  s_j of the children (eta2_j of a nonleaf child recomputed here, bit-identical
//            to its own tile's), then the closed-form AVaR kernel projection of the family
//
// xi2 never leaves the registers: the reference's L^T xi2 (solver.py:85-92) is formed from
// the same values the dual step produced, so the iteration moves 3|P| + 2|D| scalars
// (p, z+, d in; eta+, next half step out) instead of the 5|P| + 6|D| of k_cpd2 + k_cpp2.
//
// Products in the transposed form: D = W V with the weights W (16 x 4 per k-step) as the A
// operand and the node vectors V as the B operand (lane lo = node), so the accumulator of
// the L product (rows on the lane groups and registers, node on lo) is already the B
// operand of the L^T product (no transpose, no LDS). "Row layout" of an R-row vector
// (R = 4 KC): lane (lo, h = lane >> 4) holds the KC consecutive rows KC h .. KC h + KC - 1
// of node lo, slot t = 4 rt + e (register e of row tile rt) holding row KC h + t (t < KC;
// zero above). In every operand and accumulator: the k index of k-step s is KC h + s, so a
// lane's B values are consecutive entries of its node (16-B vector loads and stores where
// KC is a multiple of 4), and the A rows are permuted (MFA<T>::rows) so that the f64
// accumulator map (row h + 4 e) and the f32 one (4 h + e) both land row KC h + 4 rt + e in
// slot (rt, e). A product then takes ceil(KC_out / 4) x KC_in MFMAs: no k-step is padding
// (nx = 20: 2 x 5, against 2 x 8 with 16-row tiles).

// A row lo of an output row tile lands in lane group g, register e of the accumulator
template <class T>
struct MFA;
template <>
struct MFA<double> {  // D row = h + 4 e
    static __device__ __forceinline__ int g_of(int lo) { return lo & 3; }
    static __device__ __forceinline__ int e_of(int lo) { return lo >> 2; }
};
template <>
struct MFA<float> {  // D row = 4 h + e
    static __device__ __forceinline__ int g_of(int lo) { return lo >> 2; }
    static __device__ __forceinline__ int e_of(int lo) { return lo & 3; }
};
// the weight row A row lo of output row tile ro carries for an R-row output (-1: padding)
template <class T, int R>
__device__ __forceinline__ int wrow(int ro, int lo) {
    constexpr int KC = R / 4;
    const int t = 4 * ro + MFA<T>::e_of(lo);
    return t < KC ? KC * MFA<T>::g_of(lo) + t : -1;
}

// weight fragments of one R x K table (column-major M[k R + r]) in the transposed form,
// staged once per workgroup in LDS (registers are the scarce resource of this kernel: the
// per-parent L products and three L^T accumulators stay live over the child slots):
// lds[(ro KS + s) 64 + lane] = M[wrow(ro, lo)][K/4 h + s]
template <class T, int R, int K>
struct WL {
    static_assert(R % 4 == 0 && K % 4 == 0, "row layout: R, K multiples of 4");
    static constexpr int RO = (R / 4 + 3) / 4, KS = K / 4, N = RO * KS * 64;
    const __attribute__((address_space(3))) T* base;
    __device__ __forceinline__ T get(int ro, int s) const { return base[(ro * KS + s) * 64 + (threadIdx.x & 63)]; }
    // every thread of the workgroup takes part (a __syncthreads follows)
    template <class DP>
    static __device__ __forceinline__ void fill(DP dst, const T* tab, int t) {
        cglbp<T> M = (cglbp<T>)(tab + (size_t)t * R * K);
        for (int q = threadIdx.x; q < N; q += blockDim.x) {
            const int l = q & 63, lo = l & 15, h = l >> 4, s = (q >> 6) % KS, ro = (q >> 6) / KS;
            const int r = wrow<T, R>(ro, lo), k = KS * h + s;
            dst[q] = r >= 0 ? M[k * R + r] : T(0);
        }
    }
};

// acc[ro] += W b (b in row layout over K)
template <class T, int R, int K>
__device__ __forceinline__ void mmt(const WL<T, R, K>& W, const T (&b)[(K + 15) / 16][4],
                                    typename MF<T>::v4 (&acc)[(R + 15) / 16]) {
    _Pragma("unroll") for (int s = 0; s < WL<T, R, K>::KS; ++s)
        _Pragma("unroll") for (int ro = 0; ro < WL<T, R, K>::RO; ++ro)
            acc[ro] = MF<T>::mma(W.get(ro, s), b[s >> 2][s & 3], acc[ro]);
}

// 4 consecutive T at 4- / 8-B alignment (node rows start wherever the flat layout puts them)
template <class T>
struct V4a {
    typedef T type __attribute__((ext_vector_type(4), aligned(sizeof(T))));
};

// slot (rt, e) of an R-row vector holds a row (t = 4 rt + e < R / 4)
template <int R>
__device__ __forceinline__ constexpr bool tok(int rt, int e) {
    return 4 * rt + e < R / 4;
}
// row-layout load of an R-row node vector: a[rt][e] = v[R/4 h + 4 rt + e] (0 past R/4)
template <class T, int R>
__device__ __forceinline__ void ld_rows(cglbp<T> v, bool live, T (&a)[(R + 15) / 16][4]) {
    typedef typename V4a<T>::type vt;
    constexpr int KC = R / 4;
    cglbp<T> b = v + KC * ((threadIdx.x & 63) >> 4);
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) {
        if (live && 4 * rt + 3 < KC) {
            const vt w = *(const __attribute__((address_space(1))) vt*)(b + 4 * rt);
            _Pragma("unroll") for (int e = 0; e < 4; ++e) a[rt][e] = w[e];
        } else {
            _Pragma("unroll") for (int e = 0; e < 4; ++e) a[rt][e] = (live && tok<R>(rt, e)) ? b[4 * rt + e] : T(0);
        }
    }
}
template <class T, int R>
__device__ __forceinline__ void st_rows(glbp<T> v, bool live, const T (&a)[(R + 15) / 16][4]) {
    typedef typename V4a<T>::type vt;
    constexpr int KC = R / 4;
    glbp<T> b = v + KC * ((threadIdx.x & 63) >> 4);
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) {
        if (!live) continue;
        if (4 * rt + 3 < KC) {
            vt w;
            _Pragma("unroll") for (int e = 0; e < 4; ++e) w[e] = a[rt][e];
            *(__attribute__((address_space(1))) vt*)(b + 4 * rt) = w;
        } else {
            _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<R>(rt, e)) b[4 * rt + e] = a[rt][e];
        }
    }
}

// sum over the 4 lane groups (the rows of one node)
template <class T>
__device__ __forceinline__ T sum_h(T v) {
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    return v;
}

// per-wave scratch of the kernel projection: the family's y (2C + 1 <= 9) and the
// children's tau, s after the L^T half step (phase 5 reads them across lane groups)
template <class T>
struct KpScratch {
    T y[16][9];
    T tau[16][4];
    T s[16][4];
};

// the inputs of one child slot (child block rows of d, tau of z+ and p) and of one leaf slot
template <class T, int NX, int NU>
struct ChildIn {
    T d3[(NX + 15) / 16][4], d4[(NU + 15) / 16][4];
    T d5, d6, tz, tp;
    __device__ __forceinline__ void load(const Dev& p, cglbp<T> zp, cglbp<T> pz, cglbp<T> d, int j, bool live) {
        ld_rows<T, NX>(d + e3(p, live ? j : 1), live, d3);
        ld_rows<T, NU>(d + e4(p, live ? j : 1), live, d4);
        d5 = live ? d[p.E5 + j] : T(0);
        d6 = live ? d[p.E6 + j] : T(0);
        tz = live ? zp[p.T0 + j] : T(0);
        tp = live ? pz[p.T0 + j] : T(0);
    }
};
template <class T, int NX>
struct LeafIn {
    T lz[(NX + 15) / 16][4], lp[(NX + 15) / 16][4], d11[(NX + 15) / 16][4], d14[(NX + 15) / 16][4];
    T d12, d13, sz, sp;
    int o14;
    __device__ __forceinline__ void load(const Dev& p, cglbp<T> zp, cglbp<T> pz, cglbp<T> d, int l, bool live, int bx,
                                         int m, bool box) {
        ld_rows<T, NX>(zp + p.X0 + (size_t)(live ? l : 0) * NX, live, lz);
        ld_rows<T, NX>(pz + p.X0 + (size_t)(live ? l : 0) * NX, live, lp);
        ld_rows<T, NX>(d + e11(p, live ? l : m), live, d11);
        o14 = live && box ? o14_of<NX>(p, l, bx) : -1;
        ld_rows<T, NX>(d + (o14 >= 0 ? o14 : 0), o14 >= 0, d14);
        d12 = live ? d[p.E12 + l] : T(0);
        d13 = live ? d[p.E13 + l] : T(0);
        sz = live ? zp[p.S0 + l] : T(0);
        sp = live ? pz[p.S0 + l] : T(0);
    }
};

// The task list of a launch (host-built, raocp_capi.hip cp3_tasks): tiles of 16 leaves
// [l0, l1) when the leaves run as tasks of their own (split), then tiles of 16 parents from
// the start of each parent range [lo[r], hi[r]). Unsharded: the leaf parents, then the rest.
// A shard launches its own families and leaves plus the
// replicated top above the cut's parents, then -- after X1 -- the cut's parents, whose
// children's eta2 entries (eta+, xi2) come from the buffers the exchange filled (ext2)
// instead of being recomputed from rows another shard owns; the first launch stores xi2 of
// its roots' eta2 (parents [xlo, xhi)) for X1.
// (kCp3MaxR and Cp3Tasks: raocp_common.h, shared with raocp_cp4.hip)

// The weight fragments of the launch ([sqrtQ | sqrtR | sqrtPf] in LDS order), laid out once
// per context: every workgroup copies them by LDS-DMA (one memory round trip in front of its
// first task; the element-wise gather it replaces sat there too)
template <class T, int NX, int NU>
__global__ void __launch_bounds__(256) k_cp3_image(Dev p, double* img) {
    typedef WL<T, NX, NX> WQ;
    typedef WL<T, NU, NU> WR;
    glbp<T> w = (glbp<T>)img;
    WQ::fill(w, (const T*)p.SQ, p.crec[1].y);  // one table over the children (host check)
    WR::fill(w + WQ::N, (const T*)p.SR, p.crec[1].z);
    WQ::fill(w + WQ::N + WR::N, (const T*)p.SP, p.lrec[0].x);  // one over the leaves
}

// SH: a shard's launches (the xi2 store and ext2 paths compiled in; the unsharded kernel
// keeps its registers)
template <class T, int NX, int NU, bool SH>
__global__ void __launch_bounds__(256) k_cp3(Dev p, Ctl* __restrict__ ctl, Bufs bf, double* __restrict__ part,
                                             double* __restrict__ xi2_, int C, int bx, Cp3Tasks tk,
                                             const double* __restrict__ img) {
    typedef typename MF<T>::v4 v4;
    static_assert(NX % 4 == 0 && NU % 4 == 0, "row layout needs nx, nu multiples of 4");
    constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16;
    typedef WL<T, NX, NX> WQ;
    typedef WL<T, NU, NU> WR;
    __shared__ KpScratch<T> kps_[4];
    __shared__ double s_red[6][4];
    __shared__ __attribute__((aligned(16))) T wlds_[2 * WQ::N + WR::N];
    const int m = p.m;
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4, wv = threadIdx.x >> 6;
    const int gw = blockIdx.x * (blockDim.x >> 6) + wv, nwv = gridDim.x * (blockDim.x >> 6);
    typedef __attribute__((address_space(3))) KpScratch<T> lkps;
    lkps& ks = *(lkps*)&kps_[wv];
    cglbp<T> pz = (cglbp<T>)bf.z0;  // p
    cglbp<T> zp = (cglbp<T>)bf.z1;  // z+
    glbp<T> out = (glbp<T>)bf.z2;   // next half step
    cglbp<T> d = (cglbp<T>)bf.e0;   // eta
    glbp<T> eo = (glbp<T>)bf.e1;    // eta+
    cglbp<T> cond = (cglbp<T>)p.cond;
    double m0 = 0.0, m1 = 0.0, m2 = 0.0, m3 = 0.0, m4 = 0.0, m5 = 0.0;
    typedef __attribute__((address_space(3))) T lT;
    lT* wl = (lT*)wlds_;
    dma((ldsd*)wlds_, img, (2 * WQ::N + WR::N) * (int)sizeof(T) / 8);  // k_cp3_image (N: multiples of 64)
    const int done = ctl->done;
    const T alpha = (T)ctl->alpha, ra = T(1) / alpha;
    dma_wait();
    __syncthreads();
    if (done) return;  // uniform over the grid
    const WQ wq{wl};
    const WR wr{wl + WQ::N};
    const WQ wp{wl + WQ::N + WR::N};
    // one dual element: eta+ = alpha (v - Pi(v)), xi2 = (d - eta+) / alpha + L(z+ - p)
    auto fin = [&](T dv, T v, T pv, T b, T& ep, T& x2) {
        ep = alpha * (v - pv);
        x2 = (dv - ep) * ra + b;
        m2 = nmax(m2, (double)fabs(x2));
        m5 = nmax(m5, (double)fabs(ep - dv));
    };
    // the residual terms of one primal entry: pp = p, zz = z+, w = L^T(d - eta+), lc = L^T xi2
    auto account = [&](T pp, T zz, T w, T lc) {
        const T x1 = (pp - zz) * ra - w;
        const T x0v = x1 + lc;
        const T dl1 = zz - pp;
        const T dl0 = dl1 + w;
        m0 = nmax(m0, (double)fabs(x0v));
        m1 = nmax(m1, (double)fabs(x1));
        m3 = nmax(m3, (double)fabs(dl0));
        m4 = nmax(m4, (double)fabs(dl1));
    };
    // one leaf l (lane lo) of a slot k: full = the whole leaf (eta11..eta14 and x_l of the half
    // step), else only its SOC scalars; pside = the parent's side (s_l of the half step into
    // the kernel projection's scratch, and its residual terms)
    auto leaf_work = [&](const LeafIn<T, NX>& cur, int l, int k, bool live, bool full, bool pside) {
        const T (&lz)[RX][4] = cur.lz;
        const T (&lp)[RX][4] = cur.lp;
        const T (&d11)[RX][4] = cur.d11;
        const T (&d14)[RX][4] = cur.d14;
        const int o14 = cur.o14;
        const T d12 = cur.d12, d13 = cur.d13, sz = cur.sz, sp = cur.sp;
            v4 la[RX], lb[RX];
            {
                T a1[RX][4], a2[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    a1[rt][e] = T(2) * lz[rt][e] - lp[rt][e];
                    a2[rt][e] = lz[rt][e] - lp[rt][e];
                }
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) la[rt] = lb[rt] = v4{0, 0, 0, 0};
                mmt(wp, a1, la);
                if (full) mmt(wp, a2, lb);
            }
            T v11[RX][4];
            T ss = T(0);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                v11[rt][e] = (d11[rt][e] + alpha * la[rt][e]) * ra;
                if (tok<NX>(rt, e)) ss += v11[rt][e] * v11[rt][e];
            }
            ss = sum_h(ss);
            const T a5 = T(0.5) * (T(2) * sz - sp), b5 = T(0.5) * (sz - sp);
            const T v12 = (d12 + alpha * a5) * ra + T(-0.5);
            const T v13 = (d13 + alpha * a5) * ra + T(0.5);
            ss += v12 * v12;
            const T nf = sqrt(ss), tt = v13;
            T ep12, x212, ep13, x213;
            fin(d12, v12, soc_apply_t(v12, false, nf, tt), b5, ep12, x212);
            fin(d13, v13, soc_apply_t(v13, true, nf, tt), b5, ep13, x213);
            if (pside && live && h == 0) {
                ks.s[lo][k] = sz - alpha * (T(0.5) * (ep12 + ep13));
                account(sp, sz, T(0.5) * ((d12 - ep12) + (d13 - ep13)), T(0.5) * (x212 + x213));
            }
            if (!full) return;
            if (live && h == 0) eo[p.E12 + l] = ep12;
            if (live && h == 1) eo[p.E13 + l] = ep13;
            T eA[RX][4], eW[RX][4], eC[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                T ep = T(0), x2 = T(0);
                if (live && tok<NX>(rt, e))
                    fin(d11[rt][e], v11[rt][e], soc_apply_t(v11[rt][e], false, nf, tt), lb[rt][e], ep, x2);
                eA[rt][e] = ep;
                eW[rt][e] = d11[rt][e] - ep;
                eC[rt][e] = x2;
            }
            st_rows<T, NX>(eo + e11(p, live ? l : m), live, eA);
            v4 gA[RX], gW[RX], gC[RX];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) gA[rt] = gW[rt] = gC[rt] = v4{0, 0, 0, 0};
            mmt(wp, eA, gA);
            mmt(wp, eW, gW);
            mmt(wp, eC, gC);
            // eta14 = x_l (box) and x_l = sqrtPf eta11 + eta14 (operators.py:86-94)
            if (o14 >= 0) {
                const int bl = p.iBl[l];
                T l14[RX][4], h14[RX][4], e14[RX][4];
                ld_rows<T, NX>((cglbp<T>)p.blo_l + (size_t)bl * NX, true, l14);
                ld_rows<T, NX>((cglbp<T>)p.bhi_l + (size_t)bl * NX, true, h14);
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NX>(rt, e)) {
                        const T v = (d14[rt][e] + alpha * (T(2) * lz[rt][e] - lp[rt][e])) * ra;
                        fin(d14[rt][e], v, box_apply_t(v, l14[rt][e], h14[rt][e], ctl), lz[rt][e] - lp[rt][e], ep, x2);
                    }
                    e14[rt][e] = ep;
                    gA[rt][e] += ep;
                    gW[rt][e] += d14[rt][e] - ep;
                    gC[rt][e] += x2;
                }
                st_rows<T, NX>(eo + o14, true, e14);
            }
            T ox[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                ox[rt][e] = lz[rt][e] - alpha * gA[rt][e];
                if (live && tok<NX>(rt, e)) account(lp[rt][e], lz[rt][e], gW[rt][e], gC[rt][e]);
            }
            st_rows<T, NX>(out + p.X0 + (size_t)(live ? l : 0) * NX, live, ox);
    };
    const int G = 2 * C + 1;
    glbp<T> xi2 = (glbp<T>)xi2_;
    const int split = tk.split;
    const int nTL = (tk.l1 - tk.l0 + 15) >> 4;  // leaf tiles (split), then the parent ranges' tiles
    for (int tt = gw; tt < nTL + tk.t0[tk.nr]; tt += nwv) {
        if (tt < nTL) {
            // a tile of 16 consecutive leaves (split): everything of the leaf but s_l
            const int l = tk.l0 + 16 * tt + lo;
            const bool live = l < tk.l1;
            LeafIn<T, NX> cur;
            cur.load(p, zp, pz, d, l, live, bx, m, true);
            leaf_work(cur, l, 0, live, true, false);
            continue;
        }
        const int task = tt - nTL;
        int r = 0;
        while (r + 1 < tk.nr && task >= tk.t0[r + 1]) ++r;
        const int i0 = tk.lo[r] + 16 * (task - tk.t0[r]), iend = tk.hi[r];
        const bool leafp = tk.lo[r] >= tk.mL;
        const int i = i0 + lo;
        const bool live = i < iend;
        // ---------------- phase 4 (first, on parents of leaves): leaf children (leaf SOC, eta14
        // box, x_l of the half step); their s_l goes to the kernel projection's scratch. The
        // next slot's rows are loaded before the current slot's arithmetic (vmcnt in order).
        // split: the leaves are tasks of their own, the family computes only their SOC scalars
        if (leafp) {
            LeafIn<T, NX> cur, nxt;
            cur.load(p, zp, pz, d, 1 + C * i, live, bx, m, !split);
            for (int k = 0; k < C; ++k) {
                const int l = 1 + C * i + k;
                if (k + 1 < C) nxt.load(p, zp, pz, d, l + 1, live, bx, m, !split);
                leaf_work(cur, l, k, live, !split, true);
                if (k + 1 < C) cur = nxt;
            }
        }
        // ---------------- phase 1: the parent's rows (child slot 0's rows in flight meanwhile)
        ChildIn<T, NX, NU> ccu, cnx;
        ccu.load(p, zp, pz, d, 1 + C * i, live);
        const int o7 = live ? o7_of<NX, NU>(p, i, bx) : -1;
        // eta2_i and the y entries: every lane group loads the C + 1 entries b' y reads
        const int yo = G * i;
        T bya = T(0), byb = T(0);
        if (live) {
            for (int k = 0; k < C; ++k) {
                const T cp = cond[1 + C * i + k], zy = zp[p.Y0 + yo + k], py = pz[p.Y0 + yo + k];
                bya = fma(cp, T(2) * zy - py, bya);
                byb = fma(cp, zy - py, byb);
            }
            const T zy = zp[p.Y0 + yo + 2 * C], py = pz[p.Y0 + yo + 2 * C];
            bya += T(2) * zy - py;
            byb += zy - py;
        }
        const T zs = live ? zp[p.S0 + i] : T(0), ps = live ? pz[p.S0 + i] : T(0);
        const T d2 = live ? d[p.E2 + i] : T(0);
        T e2A, e2C;
        {
            const T av = (T(2) * zs - ps) - bya, bb = (zs - ps) - byb;
            const T v = (d2 + alpha * av) * ra;
            T x2;
            fin(d2, v, fmax(v, T(0)), bb, e2A, x2);
            e2C = x2;
            if (live && h == 0) eo[p.E2 + i] = e2A;
            if (SH && live && h == 1 && i >= tk.xlo && i < tk.xhi) xi2[p.E2 + i] = x2;  // a shard's roots (X1)
        }
        const T e2W = d2 - e2A;
        if (live && i == 0 && h == 0) {
            // root s_0: L^T -> eta2_0, then the relaxation prox s_0 -= alpha (cache.py:253-257)
            out[p.S0] = (zs - alpha * e2A) - alpha;
            account(ps, zs, e2W, e2C);
        }
        // eta1_i = y_i rows (lane group h: entries h, h + 4, h + 8) and y of the half step
        for (int q = h; q < G; q += 4) {
            if (!live) break;
            const T zy = zp[p.Y0 + yo + q], py = pz[p.Y0 + yo + q], dv = d[p.E1 + yo + q];
            const T av = T(2) * zy - py, bb = zy - py;
            const T v = (dv + alpha * av) * ra;
            T ep, x2;
            fin(dv, v, q < 2 * C ? fmax(v, T(0)) : v, bb, ep, x2);
            eo[p.E1 + yo + q] = ep;
            const T b = q < C ? cond[1 + C * i + q] : q < 2 * C ? T(0) : T(1);
            ks.y[lo][q] = zy - alpha * (ep - b * e2A);
            account(py, zy, (dv - ep) - b * e2W, x2 - b * e2C);
        }
        // L products of the parent: a = L(2z+ - p), b = L(z+ - p) on the children's rows
        v4 qa[RX], qb[RX], ua[RU], ub[RU];
        {
            // the parent's x, u rows (reloaded in phase 3: registers, not HBM, are short here)
            T xz[RX][4], xp[RX][4], uz[RU][4], up[RU][4];
            ld_rows<T, NX>(zp + p.X0 + (size_t)i * NX, live, xz);
            ld_rows<T, NX>(pz + p.X0 + (size_t)i * NX, live, xp);
            ld_rows<T, NU>(zp + p.U0 + (size_t)i * NU, live, uz);
            ld_rows<T, NU>(pz + p.U0 + (size_t)i * NU, live, up);
            T a1[RX][4], a2[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                a1[rt][e] = T(2) * xz[rt][e] - xp[rt][e];
                a2[rt][e] = xz[rt][e] - xp[rt][e];
            }
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) qa[rt] = qb[rt] = v4{0, 0, 0, 0};
            mmt(wq, a1, qa);
            mmt(wq, a2, qb);
            T c1[RU][4], c2[RU][4];
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                c1[rt][e] = T(2) * uz[rt][e] - up[rt][e];
                c2[rt][e] = uz[rt][e] - up[rt][e];
            }
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) ua[rt] = ub[rt] = v4{0, 0, 0, 0};
            mmt(wr, c1, ua);
            mmt(wr, c2, ub);
        }
        // the children's (eta+, d - eta+, xi2) eta3 / eta4 rows summed per parent in registers:
        // with one sqrtQ / sqrtR over the children, L^T's sum over them is one product of the
        // summed rows (one MFMA chain per stream and family instead of one per child)
        T sxA[RX][4], sxW[RX][4], sxC[RX][4], suA[RU][4], suW[RU][4], suC[RU][4];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
            sxA[rt][e] = sxW[rt][e] = sxC[rt][e] = T(0);
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
            suA[rt][e] = suW[rt][e] = suC[rt][e] = T(0);
        // ---------------- phase 2: child slots (child block SOC, L^T accumulation), the next
        // slot's rows loaded before the current slot's arithmetic
        for (int k = 0; k < C; ++k) {
            const int j = 1 + C * i + k;
            if (k + 1 < C) cnx.load(p, zp, pz, d, j + 1, live);
            T (&d3)[RX][4] = ccu.d3;
            T (&d4)[RU][4] = ccu.d4;
            const T d5 = ccu.d5, d6 = ccu.d6, tz = ccu.tz, tp = ccu.tp;
            T v3[RX][4], v4_[RU][4];
            T ss = T(0);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                v3[rt][e] = (d3[rt][e] + alpha * qa[rt][e]) * ra;
                if (tok<NX>(rt, e)) ss += v3[rt][e] * v3[rt][e];
            }
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                v4_[rt][e] = (d4[rt][e] + alpha * ua[rt][e]) * ra;
                if (tok<NU>(rt, e)) ss += v4_[rt][e] * v4_[rt][e];
            }
            ss = sum_h(ss);
            const T a5 = T(0.5) * (T(2) * tz - tp), b5 = T(0.5) * (tz - tp);
            const T v5 = (d5 + alpha * a5) * ra + T(-0.5);
            const T v6 = (d6 + alpha * a5) * ra + T(0.5);
            ss += v5 * v5;
            const T nf = sqrt(ss), tt = v6;
            // eta+ / (d - eta+) / xi2 of eta3 and eta4 in row layout: the L^T B operands
            T e3A[RX][4], e3W[RX][4], e3C[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                T ep = T(0), x2 = T(0);
                if (live && tok<NX>(rt, e))
                    fin(d3[rt][e], v3[rt][e], soc_apply_t(v3[rt][e], false, nf, tt), qb[rt][e], ep, x2);
                e3A[rt][e] = ep;
                e3W[rt][e] = d3[rt][e] - ep;
                e3C[rt][e] = x2;
            }
            st_rows<T, NX>(eo + e3(p, live ? j : 1), live, e3A);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                sxA[rt][e] += e3A[rt][e];
                sxW[rt][e] += e3W[rt][e];
                sxC[rt][e] += e3C[rt][e];
            }
            T e4A[RU][4], e4W[RU][4], e4C[RU][4];
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                T ep = T(0), x2 = T(0);
                if (live && tok<NU>(rt, e))
                    fin(d4[rt][e], v4_[rt][e], soc_apply_t(v4_[rt][e], false, nf, tt), ub[rt][e], ep, x2);
                e4A[rt][e] = ep;
                e4W[rt][e] = d4[rt][e] - ep;
                e4C[rt][e] = x2;
            }
            st_rows<T, NU>(eo + e4(p, live ? j : 1), live, e4A);
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                suA[rt][e] += e4A[rt][e];
                suW[rt][e] += e4W[rt][e];
                suC[rt][e] += e4C[rt][e];
            }
            // eta5 / eta6 and tau_j of the half step (before the kernel projection)
            T ep5, x25, ep6, x26;
            fin(d5, v5, soc_apply_t(v5, false, nf, tt), b5, ep5, x25);
            fin(d6, v6, soc_apply_t(v6, true, nf, tt), b5, ep6, x26);
            if (live && h == 0) eo[p.E5 + j] = ep5;
            if (live && h == 1) eo[p.E6 + j] = ep6;
            if (live && h == 0) {
                const T ltt = T(0.5) * (ep5 + ep6);
                ks.tau[lo][k] = tz - alpha * ltt;
                account(tp, tz, T(0.5) * ((d5 - ep5) + (d6 - ep6)), T(0.5) * (x25 + x26));
            }
            if (!leafp && live && h == 0) {
                // s_j of a nonleaf child: its eta2 recomputed (the same arithmetic as its own
                // tile's, phase 1) or, across a shard boundary, as X1 delivered it; then the
                // half step
                const T sz = zp[p.S0 + j], sp = pz[p.S0 + j], dj = d[p.E2 + j];
                T ep, x2;
                if (SH && tk.ext2) {
                    ep = eo[p.E2 + j];
                    x2 = xi2[p.E2 + j];
                } else {
                    const int yj = G * j;
                    T ba = T(0), bb2 = T(0);
                    for (int q = 0; q < C; ++q) {
                        const T cp = cond[1 + C * j + q], zy = zp[p.Y0 + yj + q], py = pz[p.Y0 + yj + q];
                        ba = fma(cp, T(2) * zy - py, ba);
                        bb2 = fma(cp, zy - py, bb2);
                    }
                    const T zy = zp[p.Y0 + yj + 2 * C], py = pz[p.Y0 + yj + 2 * C];
                    ba += T(2) * zy - py;
                    bb2 += zy - py;
                    const T av = (T(2) * sz - sp) - ba, bb = (sz - sp) - bb2;
                    const T v = (dj + alpha * av) * ra;
                    ep = alpha * (v - fmax(v, T(0)));
                    x2 = (dj - ep) * ra + bb;
                }
                ks.s[lo][k] = sz - alpha * ep;
                account(sp, sz, dj - ep, x2);
            }
            if (k + 1 < C) ccu = cnx;
        }
        // ---------------- phase 3: eta7 (box on [x_i; u_i]) and x_i, u_i of the half step:
        // L^T = Gamma' eta7 + sqrtQ (sum of the children's eta3) (operators.py:73-85)
        {
            T xz[RX][4], xp[RX][4], uz[RU][4], up[RU][4];
            ld_rows<T, NX>(zp + p.X0 + (size_t)i * NX, live, xz);
            ld_rows<T, NX>(pz + p.X0 + (size_t)i * NX, live, xp);
            ld_rows<T, NU>(zp + p.U0 + (size_t)i * NU, live, uz);
            ld_rows<T, NU>(pz + p.U0 + (size_t)i * NU, live, up);
            T d7x[RX][4], d7u[RU][4];
            ld_rows<T, NX>(d + (o7 >= 0 ? o7 : 0), o7 >= 0, d7x);
            ld_rows<T, NU>(d + (o7 >= 0 ? o7 + NX : 0), o7 >= 0, d7u);
            const int bi = o7 >= 0 ? p.iBnl[i] : 0;
            cglbp<T> blo = (cglbp<T>)p.blo_nl + (size_t)bi * (NX + NU), bhi = (cglbp<T>)p.bhi_nl + (size_t)bi * (NX + NU);
            v4 gxA[RX], gxW[RX], gxC[RX], guA[RU], guW[RU], guC[RU];
            {
                T lx[RX][4], hx[RX][4], e7[RX][4];
                ld_rows<T, NX>(blo, o7 >= 0, lx);
                ld_rows<T, NX>(bhi, o7 >= 0, hx);
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (o7 >= 0 && tok<NX>(rt, e)) {
                        const T v = (d7x[rt][e] + alpha * (T(2) * xz[rt][e] - xp[rt][e])) * ra;
                        fin(d7x[rt][e], v, box_apply_t(v, lx[rt][e], hx[rt][e], ctl), xz[rt][e] - xp[rt][e], ep, x2);
                    }
                    e7[rt][e] = ep;
                    gxA[rt][e] = ep;
                    gxW[rt][e] = d7x[rt][e] - ep;
                    gxC[rt][e] = x2;
                }
                st_rows<T, NX>(eo + (o7 >= 0 ? o7 : 0), o7 >= 0, e7);
            }
            {
                T lu[RU][4], hu[RU][4], e7u[RU][4];
                ld_rows<T, NU>(blo + NX, o7 >= 0, lu);
                ld_rows<T, NU>(bhi + NX, o7 >= 0, hu);
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (o7 >= 0 && tok<NU>(rt, e)) {
                        const T v = (d7u[rt][e] + alpha * (T(2) * uz[rt][e] - up[rt][e])) * ra;
                        fin(d7u[rt][e], v, box_apply_t(v, lu[rt][e], hu[rt][e], ctl), uz[rt][e] - up[rt][e], ep, x2);
                    }
                    e7u[rt][e] = ep;
                    guA[rt][e] = ep;
                    guW[rt][e] = d7u[rt][e] - ep;
                    guC[rt][e] = x2;
                }
                st_rows<T, NU>(eo + (o7 >= 0 ? o7 + NX : 0), o7 >= 0, e7u);
            }
            mmt(wq, sxA, gxA);
            mmt(wq, sxW, gxW);
            mmt(wq, sxC, gxC);
            mmt(wr, suA, guA);
            mmt(wr, suW, guW);
            mmt(wr, suC, guC);
            T ox[RX][4], ou[RU][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                ox[rt][e] = xz[rt][e] - alpha * gxA[rt][e];
                if (live && tok<NX>(rt, e)) account(xp[rt][e], xz[rt][e], gxW[rt][e], gxC[rt][e]);
            }
            st_rows<T, NX>(out + p.X0 + (size_t)i * NX, live, ox);
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                ou[rt][e] = uz[rt][e] - alpha * guA[rt][e];
                if (live && tok<NU>(rt, e)) account(up[rt][e], uz[rt][e], guW[rt][e], guC[rt][e]);
            }
            st_rows<T, NU>(out + p.U0 + (size_t)i * NU, live, ou);
        }
        // ---------------- phase 5: AVaR kernel projection of the family (cache.py:290-317,
        // closed form: r_k = alpha_r y_k - y_{C+k} + y_2C - tau_k - s_k, w = (r - 1 sum(r) /
        // (a + C)) / a, a = alpha_r^2 + 3; y_k -= alpha_r w_k, y_{C+k} += w_k, y_2C -= sum(w),
        // tau_k += w_k, s_k += w_k), every lane group on its parent, stores split by group
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (live) {
            const T al = ((cglbp<T>)p.alpha_r)[i];
            const T y2c = ks.y[lo][2 * C];
            T rk[4], sr = T(0);
            _Pragma("unroll") for (int k = 0; k < 4; ++k) {
                rk[k] = T(0);
                if (k < C) {
                    rk[k] = al * ks.y[lo][k] - ks.y[lo][C + k] + y2c - ks.tau[lo][k] - ks.s[lo][k];
                    sr += rk[k];
                }
            }
            const T a = al * al + T(3);
            T sw = T(0);
            _Pragma("unroll") for (int k = 0; k < 4; ++k) {
                if (k < C) {
                    const T w = (rk[k] - sr / (a + (T)C)) / a;
                    sw += w;
                    if (k == h) {
                        const int j = 1 + C * i + k;
                        out[p.Y0 + yo + k] = ks.y[lo][k] - al * w;
                        out[p.Y0 + yo + C + k] = ks.y[lo][C + k] + w;
                        out[p.T0 + j] = ks.tau[lo][k] + w;
                        out[p.S0 + j] = ks.s[lo][k] + w;
                    }
                }
            }
            if (h == 0) out[p.Y0 + yo + 2 * C] = y2c - sw;
        }
        __builtin_amdgcn_wave_barrier();
    }
    // per-block residual maxima -> one row of `part` (plain stores, k_cp_check reduces)
    double mm[6] = {m0, m1, m2, m3, m4, m5};
    _Pragma("unroll") for (int q = 0; q < 6; ++q)
        _Pragma("unroll") for (int off = 32; off > 0; off >>= 1) mm[q] = nmax(mm[q], __shfl_xor(mm[q], off, 64));
    if (lane == 0) _Pragma("unroll") for (int q = 0; q < 6; ++q) s_red[q][wv] = mm[q];
    __syncthreads();
    if (threadIdx.x < 6) {
        double b = s_red[threadIdx.x][0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) b = nmax(b, s_red[threadIdx.x][w]);
        part[(size_t)blockIdx.x * 6 + threadIdx.x] = b;
    }
}
