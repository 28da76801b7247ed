// raocp_dyn3.hip — the dynamics projection (cache.py:259-288) stage by stage as streaming
// MFMA wave tasks, for trees with one branching factor C <= 4 whose child slot k has the
// same (A, B) pair at every parent of a stage and whose parents of a stage share one
// offline class (host checks, raocp_capi.hip): the i.i.d. trees of configs 2, 4 and 5.
// Included by raocp_kernels.hip after raocp_cp3.hip (the row layout, WL fragments, MFA).
//
// Device form (raocp_dyn.hip header):
//   backward, stage t = N-1 .. 0, a tile of 16 parents i (lane lo = parent):
//     h = sum_k B_k' q_j, a = sum_k A_k' q_j      (child j = 1 + C i + k; q_j = -x_j at leaves)
//     v = u_i - h ;  d_i = Rinv v ;  q_i = (-x_i + a) + G v
//   forward, stage t = 0 .. N-1 (x_0 = x0bar at stage 0):
//     u_i = K x_i + d_i ;  x_j = Abar_k x_i + B_k d_i
// One launch per stage and direction (the recursion is sequential in the stage); inside a
// launch every product is a chain of 16x16x4 MFMAs in the transposed form of raocp_cp3.hip:
// the children's products accumulate per parent in the MFMA accumulators, whose row layout
// is directly the B operand of the parent's Rinv / G products. No LDS staging of vectors, no
// barrier after the weight fill: a wave reads its parents' and children's rows with 16-B
// loads straight into registers and writes its outputs from them.
//
// Weights: the stage's tables (slot k: B_k', A_k' backward, Abar_k, B_k forward; the class's
// Rinv, G, K) in fragment order (WLs below): k_dy3_image lays them out once per context as
// one contiguous image per stage and direction, which every workgroup copies into LDS by
// LDS-DMA (one memory round trip; the element-wise fragment gather it replaces was most of
// the ~10 us a launch of a one-tile stage cost at config 5, profiles/r03_v2).

// a fragment table taken from a column-major source with leading dimension ld, rows
// [r0, r0 + R), columns [c0, c0 + K): lds[(ro KS + s) 64 + lane] = M[r][k] (transposed form,
// row layout of raocp_cp3.hip)
template <class T, int R, int K>
struct WLs {
    static_assert(R % 4 == 0 && K % 4 == 0, "row layout: R, K multiples of 4");
    static constexpr int RO = (R / 4 + 3) / 4, KS = K / 4, N = RO * KS * 64;
    const __attribute__((address_space(3))) T* base;
    __device__ __forceinline__ T get(int ro, int s) const { return base[(ro * KS + s) * 64 + (threadIdx.x & 63)]; }
    template <class DP>
    static __device__ __forceinline__ void fill(DP dst, const T* M, int ld, int r0, int c0) {
        for (int q = threadIdx.x; q < N; q += blockDim.x) {
            const int l = q & 63, lo = l & 15, h = l >> 4, s = (q >> 6) % KS, ro = (q >> 6) / KS;
            const int r = wrow<T, R>(ro, lo), k = KS * h + s;
            dst[q] = r >= 0 ? ((cglbp<T>)M)[(size_t)(c0 + k) * ld + r0 + r] : T(0);
        }
    }
    // the same from a row-major source: M[r][k] = src[(r0 + r) ld + c0 + k]
    template <class DP>
    static __device__ __forceinline__ void fill_t(DP dst, const T* M, int ld, int r0, int c0) {
        for (int q = threadIdx.x; q < N; q += blockDim.x) {
            const int l = q & 63, lo = l & 15, h = l >> 4, s = (q >> 6) % KS, ro = (q >> 6) / KS;
            const int r = wrow<T, R>(ro, lo), k = KS * h + s;
            dst[q] = r >= 0 ? ((cglbp<T>)M)[(size_t)(r0 + r) * ld + c0 + k] : T(0);
        }
    }
};
template <class T, int R, int K>
__device__ __forceinline__ void mmts(const WLs<T, R, K>& W, const T (&b)[(K + 15) / 16][4],
                                     typename MF<T>::v4 (&acc)[(R + 15) / 16]) {
    _Pragma("unroll") for (int s = 0; s < WLs<T, R, K>::KS; ++s)
        _Pragma("unroll") for (int ro = 0; ro < WLs<T, R, K>::RO; ++ro)
            acc[ro] = MF<T>::mma(W.get(ro, s), b[s >> 2][s & 3], acc[ro]);
}

// one stage of the sweep (host-built)
struct Dy3Stage {
    int i0, i1;   // parents of the stage
    int leaf;     // the children are leaves (stage N - 1)
    int cls;      // offline class of the stage's parents
    int kind[4];  // child kind (A, B pair) of slot k
    int pair[4];  // (kind, class) pair of slot k
};

template <class T, int NX, int NU>
struct Dy3Lds {
    typedef WLs<T, NU, NX> WB;  // B_k'
    typedef WLs<T, NX, NX> WA;  // A_k' (backward) / Abar_k (forward)
    typedef WLs<T, NU, NU> WRI; // Rinv
    typedef WLs<T, NX, NU> WG;  // G (backward) / B_k (forward)
    typedef WLs<T, NU, NX> WK;  // K
    // LDS scalars of one stage's tables for C slots (host: dynamic shared bytes)
    static constexpr __host__ __device__ int back_n(int C) { return C * (WB::N + WA::N) + WRI::N + WG::N; }
    static constexpr __host__ __device__ int fwd_n(int C) { return WK::N + C * (WA::N + WG::N); }
};

// tables (column-major M[k R + r], raocp_capi.hip): W2[kind] = [B'; A'] (R = nu + nx rows,
// nx columns), RG2[cls] = [Rinv; G] (R rows, nu columns), KM2[cls] = K (nu x nx),
// F2[pair] = [Abar | B] (nx rows, nx + nu columns)
// backward image of a stage: per slot k [B_k' | A_k'], then [Rinv | G] of its class
template <class T, int NX, int NU, class DP>
__device__ __forceinline__ void dy3_back_tables(DP wl, const Dy3Stage& st, int C, const double* W2, const double* RG2) {
    typedef Dy3Lds<T, NX, NU> L;
    constexpr int R = NX + NU;
    const T* W = (const T*)W2;
    for (int k = 0; k < C; ++k) {
        L::WB::fill(wl + k * (L::WB::N + L::WA::N), W + (size_t)st.kind[k] * R * NX, R, 0, 0);
        L::WA::fill(wl + k * (L::WB::N + L::WA::N) + L::WB::N, W + (size_t)st.kind[k] * R * NX, R, NU, 0);
    }
    DP wr = wl + C * (L::WB::N + L::WA::N);
    L::WRI::fill(wr, (const T*)RG2 + (size_t)st.cls * R * NU, R, 0, 0);
    L::WG::fill(wr + L::WRI::N, (const T*)RG2 + (size_t)st.cls * R * NU, R, NU, 0);
}
// forward image: K of the class, then per slot k [A_k | B_k] (x_j = A_k x + B_k u with
// u = K x + d, the reference's Abar_k x + B_k d (cache.py:286-288) re-associated so that the
// slot tables do not depend on the class: the top workgroup keeps them across stages)
template <class T, int NX, int NU, class DP>
__device__ __forceinline__ void dy3_fwd_tables(DP wl, const Dy3Stage& st, int C, const double* W2,
                                               const double* KM2, const double* F2) {
    typedef Dy3Lds<T, NX, NU> L;
    constexpr int R = NX + NU;
    L::WK::fill(wl, (const T*)KM2 + (size_t)st.cls * NU * NX, NU, 0, 0);
    DP wf = wl + L::WK::N;
    for (int k = 0; k < C; ++k) {
        const T* F = (const T*)F2 + (size_t)st.pair[k] * NX * (NX + NU);
        // A_k[r][c] = (A_k')[c][r]: row NU + c, column r of W2[kind] (column-major, R rows)
        L::WA::fill_t(wf + k * (L::WA::N + L::WG::N), (const T*)W2 + (size_t)st.kind[k] * R * NX, R, 0, NU);
        L::WG::fill(wf + k * (L::WA::N + L::WG::N) + L::WA::N, F, NX, 0, NX);    // B_k
    }
}
// one workgroup per stage, at context creation: the stage's backward and forward images
template <class T, int NX, int NU>
__global__ void __launch_bounds__(512) k_dy3_image(Dy3Stage st, int C, const double* __restrict__ W2,
                                                   const double* __restrict__ RG2, const double* __restrict__ KM2,
                                                   const double* __restrict__ F2, double* bimg, double* fimg) {
    dy3_back_tables<T, NX, NU>((glbp<T>)bimg, st, C, W2, RG2);
    dy3_fwd_tables<T, NX, NU>((glbp<T>)fimg, st, C, W2, KM2, F2);
}

template <class T, int NX, int NU>
__global__ void __launch_bounds__(512) k_dy3_back(Dev p, const Ctl* ctl, ChkArg ck, double* __restrict__ z_,
                                                  double* __restrict__ q_, double* __restrict__ d_, Dy3Stage st, int C,
                                                  const double* __restrict__ img, int sp) {
    typedef typename MF<T>::v4 v4;
    typedef Dy3Lds<T, NX, NU> L;
    constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16;
    if (ck.on && blockIdx.x == gridDim.x - 1) {
        // the previous CP iteration's stopping test (defer_check, raocp_capi.hip)
        if (threadIdx.x < 64) cp_check_wave(ck);
        return;
    }
    extern __shared__ __attribute__((aligned(16))) double dsm_[];
    typedef __attribute__((address_space(3))) T lT;
    lT* wl = (lT*)dsm_;
    dma((ldsd*)dsm_, img, L::back_n(C) * (int)sizeof(T) / 8);  // whole 16-B chunks (N: multiples of 64)
    const int done = ctl_done(ctl);  // read while the image is in flight (raocp_dyn.hip)
    lT* wr = wl + C * (L::WB::N + L::WA::N);
    const typename L::WRI wri{wr};
    const typename L::WG wg{wr + L::WRI::N};
    glbp<T> z = (glbp<T>)z_;
    glbp<T> qb = (glbp<T>)q_;
    glbp<T> db = (glbp<T>)d_;
    const int lo = threadIdx.x & 15, wv = threadIdx.x >> 6;
    const int ntile = (st.i1 - st.i0 + 15) >> 4;
    // sp (stages of few tiles): a workgroup per tile, wave k on child slot k, the slot sums
    // gathered in LDS (slot order) by wave 0; else a wave per tile, slots in sequence
    const int gw = sp ? blockIdx.x : blockIdx.x * (blockDim.x >> 6) + wv;
    const int nw = (gridDim.x - ck.on) * (sp ? 1 : (blockDim.x >> 6));
    const int k0 = sp ? wv : 0, k1 = sp ? (wv < C ? wv + 1 : 0) : C;
    lT* red = wl + L::back_n(C);  // sp: [C][RU + RX][4][64 lanes]
    // a task's rows (children's q, or -x at the leaves; the parents' u and x) are read into
    // registers before its products: the first task's while the stage image is in flight
    T qj[4][RX][4], u[RU][4], x[RX][4];
    auto load = [&](int task) {
        const int i = st.i0 + 16 * task + lo;
        const bool live = i < st.i1;
        _Pragma("unroll") for (int k = 0; k < 4; ++k) {
            if (k < k0 || k >= k1) continue;
            const int j = 1 + C * (live ? i : st.i0) + k;
            if (st.leaf) ld_rows<T, NX>((cglbp<T>)z + p.X0 + (size_t)j * NX, live, qj[k]);
            else ld_rows<T, NX>((cglbp<T>)qb + (size_t)j * NX, live, qj[k]);
        }
        ld_rows<T, NU>((cglbp<T>)z + p.U0 + (size_t)i * NU, live, u);
        ld_rows<T, NX>((cglbp<T>)z + p.X0 + (size_t)i * NX, live, x);
    };
    // fp32 (config 5: two tiles per wave in the widest stage): a wave per tile, its next tile's
    // rows double-buffered, issued before the current tile's slot products, so that a wide
    // stage's load burst overlaps the MFMA chains instead of following them. Branch-free loads:
    // a dead lane reads its tile's last live row, a slot k >= C re-reads slot C - 1 (valid
    // addresses, results unused). (fp64: the second buffer spills at 32 / 12 and config 4's
    // wide stages have one tile per wave: the single-buffer loop below.)
    if constexpr (sizeof(T) == 4) if (!sp) {
        T qn[4][RX][4], un[RU][4], xn[RX][4];
        auto ld_all = [&](int task, T(&q)[4][RX][4], T(&uu)[RU][4], T(&xx)[RX][4]) {
            const int ic = min(st.i0 + 16 * task + lo, st.i1 - 1);
            cglbp<T> src = st.leaf ? (cglbp<T>)z + p.X0 : (cglbp<T>)qb;
            _Pragma("unroll") for (int k = 0; k < 4; ++k) {
                const int kk = k < C ? k : C - 1;
                ld_rows<T, NX>(src + (size_t)(1 + C * ic + kk) * NX, true, q[k]);
            }
            ld_rows<T, NU>((cglbp<T>)z + p.U0 + (size_t)ic * NU, true, uu);
            ld_rows<T, NX>((cglbp<T>)z + p.X0 + (size_t)ic * NX, true, xx);
        };
        ld_all(min(gw, ntile - 1), qj, u, x);
        dma_wait();
        __syncthreads();
        if (done) return;
        for (int task = gw; task < ntile; task += nw) {
            const int i = st.i0 + 16 * task + lo;
            const bool live = i < st.i1;
            ld_all(min(task + nw, ntile - 1), qn, un, xn);
            v4 ha[RU], aa[RX];
            _Pragma("unroll") for (int r = 0; r < RU; ++r) ha[r] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int r = 0; r < RX; ++r) aa[r] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int k = 0; k < 4; ++k) {
                if (k >= C) continue;
                if (st.leaf)
                    _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) qj[k][rt][e] = -qj[k][rt][e];
                const typename L::WB wb{wl + k * (L::WB::N + L::WA::N)};
                const typename L::WA wa{wl + k * (L::WB::N + L::WA::N) + L::WB::N};
                mmts(wb, qj[k], ha);
                mmts(wa, qj[k], aa);
            }
            T v[RU][4];
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) v[rt][e] = u[rt][e] - ha[rt][e];
            v4 dv[RU], gv[RX];
            _Pragma("unroll") for (int r = 0; r < RU; ++r) dv[r] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int r = 0; r < RX; ++r) gv[r] = v4{0, 0, 0, 0};
            mmts(wri, v, dv);
            mmts(wg, v, gv);
            T dd[RU][4], qq[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) dd[rt][e] = dv[rt][e];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                qq[rt][e] = (-x[rt][e] + aa[rt][e]) + gv[rt][e];
            st_rows<T, NU>(db + (size_t)i * NU, live, dd);
            st_rows<T, NX>(qb + (size_t)i * NX, live, qq);
            _Pragma("unroll") for (int k = 0; k < 4; ++k) _Pragma("unroll") for (int rt = 0; rt < RX; ++rt)
                _Pragma("unroll") for (int e = 0; e < 4; ++e) qj[k][rt][e] = qn[k][rt][e];
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) u[rt][e] = un[rt][e];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) x[rt][e] = xn[rt][e];
        }
        return;
    }
    // sp: a workgroup per tile (looping over tiles), wave k on child slot k; fp64: also a wave
    // per tile
    if (gw < ntile) load(gw);
    dma_wait();
    __syncthreads();
    if (done) return;
    for (int task = gw; task < ntile; task += nw) {
        const int i = st.i0 + 16 * task + lo;
        const bool live = i < st.i1;
        v4 ha[RU], aa[RX];
        _Pragma("unroll") for (int r = 0; r < RU; ++r) ha[r] = v4{0, 0, 0, 0};
        _Pragma("unroll") for (int r = 0; r < RX; ++r) aa[r] = v4{0, 0, 0, 0};
        _Pragma("unroll") for (int k = 0; k < 4; ++k) {
            if (k < k0 || k >= k1) continue;
            if (st.leaf)
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) qj[k][rt][e] = -qj[k][rt][e];
            const typename L::WB wb{wl + k * (L::WB::N + L::WA::N)};
            const typename L::WA wa{wl + k * (L::WB::N + L::WA::N) + L::WB::N};
            mmts(wb, qj[k], ha);
            mmts(wa, qj[k], aa);
        }
        if (sp) {
            const int l = threadIdx.x & 63;
            if (wv < C) {
                _Pragma("unroll") for (int r = 0; r < RU; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    red[((wv * (RU + RX) + r) * 4 + e) * 64 + l] = ha[r][e];
                _Pragma("unroll") for (int r = 0; r < RX; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    red[((wv * (RU + RX) + RU + r) * 4 + e) * 64 + l] = aa[r][e];
            }
            __syncthreads();
            if (wv == 0) {
                for (int k = 1; k < C; ++k) {
                    _Pragma("unroll") for (int r = 0; r < RU; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                        ha[r][e] += red[((k * (RU + RX) + r) * 4 + e) * 64 + l];
                    _Pragma("unroll") for (int r = 0; r < RX; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                        aa[r][e] += red[((k * (RU + RX) + RU + r) * 4 + e) * 64 + l];
                }
            }
            __syncthreads();  // red is rewritten by the next tile
            if (wv != 0) {
                if (task + nw < ntile) load(task + nw);
                continue;
            }
        }
        T v[RU][4];
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) v[rt][e] = u[rt][e] - ha[rt][e];
        T xs[RX][4];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) xs[rt][e] = x[rt][e];
        if (task + nw < ntile) load(task + nw);  // the next task's rows behind this one's products
        v4 dv[RU], gv[RX];
        _Pragma("unroll") for (int r = 0; r < RU; ++r) dv[r] = v4{0, 0, 0, 0};
        _Pragma("unroll") for (int r = 0; r < RX; ++r) gv[r] = v4{0, 0, 0, 0};
        mmts(wri, v, dv);
        mmts(wg, v, gv);
        T dd[RU][4], qq[RX][4];
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) dd[rt][e] = dv[rt][e];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
            qq[rt][e] = (-xs[rt][e] + aa[rt][e]) + gv[rt][e];
        st_rows<T, NU>(db + (size_t)i * NU, live, dd);
        st_rows<T, NX>(qb + (size_t)i * NX, live, qq);
    }
}

template <class T, int NX, int NU>
__global__ void __launch_bounds__(512) k_dy3_fwd(Dev p, const Ctl* ctl, double* __restrict__ z_,
                                                 const double* __restrict__ d_, const double* __restrict__ x0_, Dy3Stage st,
                                                 int C, const double* __restrict__ img, int sp) {
    typedef typename MF<T>::v4 v4;
    typedef Dy3Lds<T, NX, NU> L;
    constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16;
    extern __shared__ __attribute__((aligned(16))) double dsm_[];
    typedef __attribute__((address_space(3))) T lT;
    lT* wl = (lT*)dsm_;
    dma((ldsd*)dsm_, img, L::fwd_n(C) * (int)sizeof(T) / 8);
    const int done = ctl_done(ctl);
    lT* wf = wl + L::WK::N;
    const typename L::WK wk{wl};
    glbp<T> z = (glbp<T>)z_;
    cglbp<T> db = (cglbp<T>)d_;
    const int lo = threadIdx.x & 15;
    const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), nw = gridDim.x * (blockDim.x >> 6);
    const int ntile = (st.i1 - st.i0 + 15) >> 4;
    // sp (stages of few tiles): a task per (tile, child slot), slot 0 also writing u
    const int ntask = sp ? ntile * C : ntile;
    // a task's x and d rows are read before its products: the first task's while the stage
    // image is in flight, the next task's behind the current one's
    T x[RX][4], d[RU][4];
    auto load = [&](int tk) {
        const int task = sp ? tk / C : tk;
        const int i = st.i0 + 16 * task + lo;
        const bool live = i < st.i1;
        if (i == 0) ld_rows<T, NX>((cglbp<T>)x0_, true, x);  // x_0 = x0bar (cache.py:283)
        else ld_rows<T, NX>((cglbp<T>)z + p.X0 + (size_t)i * NX, live, x);
        ld_rows<T, NU>(db + (size_t)i * NU, live, d);
    };
    if (gw < ntask) load(gw);
    dma_wait();
    __syncthreads();
    if (done) return;
    for (int tk = gw; tk < ntask; tk += nw) {
        const int task = sp ? tk / C : tk, ks = sp ? tk % C : 0, ke = sp ? ks + 1 : C;
        const int i = st.i0 + 16 * task + lo;
        const bool live = i < st.i1;
        T xc[RX][4], dc[RU][4];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) xc[rt][e] = x[rt][e];
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) dc[rt][e] = d[rt][e];
        if (tk + nw < ntask) load(tk + nw);
        if (i == 0 && ks == 0) st_rows<T, NX>(z + p.X0, true, xc);  // x_0 into the iterate (slot-0 task)
        v4 ku[RU];
        _Pragma("unroll") for (int r = 0; r < RU; ++r) ku[r] = v4{0, 0, 0, 0};
        mmts(wk, xc, ku);
        T u[RU][4];
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) u[rt][e] = ku[rt][e] + dc[rt][e];
        if (ks == 0) st_rows<T, NU>(z + p.U0 + (size_t)i * NU, live, u);
        for (int k = ks; k < ke; ++k) {
            const int j = 1 + C * (live ? i : st.i0) + k;
            const typename L::WA wa{wf + k * (L::WA::N + L::WG::N)};
            const typename L::WG wb{wf + k * (L::WA::N + L::WG::N) + L::WA::N};
            v4 xa[RX];
            _Pragma("unroll") for (int r = 0; r < RX; ++r) xa[r] = v4{0, 0, 0, 0};
            mmts(wa, xc, xa);
            mmts(wb, u, xa);
            T xj[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) xj[rt][e] = xa[rt][e];
            st_rows<T, NX>(z + p.X0 + (size_t)j * NX, live, xj);
        }
    }
}

// ---- the small top stages of both sweeps in ONE workgroup each (k_dy3_top_back /
// k_dy3_top_fwd): a stage of a few tiles costs a launch (dispatch, image fill, one tile's
// MFMA chain, drain: 3.5-7 us at configs 4 / 5) for a few microseconds of work, so the
// stages t < ts run back to back in one 512-lane workgroup, the image of each filled into
// the same LDS by LDS-DMA, a barrier between stages (the rows a stage writes are the next
// one's inputs: the same CU, so workgroup-scope visibility suffices).
constexpr int kDy3TopMax = 8;
struct Dy3Top {
    Dy3Stage st[kDy3TopMax];
    int ts;          // stages 0 .. ts - 1
    int same_kinds;  // every top stage has the same child-slot kinds (the slot tables stay in LDS)
};

// backward, t = ts - 1 .. 0: rounds of TPR = waves / C tiles, wave w on tile w / C and child
// slot w % C (the slot order of the sp launches: bit-identical sums), the slot sums of
// slots >= 1 through LDS to the tile's slot-0 wave, which finishes the tile (v, d, q)
template <class T, int NX, int NU>
__global__ void __launch_bounds__(512) k_dy3_top_back(Dev p, const Ctl* ctl, double* __restrict__ z_,
                                                      double* __restrict__ q_, double* __restrict__ d_, Dy3Top tp, int C,
                                                      const double* __restrict__ img0) {
    typedef typename MF<T>::v4 v4;
    typedef Dy3Lds<T, NX, NU> L;
    constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16;
    extern __shared__ __attribute__((aligned(16))) double dsm_[];
    typedef __attribute__((address_space(3))) T lT;
    lT* wl = (lT*)dsm_;
    if (ctl_done(ctl)) return;
    glbp<T> z = (glbp<T>)z_;
    glbp<T> qb = (glbp<T>)q_;
    glbp<T> db = (glbp<T>)d_;
    const int lo = threadIdx.x & 15, l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int tpr = (blockDim.x >> 6) / C, tl = wv / C, k = wv - tl * C;
    lT* wr = wl + C * (L::WB::N + L::WA::N);
    lT* red = wl + L::back_n(C);  // [tpr][C][RU + RX][4][64 lanes]
    // a round's rows (the children's q, the parents' u and x) are read into registers before
    // the wait for the stage image, the first round's while the image is in flight: the image's
    // and the rows' memory latencies overlap instead of following each other
    T qj[RX][4], u[RU][4], x[RX][4];
    auto load = [&](const Dy3Stage& st, int t0) {
        const int task = t0 + tl;
        const bool act = tl < tpr && task < ((st.i1 - st.i0 + 15) >> 4);
        const int i = st.i0 + 16 * task + lo;
        const bool live = act && i < st.i1;
        if (!act) return;
        const int j = 1 + C * (live ? i : st.i0) + k;
        if (st.leaf) ld_rows<T, NX>((cglbp<T>)z + p.X0 + (size_t)j * NX, live, qj);
        else ld_rows<T, NX>((cglbp<T>)qb + (size_t)j * NX, live, qj);
        if (k == 0) {
            ld_rows<T, NU>((cglbp<T>)z + p.U0 + (size_t)i * NU, live, u);
            ld_rows<T, NX>((cglbp<T>)z + p.X0 + (size_t)i * NX, live, x);
        }
    };
    // the child slots' tables [B_k' | A_k'] depend on the slot's (A, B) kind only: when every
    // top stage has the same kinds (tp.same_kinds) they stay in LDS after the first stage and a
    // stage loads only its class's [Rinv | G] (a CU ingests ~12 B/cycle: the whole fp32 64/16
    // image is ~3 us, the class part ~0.2 us)
    const int off = C * (L::WB::N + L::WA::N);  // elements; a multiple of 64
    for (int si = tp.ts - 1; si >= 0; --si) {
        const Dy3Stage st = tp.st[si];
        const double* src = img0 + (size_t)si * L::back_n(C) * sizeof(T) / 8;
        if (tp.same_kinds && si < tp.ts - 1)
            dma((ldsd*)(wl + off), src + (size_t)off * sizeof(T) / 8, (L::back_n(C) - off) * (int)sizeof(T) / 8);
        else
            dma((ldsd*)dsm_, src, L::back_n(C) * (int)sizeof(T) / 8);
        load(st, 0);
        dma_wait();
        __syncthreads();
        const typename L::WRI wri{wr};
        const typename L::WG wg{wr + L::WRI::N};
        const int ntile = (st.i1 - st.i0 + 15) >> 4;
        for (int t0 = 0; t0 < ntile; t0 += tpr) {
            const int task = t0 + tl;
            const bool act = tl < tpr && task < ntile;
            const int i = st.i0 + 16 * task + lo;
            const bool live = act && i < st.i1;
            v4 ha[RU], aa[RX];
            _Pragma("unroll") for (int r = 0; r < RU; ++r) ha[r] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int r = 0; r < RX; ++r) aa[r] = v4{0, 0, 0, 0};
            if (act) {
                if (st.leaf)
                    _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) qj[rt][e] = -qj[rt][e];
                const typename L::WB wb{wl + k * (L::WB::N + L::WA::N)};
                const typename L::WA wa{wl + k * (L::WB::N + L::WA::N) + L::WB::N};
                mmts(wb, qj, ha);
                mmts(wa, qj, aa);
                if (k > 0) {
                    lT* rd = red + (size_t)(tl * C + k) * (RU + RX) * 4 * 64;
                    _Pragma("unroll") for (int r = 0; r < RU; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                        rd[(r * 4 + e) * 64 + l] = ha[r][e];
                    _Pragma("unroll") for (int r = 0; r < RX; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                        rd[((RU + r) * 4 + e) * 64 + l] = aa[r][e];
                    load(st, t0 + tpr);  // the next round's rows behind this one's products
                }
            }
            __syncthreads();
            if (act && k == 0) {
                for (int kk = 1; kk < C; ++kk) {
                    const lT* rd = red + (size_t)(tl * C + kk) * (RU + RX) * 4 * 64;
                    _Pragma("unroll") for (int r = 0; r < RU; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                        ha[r][e] += rd[(r * 4 + e) * 64 + l];
                    _Pragma("unroll") for (int r = 0; r < RX; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                        aa[r][e] += rd[((RU + r) * 4 + e) * 64 + l];
                }
                T v[RU][4];
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) v[rt][e] = u[rt][e] - ha[rt][e];
                v4 dv[RU], gv[RX];
                _Pragma("unroll") for (int r = 0; r < RU; ++r) dv[r] = v4{0, 0, 0, 0};
                _Pragma("unroll") for (int r = 0; r < RX; ++r) gv[r] = v4{0, 0, 0, 0};
                mmts(wri, v, dv);
                mmts(wg, v, gv);
                T dd[RU][4], qq[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) dd[rt][e] = dv[rt][e];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    qq[rt][e] = (-x[rt][e] + aa[rt][e]) + gv[rt][e];
                st_rows<T, NU>(db + (size_t)i * NU, live, dd);
                st_rows<T, NX>(qb + (size_t)i * NX, live, qq);
                load(st, t0 + tpr);
            }
            __syncthreads();  // red is rewritten by the next round; the rows by the next stage
        }
    }
}

// forward, t = 0 .. ts - 1: the (tile, child slot) tasks of a stage over the waves (the sp
// launches' task order), slot 0 also writing u
template <class T, int NX, int NU>
__global__ void __launch_bounds__(512) k_dy3_top_fwd(Dev p, const Ctl* ctl, double* __restrict__ z_,
                                                     const double* __restrict__ d_, const double* __restrict__ x0_,
                                                     Dy3Top tp, int C, const double* __restrict__ img0) {
    typedef typename MF<T>::v4 v4;
    typedef Dy3Lds<T, NX, NU> L;
    constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16;
    extern __shared__ __attribute__((aligned(16))) double dsm_[];
    typedef __attribute__((address_space(3))) T lT;
    lT* wl = (lT*)dsm_;
    if (ctl_done(ctl)) return;
    glbp<T> z = (glbp<T>)z_;
    cglbp<T> db = (cglbp<T>)d_;
    const int lo = threadIdx.x & 15, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    lT* wf = wl + L::WK::N;
    // a task's x and d rows are read before the wait for the stage image (the first task's
    // while the image is in flight, the next task's behind the current one's products)
    T x[RX][4], d[RU][4];
    auto load = [&](const Dy3Stage& st, int tk) {
        const int task = tk / C;
        const int i = st.i0 + 16 * task + lo;
        const bool live = i < st.i1;
        if (i == 0) ld_rows<T, NX>((cglbp<T>)x0_, true, x);  // x_0 = x0bar (cache.py:283)
        else ld_rows<T, NX>((cglbp<T>)z + p.X0 + (size_t)i * NX, live, x);
        ld_rows<T, NU>(db + (size_t)i * NU, live, d);
    };
    for (int si = 0; si < tp.ts; ++si) {
        const Dy3Stage st = tp.st[si];
        const int ntile = (st.i1 - st.i0 + 15) >> 4, ntask = ntile * C;
        // the slot tables [A_k | B_k] stay in LDS after the first stage when the kinds agree
        const int nload = tp.same_kinds && si > 0 ? L::WK::N : L::fwd_n(C);
        dma((ldsd*)dsm_, img0 + (size_t)si * L::fwd_n(C) * sizeof(T) / 8, nload * (int)sizeof(T) / 8);
        if (wv < ntask) load(st, wv);
        dma_wait();
        __syncthreads();
        const typename L::WK wk{wl};
        for (int tk = wv; tk < ntask; tk += nwv) {
            const int task = tk / C, ks = tk - task * C;
            const int i = st.i0 + 16 * task + lo;
            const bool live = i < st.i1;
            T xc[RX][4], dc[RU][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) xc[rt][e] = x[rt][e];
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) dc[rt][e] = d[rt][e];
            if (tk + nwv < ntask) load(st, tk + nwv);
            if (i == 0 && ks == 0) st_rows<T, NX>(z + p.X0, true, xc);
            v4 ku[RU];
            _Pragma("unroll") for (int r = 0; r < RU; ++r) ku[r] = v4{0, 0, 0, 0};
            mmts(wk, xc, ku);
            T u[RU][4];
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) u[rt][e] = ku[rt][e] + dc[rt][e];
            if (ks == 0) st_rows<T, NU>(z + p.U0 + (size_t)i * NU, live, u);
            const int j = 1 + C * (live ? i : st.i0) + ks;
            const typename L::WA wa{wf + ks * (L::WA::N + L::WG::N)};
            const typename L::WG wb{wf + ks * (L::WA::N + L::WG::N) + L::WA::N};
            v4 xa[RX];
            _Pragma("unroll") for (int r = 0; r < RX; ++r) xa[r] = v4{0, 0, 0, 0};
            mmts(wa, xc, xa);
            mmts(wb, u, xa);
            T xj[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) xj[rt][e] = xa[rt][e];
            st_rows<T, NX>(z + p.X0 + (size_t)j * NX, live, xj);
        }
        __syncthreads();  // the children's x rows are the next stage's inputs; the image is rewritten
    }
}
