// raocp_cp2.hip — the two node-block kernels of one Chambolle–Pock iteration, with the
// matrix-vector products of L and L^T as MFMA tiles (included by raocp_kernels.hip,
// inside namespace raocp).
//
//   k_cpd2: dual half step + prox of g* + xi2 (solver.py:44-61, cache.py:321-393, 63-95)
//   k_cpp2: next primal half step + AVaR kernel projection + the finished iteration's
//           xi0, xi1, delta0, delta1 (solver.py:27-39, cache.py:248-317, 63-95)
//
// Blocks (host table Dev::cp2_tab): a FAMILY block owns parents [i0, i1) with all their
// children [cb, ce) — everything the L / L^T rows of a family touch is inside it — and a
// LEAF block owns leaves [l0, l1). A block first stages every input range it reads into
// LDS by LDS-DMA (one memory round trip; ranges are contiguous in the BFS numbering),
// while each wave loads the weight fragments of its tiles into registers (the tables
// are per mode and deduplicated, so a block's children usually share one table: the
// host flags the block's table index; a tree with a block whose nodes use different
// tables runs the scalar kernels of raocp_cp.hip instead). Then:
//   * the products sqrtQ x_anc(j), sqrtR u_anc(j) (k_cpd2), sqrtQ eta3_j, sqrtR eta4_j
//     (k_cpp2) and sqrtPf x_l / sqrtPf eta11_l are 16-node x 16-row MFMA tiles
//     (v_mfma_f64_16x16x4f64 / v_mfma_f32_16x16x4f32), one tile per wave;
//   * k_cpd2's second-order-cone projection of a child block (eta3, eta4, eta5, eta6) is
//     done in the registers of the tile: the squared norm is summed over the row tiles
//     in-lane and over the 16 lanes of the node by xor shuffles, no LDS, no barrier;
//   * k_cpp2 sums the children's products per parent in the lanes: on a regular block
//     (every parent has the same child count c <= 4, uniform tables) tile row h + 4e
//     (f64 layout; 4h + e for f32) is child e % c of parent h + 4 (e / c), so the c
//     products of a parent land in one lane, which adds them in child order.
// The elementwise rows (eta1, eta2, eta7, eta14 boxes; the AVaR kernel projection) keep
// the lanes-over-rows mapping. Rows are stored from the tiles: 16 consecutive rows of a
// node per 16-lane group.
//
// Arithmetic (the reference's): L(2z+ - p) and L(z+ - p) are formed from A operands
// 2z+ - p and z+ - p, not as 2Lz+ - Lp, so only the summation order differs from numpy.

// ---- 16x16x4 MFMA in T -------------------------------------------------------------
template <class T>
struct MF;
template <>
struct MF<double> {
    typedef double v4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ v4 mma(double a, double b, v4 c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // tile row (A row) of accumulator element e in lane group h = lane >> 4, and back
    static __device__ __forceinline__ int row(int h, int e) { return h + 4 * e; }
    static __device__ __forceinline__ int h_of(int a) { return a & 3; }
    static __device__ __forceinline__ int e_of(int a) { return a >> 2; }
};
template <>
struct MF<float> {
    typedef float v4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ v4 mma(float a, float b, v4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int h, int e) { return 4 * h + e; }
    static __device__ __forceinline__ int h_of(int a) { return a >> 2; }
    static __device__ __forceinline__ int e_of(int a) { return a & 3; }
};

template <class U>
using ldsp = const __attribute__((address_space(3))) U*;
template <class U>
using glbp = __attribute__((address_space(1))) U*;
template <class U>
using cglbp = const __attribute__((address_space(1))) U*;

// LDS-DMA staging of any element type: each region gets whole 16-B chunk slots starting
// at the 16-B boundary below its source (the returned pointer is shifted by the source's
// misalignment); host mirror: cp2_region_bytes in raocp_capi.hip.
struct StgB {
    ldsd* base;
    int o = 0;  // next free byte offset (multiple of 16)
    StgTable tab;
    template <class U>
    __device__ __forceinline__ ldsp<U> arr(const U* src, int count) {
        typedef __attribute__((address_space(3))) char lchar;
        const uintptr_t a = (uintptr_t)src;
        const int sh = (int)(a & 15);
        const int nb = count > 0 ? count * (int)sizeof(U) : 0;
        const int chunks = nb > 0 ? (sh + nb + 15) >> 4 : 0;
        lchar* dst = (lchar*)base + o;
        tab.record((const char*)(a - sh), chunks ? sh + nb : 0, o >> 4);
        o += 16 * chunks + 16;
        return (ldsp<U>)(dst + sh);
    }
    // send the recorded regions (StgTable::issue: packed or one pass per region)
    __device__ __forceinline__ void issue() const { tab.issue(base, o >> 4); }
};

// sum over the 16 lanes of a lane group (lanes h*16 .. h*16+15)
template <class T>
__device__ __forceinline__ T sum16(T v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    return v;
}

template <class T>
__device__ __forceinline__ T soc_apply_t(T v, bool is_t, T nf, T t) {
    // SecondOrderCone.project (cones.py:113-132) for one coordinate of the block
    if (nf <= t) return v;
    if (nf <= -t) return T(0);
    const T s = (nf + t) / T(2);
    return is_t ? s : s * (v / nf);
}
template <class T>
__device__ __forceinline__ T box_apply_t(T v, T lo, T hi, Ctl* ctl) {
    // Rectangle._constrain (rectangle.py:50-59); a NaN raises ValueError on the host
    if (lo <= v && v <= hi) return v;
    if (v <= lo) return lo;
    if (v >= hi) return hi;
    atomicOr(&ctl->flags, 1);
    return v;
}

// Weight fragments of one table of R rows x K columns (column-major M[k R + r] = M_rk; the
// L tables are square, R = K = n), RT row tiles: b[rt][s] = M[row 16 rt + lo][k = 4 s + h].
// Stationary in registers when small (STAT), else read per use (L1 / L2 resident).
template <class T, int RT, int KSM = 4 * RT>
struct WFr {
    static constexpr int KS = KSM;  // k-steps of the largest K
    static constexpr bool STAT = RT * KS * sizeof(T) <= 32 * 8;
    typedef T bvec __attribute__((ext_vector_type(STAT ? RT * KS : 1)));
    bvec b;
    const T* M = nullptr;
    int R = 0, K = 0;
    __device__ __forceinline__ void load(const T* tab, int t, int n) { load_rk(tab, t, n, n); }
    __device__ __forceinline__ void load_rk(const T* tab, int t, int R_, int K_) {
        R = R_;
        K = K_;
        M = tab + (size_t)t * R * K;
        if constexpr (STAT) {
            const int l = threadIdx.x & 63, lo = l & 15, h = l >> 4;
            _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
                _Pragma("unroll") for (int s = 0; s < KS; ++s) {
                    const int r = 16 * rt + lo, k = 4 * s + h;
                    b[rt * KS + s] = (r < R && k < K) ? ((cglbp<T>)M)[k * R + r] : T(0);
                }
            }
        }
    }
    __device__ __forceinline__ T get(int rt, int s) const {
        if constexpr (STAT) {
            return b[rt * KS + s];
        } else {
            const int l = threadIdx.x & 63, lo = l & 15, h = l >> 4;
            const int r = 16 * rt + lo, k = 4 * s + h;
            return (r < R && k < K) ? ((cglbp<T>)M)[k * R + r] : T(0);
        }
    }
};

// one A operand stream: acc[rt] += M (A rows); afun(k, a) gives this lane's A value at k
template <class T, int RT, int KSM, class AF>
__device__ __forceinline__ void tile1(const WFr<T, RT, KSM>& wf, int K, AF afun, typename MF<T>::v4 (&acc)[RT]) {
    const int h = (threadIdx.x & 63) >> 4;
    const int ks = (K + 3) >> 2;
    _Pragma("unroll") for (int s = 0; s < KSM; ++s) {
        if (s < ks) {
            const int k = 4 * s + h;
            T a = T(0);
            if (k < K) afun(k, a);
            _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) acc[rt] = MF<T>::mma(a, wf.get(rt, s), acc[rt]);
        }
    }
}

// One 16-node tile of products with ONE table (wf) and two A operand streams:
// acc1[rt] += M (A1 rows), acc2[rt] += M (A2 rows); afun(k, a1, a2) gives this lane's
// A-row values at column k (k < n; the caller zeroes dead rows).
template <class T, int RT, class AF>
__device__ __forceinline__ void tile2(const WFr<T, RT>& wf, int n, AF afun, typename MF<T>::v4 (&acc1)[RT],
                                      typename MF<T>::v4 (&acc2)[RT]) {
    const int h = (threadIdx.x & 63) >> 4;
    const int ks = (n + 3) >> 2;
    _Pragma("unroll") for (int s = 0; s < WFr<T, RT>::KS; ++s) {
        if (s < ks) {
            const int k = 4 * s + h;
            T a1 = T(0), a2 = T(0);
            if (k < n) afun(k, a1, a2);
            _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
                const T b = wf.get(rt, s);
                acc1[rt] = MF<T>::mma(a1, b, acc1[rt]);
                acc2[rt] = MF<T>::mma(a2, b, acc2[rt]);
            }
        }
    }
}
// the same with three A streams
template <class T, int RT, class AF>
__device__ __forceinline__ void tile3(const WFr<T, RT>& wf, int n, AF afun, typename MF<T>::v4 (&acc1)[RT],
                                      typename MF<T>::v4 (&acc2)[RT], typename MF<T>::v4 (&acc3)[RT]) {
    const int h = (threadIdx.x & 63) >> 4;
    const int ks = (n + 3) >> 2;
    _Pragma("unroll") for (int s = 0; s < WFr<T, RT>::KS; ++s) {
        if (s < ks) {
            const int k = 4 * s + h;
            T a1 = T(0), a2 = T(0), a3 = T(0);
            if (k < n) afun(k, a1, a2, a3);
            _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
                const T b = wf.get(rt, s);
                acc1[rt] = MF<T>::mma(a1, b, acc1[rt]);
                acc2[rt] = MF<T>::mma(a2, b, acc2[rt]);
                acc3[rt] = MF<T>::mma(a3, b, acc3[rt]);
            }
        }
    }
}

// block table of the CP kernels (host: build_cp_blocks): per family block
//   {cb, ce, y0, y1}, {e7a, e7b, i0, i1}, {SQ table, SR table, regular child count, 0}
// and per leaf block {e14a, e14b, l0, l1}, {SP table, 0, 0, 0} (always uniform tables: the
// host falls back to raocp_cp.hip otherwise).
constexpr int kCpFamRecs = 3;
constexpr int kCpLeafRecs = 2;

// block max of non-negative values (NaN wins) -> one plain store
__device__ __forceinline__ void blk_max_store(double v, double* dst, double* s_red) {
    for (int off = 32; off > 0; off >>= 1) v = nmax(v, __shfl_xor(v, off, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = s_red[0];
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) b = nmax(b, s_red[i]);
        *dst = b;
    }
}

// ==============================================================================
// k_cpd2 — dual. Blocks [0, nbF) families, [nbF, nbF + nbL) leaves.
// Buffers: p = z0, z+ = z1, d = e0 (this iteration's dual), eta+ -> e1, xi2.
// ==============================================================================
template <class T, int RTX, int RTU>
__global__ void __launch_bounds__(256) k_cpd2(Dev p, Ctl* __restrict__ ctl, Bufs bf, double* __restrict__ xi2_,
                                              double* __restrict__ part, int nbF) {
    typedef typename MF<T>::v4 v4;
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ double s_red[2][4];
    const int nx = p.nx, nu = p.nu;
    const T* pz = (const T*)bf.z0;  // p
    const T* zp = (const T*)bf.z1;  // z+
    const T* d = (const T*)bf.e0;   // eta
    glbp<T> eo = (glbp<T>)bf.e1;    // eta+
    glbp<T> xi2 = (glbp<T>)xi2_;
    const int bid = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
    const int lo = lane & 15, h = lane >> 4;
    const crec4* tab = (const crec4*)p.cp2_tab;
    StgB st{(ldsd*)smem_, 0, stg_table()};
    double m2 = 0.0, m5 = 0.0;
    T alpha = T(0), ra = T(0);  // alpha and 1 / alpha (products instead of divisions: 1 ulp)
    auto finish = [&](int e, T dv, T v, T pv, T b) {
        const T ep = alpha * (v - pv);
        eo[e] = ep;
        const T x2 = (dv - ep) * ra + b;
        xi2[e] = x2;
        m2 = nmax(m2, (double)fabs(x2));
        m5 = nmax(m5, (double)fabs(ep - dv));
    };
    if (bid < nbF) {
        const Rec t0 = tab[kCpFamRecs * bid], t1 = tab[kCpFamRecs * bid + 1], t2 = tab[kCpFamRecs * bid + 2];
        const int i0 = t1.z, i1 = t1.w, P = i1 - i0;
        const int cb = t0.x, ce = t0.y, C = ce - cb, y0 = t0.z, Y = t0.w - t0.z, e7a = t1.x, E7n = t1.y - t1.x;
        const ldsp<T> Xz = st.arr(zp + p.X0 + (size_t)i0 * nx, P * nx);
        const ldsp<T> Xp = st.arr(pz + p.X0 + (size_t)i0 * nx, P * nx);
        const ldsp<T> Uz = st.arr(zp + p.U0 + (size_t)i0 * nu, P * nu);
        const ldsp<T> Up = st.arr(pz + p.U0 + (size_t)i0 * nu, P * nu);
        const ldsp<T> Yz = st.arr(zp + p.Y0 + y0, Y);
        const ldsp<T> Yp = st.arr(pz + p.Y0 + y0, Y);
        const ldsp<T> Sz = st.arr(zp + p.S0 + i0, P);
        const ldsp<T> Sp = st.arr(pz + p.S0 + i0, P);
        const ldsp<T> Tz = st.arr(zp + p.T0 + cb, C);
        const ldsp<T> Tp = st.arr(pz + p.T0 + cb, C);
        const ldsp<T> CD = st.arr((const T*)p.cond + cb, C);
        const ldsp<T> D1 = st.arr(d + p.E1 + y0, Y);
        const ldsp<T> D2 = st.arr(d + p.E2 + i0, P);
        const ldsp<T> D7 = st.arr(d + e7a, E7n);
        const ldsp<T> D3 = st.arr(d + e3(p, cb), C * nx);
        const ldsp<T> D4 = st.arr(d + e4(p, cb), C * nu);
        const ldsp<T> D5 = st.arr(d + p.E5 + cb, C);
        const ldsp<T> D6 = st.arr(d + p.E6 + cb, C);
        const ldsp<Rec> FR = st.arr(p.frec + i0, P);  // {yrel, nch, ch_start, e7off}
        const ldsp<Rec> CR = st.arr(p.crec + cb, C);  // {anc, iSQ, iSR, 0}
        const ldsp<int> BI = st.arr(p.iBnl + i0, P);
        const int nBx = p.nBnl * (nx + nu);
        const ldsp<T> BL = st.arr((const T*)p.blo_nl, nBx);
        const ldsp<T> BH = st.arr((const T*)p.bhi_nl, nBx);
        st.issue();
        const int tq = t2.x, tr = t2.y;
        WFr<T, RTX> wq;
        WFr<T, RTU> wr;
        if (tq >= 0) wq.load((const T*)p.SQ, tq, nx);  // while the gather is in flight
        if (tr >= 0) wr.load((const T*)p.SR, tr, nu);
        const int done = ctl->done;
        alpha = (T)ctl->alpha;
        ra = T(1) / alpha;
        dma_wait();
        lds_sync();
        if (done) return;
        // (1) child tiles: eta3 (nx), eta4 (nu), eta5, eta6 -> one SOC of dim nx + nu + 2
        const int ntc = (C + 15) >> 4;
        for (int t = wv; t < ntc; t += nw) {
            const int j0 = 16 * t, ja = j0 + lo;
            const bool la = ja < C;
            const int ax0 = la ? (CR[ja].x - i0) : 0;
            v4 ax[RTX], bx[RTX], au[RTU], bu[RTU];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) ax[r] = bx[r] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int r = 0; r < RTU; ++r) au[r] = bu[r] = v4{0, 0, 0, 0};
            if (tq >= 0) {
                tile2<T, RTX>(wq, nx, [&](int k, T& a1, T& a2) {
                    if (la) {
                        const T z = Xz[ax0 * nx + k], q = Xp[ax0 * nx + k];
                        a1 = T(2) * z - q;
                        a2 = z - q;
                    }
                }, ax, bx);
            }
            if (tr >= 0) {
                tile2<T, RTU>(wr, nu, [&](int k, T& a1, T& a2) {
                    if (la) {
                        const T z = Uz[ax0 * nu + k], q = Up[ax0 * nu + k];
                        a1 = T(2) * z - q;
                        a2 = z - q;
                    }
                }, au, bu);
            }
            // epilogue: the SOC of each of this lane group's 4 children
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                const int jn = j0 + MF<T>::row(h, e);
                const bool live = jn < C;
                const int j = cb + jn;
                T vx[RTX], vu[RTU];
                T ss = T(0);
                _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt) {
                    const int r = 16 * rt + lo;
                    vx[rt] = T(0);
                    if (live && r < nx) {
                        const T dv = D3[jn * nx + r];
                        vx[rt] = (dv + alpha * ax[rt][e]) * ra;
                        ss += vx[rt] * vx[rt];
                    }
                }
                _Pragma("unroll") for (int rt = 0; rt < RTU; ++rt) {
                    const int r = 16 * rt + lo;
                    vu[rt] = T(0);
                    if (live && r < nu) {
                        const T dv = D4[jn * nu + r];
                        vu[rt] = (dv + alpha * au[rt][e]) * ra;
                        ss += vu[rt] * vu[rt];
                    }
                }
                ss = sum16(ss);
                T d5 = T(0), d6 = T(0), a5 = T(0), b5 = T(0);
                if (live) {
                    d5 = D5[jn];
                    d6 = D6[jn];
                    const T zt = Tz[jn], pt = Tp[jn];
                    a5 = T(0.5) * (T(2) * zt - pt);
                    b5 = T(0.5) * (zt - pt);
                }
                const T v5 = (d5 + alpha * a5) * ra + T(-0.5);
                const T v6 = (d6 + alpha * a5) * ra + T(0.5);
                ss += v5 * v5;
                const T nf = sqrt(ss), tt = v6;
                if (live) {
                    _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt) {
                        const int r = 16 * rt + lo;
                        if (r < nx) finish(e3(p, j) + r, D3[jn * nx + r], vx[rt], soc_apply_t(vx[rt], false, nf, tt),
                                           bx[rt][e]);
                    }
                    _Pragma("unroll") for (int rt = 0; rt < RTU; ++rt) {
                        const int r = 16 * rt + lo;
                        if (r < nu) finish(e4(p, j) + r, D4[jn * nu + r], vu[rt], soc_apply_t(vu[rt], false, nf, tt),
                                           bu[rt][e]);
                    }
                    if (lo == 0) finish(p.E5 + j, d5, v5, soc_apply_t(v5, false, nf, tt), b5);
                    if (lo == 1) finish(p.E6 + j, d6, v6, soc_apply_t(v6, true, nf, tt), b5);
                }
            }
        }
        // (2) parent rows eta1 (2c+1), eta2, eta7 (nx+nu): lanes over rows
        {
            const int G = 2 * p.cmax + 2 + nx + nu, per = blockDim.x / G;
            const int gl = tid / G, r = tid - gl * G;
            for (int q0 = 0; q0 < P; q0 += per) {
                const int ii = q0 + gl, i = i0 + ii;
                if (!(gl < per && ii < P)) continue;
                const Rec fr = FR[ii];
                const int c = fr.y, yo = fr.x - y0, cl = fr.z - cb;
                if (r < 2 * c + 1) {
                    const T zy = Yz[yo + r], py = Yp[yo + r];
                    const T av = T(2) * zy - py, bb = zy - py;
                    const T dv = D1[yo + r];
                    const T v = (dv + alpha * av) * ra;
                    finish(p.E1 + fr.x + r, dv, v, r < 2 * c ? fmax(v, T(0)) : v, bb);
                } else if (r == 2 * p.cmax + 1) {
                    T bya = T(0), byb = T(0);
                    for (int k = 0; k < c; ++k) {
                        const T cp = CD[cl + k];
                        bya = fma(cp, T(2) * Yz[yo + k] - Yp[yo + k], bya);
                        byb = fma(cp, Yz[yo + k] - Yp[yo + k], byb);
                    }
                    bya += T(2) * Yz[yo + 2 * c] - Yp[yo + 2 * c];
                    byb += Yz[yo + 2 * c] - Yp[yo + 2 * c];
                    const T zs = Sz[ii], ps = Sp[ii];
                    const T av = (T(2) * zs - ps) - bya, bb = (zs - ps) - byb;
                    const T dv = D2[ii];
                    const T v = (dv + alpha * av) * ra;
                    finish(p.E2 + i, dv, v, fmax(v, T(0)), bb);
                } else if (r >= 2 * p.cmax + 2 && fr.w >= 0) {
                    const int rr = r - (2 * p.cmax + 2);
                    const T zv = rr < nx ? Xz[ii * nx + rr] : Uz[ii * nu + rr - nx];
                    const T pv_ = rr < nx ? Xp[ii * nx + rr] : Up[ii * nu + rr - nx];
                    const T av = T(2) * zv - pv_, bb = zv - pv_;
                    const T dv = D7[fr.w - e7a + rr];
                    const T v = (dv + alpha * av) * ra;
                    const int bi = BI[ii];
                    finish(fr.w + rr, dv, v, box_apply_t(v, BL[bi * (nx + nu) + rr], BH[bi * (nx + nu) + rr], ctl), bb);
                }
            }
        }
    } else {
        // leaves [l0, l1): eta11 (nx), eta12, eta13 -> SOC of dim nx + 2; eta14 (nx) box
        const int lb = bid - nbF;
        const Rec t0 = tab[kCpFamRecs * nbF + kCpLeafRecs * lb], t1 = tab[kCpFamRecs * nbF + kCpLeafRecs * lb + 1];
        const int l0 = t0.z, l1 = t0.w, Lc = l1 - l0;
        const int e14a = t0.x, E14n = t0.y - t0.x;
        const ldsp<T> Xz = st.arr(zp + p.X0 + (size_t)l0 * nx, Lc * nx);
        const ldsp<T> Xp = st.arr(pz + p.X0 + (size_t)l0 * nx, Lc * nx);
        const ldsp<T> Sz = st.arr(zp + p.S0 + l0, Lc);
        const ldsp<T> Sp = st.arr(pz + p.S0 + l0, Lc);
        const ldsp<T> D11 = st.arr(d + e11(p, l0), Lc * nx);
        const ldsp<T> D12 = st.arr(d + p.E12 + l0, Lc);
        const ldsp<T> D13 = st.arr(d + p.E13 + l0, Lc);
        const ldsp<T> D14 = st.arr(d + e14a, E14n);
        const ldsp<Rec> LR = st.arr(p.lrec + (l0 - p.m), Lc);  // {iSP, iBl, e14off, 0}
        const int nBx = p.nBl * nx;
        const ldsp<T> BL = st.arr((const T*)p.blo_l, nBx);
        const ldsp<T> BH = st.arr((const T*)p.bhi_l, nBx);
        st.issue();
        const int tp = t1.x;
        WFr<T, RTX> wp;
        if (tp >= 0) wp.load((const T*)p.SP, tp, nx);
        const int done = ctl->done;
        alpha = (T)ctl->alpha;
        ra = T(1) / alpha;
        dma_wait();
        lds_sync();
        if (done) return;
        const int ntl = (Lc + 15) >> 4;
        for (int t = wv; t < ntl; t += nw) {
            const int q0 = 16 * t, qa = q0 + lo;
            const bool la = qa < Lc;
            v4 ax[RTX], bx[RTX];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) ax[r] = bx[r] = v4{0, 0, 0, 0};
            if (tp >= 0) {
                tile2<T, RTX>(wp, nx, [&](int k, T& a1, T& a2) {
                    if (la) {
                        const T z = Xz[qa * nx + k], q = Xp[qa * nx + k];
                        a1 = T(2) * z - q;
                        a2 = z - q;
                    }
                }, ax, bx);
            }
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                const int qn = q0 + MF<T>::row(h, e);
                const bool live = qn < Lc;
                const int l = l0 + qn;
                T vx[RTX];
                T ss = T(0);
                _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt) {
                    const int r = 16 * rt + lo;
                    vx[rt] = T(0);
                    if (live && r < nx) {
                        vx[rt] = (D11[qn * nx + r] + alpha * ax[rt][e]) * ra;
                        ss += vx[rt] * vx[rt];
                    }
                }
                ss = sum16(ss);
                T d12 = T(0), d13 = T(0), a5 = T(0), b5 = T(0);
                Rec lr = {0, 0, -1, 0};
                if (live) {
                    d12 = D12[qn];
                    d13 = D13[qn];
                    const T zs = Sz[qn], ps = Sp[qn];
                    a5 = T(0.5) * (T(2) * zs - ps);
                    b5 = T(0.5) * (zs - ps);
                    lr = LR[qn];
                }
                const T v12 = (d12 + alpha * a5) * ra + T(-0.5);
                const T v13 = (d13 + alpha * a5) * ra + T(0.5);
                ss += v12 * v12;
                const T nf = sqrt(ss), tt = v13;
                if (live) {
                    _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt) {
                        const int r = 16 * rt + lo;
                        if (r < nx) {
                            finish(e11(p, l) + r, D11[qn * nx + r], vx[rt], soc_apply_t(vx[rt], false, nf, tt), bx[rt][e]);
                            if (lr.z >= 0) {  // eta14 = x (box)
                                const T zv = Xz[qn * nx + r], pv_ = Xp[qn * nx + r];
                                const T dv = D14[lr.z - e14a + r];
                                const T v = (dv + alpha * (T(2) * zv - pv_)) * ra;
                                finish(lr.z + r, dv, v, box_apply_t(v, BL[lr.y * nx + r], BH[lr.y * nx + r], ctl), zv - pv_);
                            }
                        }
                    }
                    if (lo == 0) finish(p.E12 + l, d12, v12, soc_apply_t(v12, false, nf, tt), b5);
                    if (lo == 1) finish(p.E13 + l, d13, v13, soc_apply_t(v13, true, nf, tt), b5);
                }
            }
        }
    }
    double* prow = part + (size_t)bid * 6;
    blk_max_store(m2, prow + 2, s_red[0]);
    blk_max_store(m5, prow + 5, s_red[1]);
}

// ==============================================================================
// k_cpp2 — next primal half step from eta+ (and the finished iteration's residuals):
//   out = z+ - alpha L^T(eta+), s_0 -= alpha, kernel projection of (y, tau, s);
//   xi1 = (p - z+)/alpha - L^T(d - eta+), xi0 = xi1 + L^T xi2, delta1 = z+ - p,
//   delta0 = delta1 + L^T(d - eta+)
// Buffers: p = z0, z+ = z1, out = z2, d = e0, eta+ = e1.
// ==============================================================================
template <class T, int RTX, int RTU>
__global__ void __launch_bounds__(256) k_cpp2(Dev p, Ctl* __restrict__ ctl, Bufs bf, const double* __restrict__ xi2_,
                                              double* __restrict__ part, int nbF) {
    typedef typename MF<T>::v4 v4;
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ double s_red[4][4];
    __shared__ T s_x[256];
    const int nx = p.nx, nu = p.nu;
    const T* pz = (const T*)bf.z0;  // p_prev
    const T* zp = (const T*)bf.z1;  // z+ (also where the half step starts)
    glbp<T> out = (glbp<T>)bf.z2;
    const T* dP = (const T*)bf.e0;  // d_prev
    const T* dA = (const T*)bf.e1;  // eta+
    const T* xg = (const T*)xi2_;
    const int bid = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
    const int lo = lane & 15, h = lane >> 4;
    const crec4* tab = (const crec4*)p.cp2_tab;
    StgB st{(ldsd*)smem_, 0, stg_table()};
    double m0 = 0.0, m1 = 0.0, m3 = 0.0, m4 = 0.0;
    T alpha = T(0), ra = T(0);
    // residual terms of one primal entry: pp = p, zz = z+, w = L^T(d - eta+), lc = L^T xi2
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
    if (bid < nbF) {
        const Rec t0 = tab[kCpFamRecs * bid], t1 = tab[kCpFamRecs * bid + 1], t2 = tab[kCpFamRecs * bid + 2];
        const int i0 = t1.z, i1 = t1.w, P = i1 - i0;
        const int cb = t0.x, ce = t0.y, C = ce - cb, y0 = t0.z, Y = t0.w - t0.z, e7a = t1.x, E7n = t1.y - t1.x;
        // three duals (0: eta+, 1: d_prev, 2: xi2) over the family's ranges
        const T* dsrc[3] = {dA, dP, xg};
        ldsp<T> D1[3], D2[3], D2c[3], D3[3], D4[3], D5[3], D6[3], D7[3], Dc12[3], Dc13[3];
        _Pragma("unroll") for (int a = 0; a < 3; ++a) {
            const T* s = dsrc[a];
            D1[a] = st.arr(s + p.E1 + y0, Y);
            D2[a] = st.arr(s + p.E2 + i0, P);
            D3[a] = st.arr(s + e3(p, cb), C * nx);
            D4[a] = st.arr(s + e4(p, cb), C * nu);
            D5[a] = st.arr(s + p.E5 + cb, C);
            D6[a] = st.arr(s + p.E6 + cb, C);
            D7[a] = st.arr(s + e7a, E7n);
            D2c[a] = st.arr(s + p.E2 + cb, C);    // s_j of nonleaf children: eta2_j
            Dc12[a] = st.arr(s + p.E12 + cb, C);  // s_j of leaf children: (eta12_j + eta13_j) / 2
            Dc13[a] = st.arr(s + p.E13 + cb, C);
        }
        const ldsp<T> Xz = st.arr(zp + p.X0 + (size_t)i0 * nx, P * nx);
        const ldsp<T> Xp = st.arr(pz + p.X0 + (size_t)i0 * nx, P * nx);
        const ldsp<T> Uz = st.arr(zp + p.U0 + (size_t)i0 * nu, P * nu);
        const ldsp<T> Up = st.arr(pz + p.U0 + (size_t)i0 * nu, P * nu);
        const ldsp<T> Yz = st.arr(zp + p.Y0 + y0, Y);
        const ldsp<T> Yp = st.arr(pz + p.Y0 + y0, Y);
        const ldsp<T> Tz = st.arr(zp + p.T0 + cb, C);
        const ldsp<T> Tp = st.arr(pz + p.T0 + cb, C);
        const ldsp<T> Scz = st.arr(zp + p.S0 + cb, C);
        const ldsp<T> Scp = st.arr(pz + p.S0 + cb, C);
        const ldsp<T> CD = st.arr((const T*)p.cond + cb, C);
        const ldsp<T> AR = st.arr((const T*)p.alpha_r + i0, P);
        const ldsp<Rec> FR = st.arr(p.frec + i0, P);  // {yrel, nch, ch_start, e7off}
        const ldsp<Rec> CR = st.arr(p.crec + cb, C);  // {anc, iSQ, iSR, 0}
        st.issue();
        const int tq = t2.x, tr = t2.y, creg = t2.z;
        WFr<T, RTX> wq;
        WFr<T, RTU> wr;
        if (tq >= 0) wq.load((const T*)p.SQ, tq, nx);
        if (tr >= 0) wr.load((const T*)p.SR, tr, nu);
        const int done = ctl->done;
        alpha = (T)ctl->alpha;
        ra = T(1) / alpha;
        dma_wait();
        lds_sync();
        if (done) return;
        // the parent row (x or u, row r of parent q) from its children's product sums
        // (sA: eta+, sW: d - eta+, sC: xi2, in child order) plus Gamma' eta7
        auto xu_row = [&](int q, bool isx, int r, T sA, T sW, T sC) {
            const Rec fr = FR[q];
            T accA = T(0), accW = T(0), accC = T(0);
            if (fr.w >= 0) {
                const int o = fr.w - e7a + (isx ? r : nx + r);
                accA = D7[0][o];
                accW = D7[1][o] - D7[0][o];
                accC = D7[2][o];
            }
            accA += sA;
            accW += sW;
            accC += sC;
            const int e = isx ? p.X0 + (i0 + q) * nx + r : p.U0 + (i0 + q) * nu + r;
            const T zz = isx ? Xz[q * nx + r] : Uz[q * nu + r];
            const T pp = isx ? Xp[q * nx + r] : Up[q * nu + r];
            out[e] = zz - alpha * accA;
            account(pp, zz, accW, accC);
        };
        // (1) x / u rows
        if (creg > 0 && tq >= 0 && tr >= 0) {
            // regular block: per-parent tiles (4 (4 / c) parents per tile); x rows, then u rows
            const int Q = 4 / creg, PT = 4 * Q;
            const int hA = MF<T>::h_of(lo), eA = MF<T>::e_of(lo);
            const int pA = hA + 4 * (eA / creg), kA = eA % creg;
            const int ntp = (P + PT - 1) / PT;
            auto pass = [&](auto rtc, const auto& wf, int n, const ldsp<T>(&DD)[3], bool isx) {
                constexpr int RT = decltype(rtc)::value;
                for (int t = wv; t < ntp; t += nw) {
                    const int pb = t * PT;
                    const bool la = eA < Q * creg && pb + pA < P;
                    const int ja = la ? (pb + pA) * creg + kA : 0;  // block-local child of this lane's A row
                    v4 cA[RT], cW[RT], cC[RT];
                    _Pragma("unroll") for (int r = 0; r < RT; ++r) cA[r] = cW[r] = cC[r] = v4{0, 0, 0, 0};
                    tile3<T, RT>(wf, n, [&](int k, T& a1, T& a2, T& a3) {
                        if (la) {
                            const T va = DD[0][ja * n + k];
                            a1 = va;
                            a2 = DD[1][ja * n + k] - va;
                            a3 = DD[2][ja * n + k];
                        }
                    }, cA, cW, cC);
                    // element e of this lane is child e % c of parent h + 4 (e / c): the sums of
                    // parent slot s add the elements with e / c == s, in child order
                    _Pragma("unroll") for (int sl = 0; sl < 4; ++sl) {
                        const int q = pb + h + 4 * sl;
                        if (sl >= Q || q >= P) continue;
                        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
                            const int r = 16 * rt + lo;
                            if (r >= n) continue;
                            T sA = T(0), sW = T(0), sC = T(0);
                            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                                if (e / creg == sl && e < Q * creg) {
                                    sA += cA[rt][e];
                                    sW += cW[rt][e];
                                    sC += cC[rt][e];
                                }
                            }
                            xu_row(q, isx, r, sA, sW, sC);
                        }
                    }
                }
            };
            pass(std::integral_constant<int, RTX>{}, wq, nx, D3, true);
            pass(std::integral_constant<int, RTU>{}, wr, nu, D4, false);
        } else {
            // irregular block: child products into LDS (3 duals), then per-parent sums
            typedef __attribute__((address_space(3))) T lT;
            lT* PX = (lT*)((__attribute__((address_space(3))) char*)smem_ + st.o);
            lT* PU = PX + 3 * C * nx;
            const int ntc = (C + 15) >> 4;
            auto prod = [&](auto rtc, const auto& wf, int tu, int n, const T* tabs, int which, const ldsp<T>(&DD)[3],
                            lT* PO) {
                constexpr int RT = decltype(rtc)::value;
                for (int t = wv; t < ntc; t += nw) {
                    const int j0 = 16 * t, ja = j0 + lo;
                    const bool la = ja < C;
                    v4 cc[3][RT];
                    {
                        _Pragma("unroll") for (int r = 0; r < RT; ++r) cc[0][r] = cc[1][r] = cc[2][r] = v4{0, 0, 0, 0};
                        tile3<T, RT>(wf, n, [&](int k, T& a1, T& a2, T& a3) {
                            if (la) {
                                const T va = DD[0][ja * n + k];
                                a1 = va;
                                a2 = DD[1][ja * n + k] - va;
                                a3 = DD[2][ja * n + k];
                            }
                        }, cc[0], cc[1], cc[2]);
                    }
                    _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                        const int jn = j0 + MF<T>::row(h, e);
                        if (jn >= C) continue;
                        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
                            const int r = 16 * rt + lo;
                            if (r < n)
                                _Pragma("unroll") for (int a = 0; a < 3; ++a) PO[(a * C + jn) * n + r] = cc[a][rt][e];
                        }
                    }
                }
            };
            prod(std::integral_constant<int, RTX>{}, wq, tq, nx, (const T*)p.SQ, 0, D3, PX);
            prod(std::integral_constant<int, RTU>{}, wr, tr, nu, (const T*)p.SR, 1, D4, PU);
            lds_sync();
            for (int e = tid; e < P * (nx + nu); e += blockDim.x) {
                const int q = e / (nx + nu), rr = e - q * (nx + nu);
                const bool isx = rr < nx;
                const int r = isx ? rr : rr - nx, n_ = isx ? nx : nu;
                const lT* PP = isx ? PX : PU;
                const Rec fr = FR[q];
                T sA = T(0), sW = T(0), sC = T(0);
                for (int jj = fr.z - cb; jj < fr.z - cb + fr.y; ++jj) {
                    sA += PP[(0 * C + jj) * n_ + r];
                    sW += PP[(1 * C + jj) * n_ + r];
                    sC += PP[(2 * C + jj) * n_ + r];
                }
                xu_row(q, isx, r, sA, sW, sC);
            }
        }
        // (2) y, tau, s rows and the AVaR kernel projection (cache.py:290-317, closed form:
        // r_k = alpha_r y_k - y_{c+k} + y_{2c} - tau_k - s_k, w = (r - 1 sum(r) / (a + c)) / a,
        // a = alpha_r^2 + 3; y_k -= alpha_r w_k, y_{c+k} += w_k, y_{2c} -= sum(w), tau_k += w_k,
        // s_k += w_k). Lane rk < cmax: child rk; rk == cmax: y_2c (and the root's s_0).
        {
            const int cmax = p.cmax, G = cmax + 1, per = blockDim.x / G;
            const int gl = tid / G, rk = tid - gl * G, kb = gl * G;
            for (int q0 = 0; q0 < P; q0 += per) {
                const int ii = q0 + gl, i = i0 + ii;
                const bool live = gl < per && ii < P;
                Rec fr = {0, 0, 0, -1};
                if (live) fr = FR[ii];
                const int c = fr.y, cl = fr.z - cb, yo = fr.x - y0;
                T vals[4] = {T(0), T(0), T(0), T(0)};
                T y2c = T(0);
                const T e2A = live ? D2[0][ii] : T(0);
                T e2W = T(0), e2C = T(0);
                if (live) {
                    e2W = D2[1][ii] - D2[0][ii];
                    e2C = D2[2][ii];
                }
                if (live && rk < c) {
                    const int jj = cl + rk, j = cb + jj;
                    const T b = CD[jj];
                    const int f0 = yo + rk, f1 = yo + c + rk;
                    const T lt0 = D1[0][f0] - b * e2A, lt1 = D1[0][f1] - T(0) * e2A;
                    vals[0] = Yz[f0] - alpha * lt0;
                    vals[1] = Yz[f1] - alpha * lt1;
                    const T ltt = T(0.5) * (D5[0][jj] + D6[0][jj]);
                    vals[2] = Tz[jj] - alpha * ltt;
                    const T lts = j < p.m ? D2c[0][jj] : T(0.5) * (Dc12[0][jj] + Dc13[0][jj]);
                    vals[3] = Scz[jj] - alpha * lts;
                    const T w0 = (D1[1][f0] - D1[0][f0]) - b * e2W, c0 = D1[2][f0] - b * e2C;
                    const T w1 = (D1[1][f1] - D1[0][f1]) - T(0) * e2W, c1 = D1[2][f1] - T(0) * e2C;
                    const T wt = T(0.5) * ((D5[1][jj] - D5[0][jj]) + (D6[1][jj] - D6[0][jj]));
                    const T ct = T(0.5) * (D5[2][jj] + D6[2][jj]);
                    T ws, cs2;
                    if (j < p.m) {
                        ws = D2c[1][jj] - D2c[0][jj];
                        cs2 = D2c[2][jj];
                    } else {
                        ws = T(0.5) * ((Dc12[1][jj] - Dc12[0][jj]) + (Dc13[1][jj] - Dc13[0][jj]));
                        cs2 = T(0.5) * (Dc12[2][jj] + Dc13[2][jj]);
                    }
                    account(Yp[f0], Yz[f0], w0, c0);
                    account(Yp[f1], Yz[f1], w1, c1);
                    account(Tp[jj], Tz[jj], wt, ct);
                    account(Scp[jj], Scz[jj], ws, cs2);
                }
                if (live && rk == cmax) {
                    const int f2 = yo + 2 * c;
                    y2c = Yz[f2] - alpha * (D1[0][f2] - T(1) * e2A);
                    account(Yp[f2], Yz[f2], (D1[1][f2] - D1[0][f2]) - T(1) * e2W, D1[2][f2] - T(1) * e2C);
                    if (i == 0) {
                        // root s_0: L^T -> eta2_0; then the relaxation prox s_0 -= alpha (cache.py:253-257)
                        const T z0s = zp[p.S0], p0s = pz[p.S0];
                        out[p.S0] = (z0s - alpha * e2A) - alpha;
                        account(p0s, z0s, e2W, e2C);
                    }
                }
                const bool mine = live && rk <= cmax;
                const T al = live ? AR[ii] : T(0);
                if (mine && rk == cmax) s_x[kb + cmax] = y2c;
                __syncthreads();
                T rkv = T(0);
                if (live && rk < c) rkv = al * vals[0] - vals[1] + s_x[kb + cmax] - vals[2] - vals[3];
                __syncthreads();
                if (mine && rk < cmax) s_x[kb + rk] = rkv;
                __syncthreads();
                T sr = T(0);
                if (mine) for (int q = 0; q < c; ++q) sr += s_x[kb + q];
                const T a = al * al + T(3);
                T w = T(0);
                if (live && rk < c) w = (rkv - sr / (a + (T)c)) / a;
                __syncthreads();
                if (mine && rk < cmax) s_x[kb + rk] = w;
                __syncthreads();
                if (live && rk < c) {
                    vals[0] -= al * w;
                    vals[1] += w;
                    vals[2] += w;
                    vals[3] += w;
                }
                if (live && rk == cmax) {
                    T sw = T(0);
                    for (int q = 0; q < c; ++q) sw += s_x[kb + q];
                    y2c -= sw;
                }
                __syncthreads();
                if (live && rk < c) {
                    const int j = cb + cl + rk;
                    out[p.Y0 + fr.x + rk] = vals[0];
                    out[p.Y0 + fr.x + c + rk] = vals[1];
                    out[p.T0 + j] = vals[2];
                    out[p.S0 + j] = vals[3];
                }
                if (live && rk == cmax) out[p.Y0 + fr.x + 2 * c] = y2c;
            }
        }
    } else {
        // leaves: x = sqrtPf eta11 + eta14 for the three duals
        const int lb = bid - nbF;
        const Rec t0 = tab[kCpFamRecs * nbF + kCpLeafRecs * lb], t1 = tab[kCpFamRecs * nbF + kCpLeafRecs * lb + 1];
        const int l0 = t0.z, l1 = t0.w, Lc = l1 - l0;
        const int e14a = t0.x, E14n = t0.y - t0.x;
        const T* dsrc[3] = {dA, dP, xg};
        ldsp<T> D11[3], D14[3];
        _Pragma("unroll") for (int a = 0; a < 3; ++a) {
            D11[a] = st.arr(dsrc[a] + e11(p, l0), Lc * nx);
            D14[a] = st.arr(dsrc[a] + e14a, E14n);
        }
        const ldsp<T> Xz = st.arr(zp + p.X0 + (size_t)l0 * nx, Lc * nx);
        const ldsp<T> Xp = st.arr(pz + p.X0 + (size_t)l0 * nx, Lc * nx);
        const ldsp<Rec> LR = st.arr(p.lrec + (l0 - p.m), Lc);
        st.issue();
        const int tp = t1.x;
        WFr<T, RTX> wp;
        if (tp >= 0) wp.load((const T*)p.SP, tp, nx);
        const int done = ctl->done;
        alpha = (T)ctl->alpha;
        ra = T(1) / alpha;
        dma_wait();
        lds_sync();
        if (done) return;
        const int ntl = (Lc + 15) >> 4;
        for (int t = wv; t < ntl; t += nw) {
            const int q0 = 16 * t, qa = q0 + lo;
            const bool la = qa < Lc;
            v4 c3[3][RTX];
            if (tp >= 0) {
                _Pragma("unroll") for (int r = 0; r < RTX; ++r) c3[0][r] = c3[1][r] = c3[2][r] = v4{0, 0, 0, 0};
                tile3<T, RTX>(wp, nx, [&](int k, T& a1, T& a2, T& a3) {
                    if (la) {
                        const T va = D11[0][qa * nx + k];
                        a1 = va;
                        a2 = D11[1][qa * nx + k] - va;
                        a3 = D11[2][qa * nx + k];
                    }
                }, c3[0], c3[1], c3[2]);
            }
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                const int qn = q0 + MF<T>::row(h, e);
                if (qn >= Lc) continue;
                const Rec lr = LR[qn];
                _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt) {
                    const int r = 16 * rt + lo;
                    if (r >= nx) continue;
                    T sA = c3[0][rt][e], sW = c3[1][rt][e], sC = c3[2][rt][e];
                    if (lr.z >= 0) {
                        const int q = lr.z - e14a + r;
                        sA += D14[0][q];
                        sW += D14[1][q] - D14[0][q];
                        sC += D14[2][q];
                    }
                    const T zz = Xz[qn * nx + r], pp = Xp[qn * nx + r];
                    out[p.X0 + (size_t)(l0 + qn) * nx + r] = zz - alpha * sA;
                    account(pp, zz, sW, sC);
                }
            }
        }
    }
    double* prow = part + (size_t)bid * 6;
    blk_max_store(m0, prow + 0, s_red[0]);
    blk_max_store(m1, prow + 1, s_red[1]);
    blk_max_store(m3, prow + 3, s_red[2]);
    blk_max_store(m4, prow + 4, s_red[3]);
}
