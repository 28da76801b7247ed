// raocp_ell3.hip — L (operators.py:19-53) as streaming wave tasks: no LDS, no block
// barriers. A wave takes 16-node tiles in a grid-stride loop and loads each tile's A rows
// (a node vector is contiguous) straight into registers: with the MFMA k index permuted to
// k = KC h + s (KC = ceil(n / 4) steps, h = lane >> 4), lane (lo, h) needs the KC
// consecutive entries x[KC h .. KC h + KC) of its node, i.e. whole 16-B vector loads; the
// weight fragments use the same permutation and stay in registers while consecutive tiles
// share a table. Included by raocp_kernels.hip after raocp_cp2.hip (namespace raocp).
//
// Tasks (computed from the task index, no table):
//   [0, Tc)          child tiles: eta3_j = sqrtQ x_anc(j), eta4_j = sqrtR u_anc(j), eta5 = eta6 = tau/2
//   [Tc, Tc + Tl)    leaf tiles: eta11_l = sqrtPf x_l, eta12 = eta13 = s_l / 2, eta14_l = x_l
//   [.., + Tp)       parent chunks of 64 rows of the flat list [eta7 rows | eta1 | eta2]

// waves per SIMD the compiler budgets k_ell3 / k_ellt3's registers for (build-time
// -DELL3_WPE=...): 3 = at most 168 registers (<double, 32, 12>: 146, no spills, from 156 + 24
// AGPRs at two waves); nx = 64 asks for two waves in fp32 and none in fp64 (its tiles spill
// at 168 and 256 registers)
#ifndef ELL3_WPE
#define ELL3_WPE 3
#endif
// output stores of k_ell3 (ELL3_NT) / k_ellt3 (ELLT3_NT): 1 = nontemporal (the rows are
// streamed out, never re-read by the launch). Measured over rotating HBM-sized buffer sets
// (profiles/r05/l_sweep_variants.log): L^T at config 4 27.1 -> 22.7 us with nontemporal
// stores (config 5 unchanged), L 27.5 -> 38.4 us (its 16-node tiles replicated to the C
// children through the per-wave LDS image): on for L^T only
#ifndef ELL3_NT
#define ELL3_NT 0
#endif
#ifndef ELLT3_NT
#define ELLT3_NT 1
#endif
template <bool NT, class P, class V>
__device__ __forceinline__ void ostn(P* p, V v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <class P, class V>
__device__ __forceinline__ void ost(P* p, V v) {
    ostn<ELL3_NT != 0>(p, v);
}
#ifndef ELL3_WPE64
#define ELL3_WPE64 2
#endif
#define ELL3_WPE_OF(T, NX) ((NX) >= 64 ? (sizeof(T) == 8 ? 1 : ELL3_WPE64) : ELL3_WPE)
// weights of one table, k-permuted: b[rt][s] = M[row 16 rt + lo][KC h + s]; R rows, K cols
template <class T, int R, int K>
struct WPerm {
    static constexpr int RT = (R + 15) / 16, KC = (K + 3) / 4;
    T b[RT][KC];
    int t = -1;
    __device__ __forceinline__ void load(const T* tab, int t_) {
        t = t_;
        const int l = threadIdx.x & 63, lo = l & 15, h = l >> 4;
        cglbp<T> M = (cglbp<T>)(tab + (size_t)t_ * R * K);
        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
            _Pragma("unroll") for (int s = 0; s < KC; ++s) {
                const int r = 16 * rt + lo, k = KC * h + s;
                b[rt][s] = (r < R && k < K) ? M[k * R + r] : T(0);
            }
        }
    }
};

// 16-B vectors of T at 4- / 8-B alignment (rows and output tiles start wherever the
// reference's flat layout puts them; gfx950 global memory takes unaligned vector accesses)
template <class T>
struct Vec16 {
    static constexpr int V = 16 / (int)sizeof(T);
    typedef T type __attribute__((ext_vector_type(16 / sizeof(T)), aligned(sizeof(T))));
};

// A values of a lane: a[s] = v[KC h + s] for k < K (v a global row pointer or null)
template <class T, int K>
__device__ __forceinline__ void load_arow(cglbp<T> v, T (&a)[(K + 3) / 4]) {
    constexpr int KC = (K + 3) / 4, V = Vec16<T>::V;
    typedef typename Vec16<T>::type vt;
    const int h = (threadIdx.x & 63) >> 4;
    if constexpr (K % 4 == 0 && KC % V == 0) {
        if (v) {  // whole 16-B loads
            _Pragma("unroll") for (int s = 0; s < KC; s += V) {
                const vt w = *(const __attribute__((address_space(1))) vt*)(v + KC * h + s);
                _Pragma("unroll") for (int u = 0; u < V; ++u) a[s + u] = w[u];
            }
        } else {
            _Pragma("unroll") for (int s = 0; s < KC; ++s) a[s] = T(0);
        }
        return;
    }
    if (v && (K % 4 == 0 || h < 3)) {
        _Pragma("unroll") for (int s = 0; s < KC; ++s) a[s] = v[KC * h + s];
    } else {
        _Pragma("unroll") for (int s = 0; s < KC; ++s) a[s] = (v && KC * h + s < K) ? v[KC * h + s] : T(0);
    }
}

// the inverse of load_arow: v[KC h + s] = a[s] for k < K, as 16-B stores where a lane's KC
// values are whole vectors (eta7 / eta14 rows: a lane writes KC consecutive elements of its
// node's row; one element per lane and instruction scattered them over 64 rows)
template <class T, int K>
__device__ __forceinline__ void store_arow(glbp<T> v, const T (&a)[(K + 3) / 4]) {
    constexpr int KC = (K + 3) / 4, V = Vec16<T>::V;
    typedef typename Vec16<T>::type vt;
    const int h = (threadIdx.x & 63) >> 4;
    if constexpr (K % 4 == 0 && KC % V == 0) {
        _Pragma("unroll") for (int s = 0; s < KC; s += V) {
            vt w;
            _Pragma("unroll") for (int u = 0; u < V; ++u) w[u] = a[s + u];
            ost((__attribute__((address_space(1))) vt*)(v + KC * h + s), w);
        }
    } else if constexpr (K % 4 == 0 && V == 2 && KC % 2 == 1) {  // fp64, odd KC (nu = 12): pairs + one
        _Pragma("unroll") for (int s = 0; s + 1 < KC; s += 2) {
            vt w;
            w[0] = a[s];
            w[1] = a[s + 1];
            ost((__attribute__((address_space(1))) vt*)(v + KC * h + s), w);
        }
        v[KC * h + KC - 1] = a[KC - 1];
    } else {
        _Pragma("unroll") for (int s = 0; s < KC; ++s)
            if (KC * h + s < K) v[KC * h + s] = a[s];
    }
}

template <class T, int R, int K>
__device__ __forceinline__ void mma_perm(const WPerm<T, R, K>& w, const T (&a)[(K + 3) / 4],
                                         typename MF<T>::v4 (&acc)[(R + 15) / 16]) {
    _Pragma("unroll") for (int s = 0; s < WPerm<T, R, K>::KC; ++s)
        _Pragma("unroll") for (int rt = 0; rt < WPerm<T, R, K>::RT; ++rt) acc[rt] = MF<T>::mma(a[s], w.b[rt][s], acc[rt]);
}

// store a 16-node x R-row tile (accumulators of RT row tiles) to rows dst + node * R + r of
// a contiguous block, through a per-wave LDS image (row stride R + 1: conflict-free writes)
// so every store instruction writes 64 consecutive elements. rep > 1: every image row is
// stored rep times to consecutive destination rows (cnt image rows -> cnt rep rows)
template <class T, int R>
__device__ __forceinline__ void store_tile(__attribute__((address_space(3))) T* img, const typename MF<T>::v4 (&acc)[(R + 15) / 16],
                                           int cnt, glbp<T> dst, int rep = 1) {
    constexpr int RT = (R + 15) / 16, S = R + 1;
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4;
    _Pragma("unroll") for (int e = 0; e < 4; ++e) {
        const int a = MF<T>::row(h, e);
        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
            const int r = 16 * rt + lo;
            if (r < R) img[a * S + r] = acc[rt][e];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int tot = cnt * rep * R;
    constexpr int V = Vec16<T>::V;
    if constexpr (R % V == 0) {
        // 16 B per lane (a lane's V elements lie in one row): a quarter (fp32) / half (fp64)
        // of the store instructions of one element per lane
        typedef typename Vec16<T>::type vt;
        for (int q = lane * V; q < tot; q += 64 * V) {
            const int a = q / R, r = q - a * R, ia = rep == 1 ? a : a / rep;
            vt w;
            _Pragma("unroll") for (int u = 0; u < V; ++u) w[u] = img[ia * S + r + u];
            ost((__attribute__((address_space(1))) vt*)(dst + q), w);
        }
    } else {
        for (int q = lane; q < tot; q += 64) {
            const int a = q / R, r = q - a * R, ia = rep == 1 ? a : a / rep;
            ost(&dst[q], (T)img[ia * S + r]);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// rows per flat task: L^T 256 (4 per lane, branch-free loads: config 5 L^T 115 -> 111 us),
// L 64 (its eta2 rows walk the children; 256 measured slower: config 5 L 116 -> 135 us,
// profiles/r02_v3/ab_flat.log)
constexpr int kFlatRows = 256, kFlatRowsL = 64;

// eta7 / eta14 offsets of a node. bx (host-built): bits 0-1 nonleaf boxes, bits 2-3 leaf
// boxes; 1 = every node boxed (offsets computed, no record load), 2 = none, 0 = mixed (table)
template <int NX, int NU>
__device__ __forceinline__ int o7_of(const Dev& p, int i, int bx) {
    const int md = bx & 3;
    return md == 1 ? p.E7 + i * (NX + NU) : md == 2 ? -1 : p.e7off[i];
}
template <int NX>
__device__ __forceinline__ int o14_of(const Dev& p, int l, int bx) {
    const int md = (bx >> 2) & 3;
    return md == 1 ? p.E14 + p.m + (l - p.m) * NX : md == 2 ? -1 : p.lrec[l - p.m].z;
}

// Loop order of the streaming kernels: a tile's epilogue operands are loaded first, then the
// wave's next tile, then the MFMAs and stores: vmcnt is in order, so an operand loaded after
// the prefetch would make the epilogue wait for the prefetched tile too.
template <class T, int NX, int NU>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ELL3_WPE_OF(T, NX))))
k_ell3(Dev p, const double* __restrict__ z_, double* __restrict__ eta_, int C, int bx) {
    typedef typename MF<T>::v4 v4;
    constexpr int nx = NX, nu = NU, RTX = (NX + 15) / 16, RTU = (NU + 15) / 16;
    const int n = p.n, m = p.m;
    cglbp<T> z = (cglbp<T>)z_;
    glbp<T> eg = (glbp<T>)eta_;
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4;
    const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), nwv = gridDim.x * (blockDim.x >> 6);
    // C > 0 (uniform branching): parent tiles of 16 parents, each product sqrtQ x_i / sqrtR u_i
    // computed once and stored to the C children's eta3 / eta4 rows (one table over the
    // children); C == 0: child tiles of 16 children reading their ancestors' rows
    const int Tc = C ? (m + 15) >> 4 : (n - 1 + 15) >> 4, Tl = (n - m + 15) >> 4;
    const int y1 = p.T0 - p.Y0;  // eta1 = y over the whole y segment
    const int nrow = m * (nx + nu) + y1 + m;
    const int fbeg = C ? m * (nx + nu) : 0;  // eta7 rows: written by the child tiles when C > 0
    const int Tp = (nrow - fbeg + kFlatRowsL - 1) / kFlatRowsL;
    WPerm<T, NX, NX> wq;  // sqrtQ for child tiles, sqrtPf for leaf tiles
    WPerm<T, NU, NU> wr;
    // per-wave LDS image of one output tile (16 nodes x (nx + 1))
    __shared__ T simg[4][16 * (NX + 1)];
    __attribute__((address_space(3))) T* img = (__attribute__((address_space(3))) T*)simg[threadIdx.x >> 6];
    if (C) {
        int task = gw;
        // cr.w: eta7 offset of parent lo of the tile (-1: unboxed / none)
        auto fetch = [&](int tk, int& o7, T (&ax)[(NX + 3) / 4], T (&au)[(NU + 3) / 4]) {
            const int i = 16 * tk + lo;
            const bool la = tk < Tc && i < m;
            o7 = la ? o7_of<NX, NU>(p, i, bx) : -1;
            load_arow<T, NX>(la ? z + p.X0 + (size_t)i * nx : nullptr, ax);
            load_arow<T, NU>(la ? z + p.U0 + (size_t)i * nu : nullptr, au);
        };
        int o7;
        T ax[(NX + 3) / 4], au[(NU + 3) / 4];
        if (task < Tc) {
            fetch(task, o7, ax, au);
            wq.load((const T*)p.SQ, p.crec[1].y);  // one table over the children (host check)
            wr.load((const T*)p.SR, p.crec[1].z);
        }
        for (; task < Tc; task += nwv) {
            const int i0 = 16 * task, cnt = min(16, m - i0);
            const int j0 = 1 + C * i0, cc = C * cnt;  // the tile's children j0 .. j0 + cc
            // eta5 = eta6 = tau_j / 2 of the cc <= 64 children: lane -> child j0 + lane
            const T tv = lane < cc ? z[p.T0 + j0 + lane] : T(0);
            int o7b;
            T ax2[(NX + 3) / 4], au2[(NU + 3) / 4];
            fetch(task + nwv, o7b, ax2, au2);
            v4 cx[RTX], cu[RTU];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) cx[r] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int r = 0; r < RTU; ++r) cu[r] = v4{0, 0, 0, 0};
            mma_perm(wq, ax, cx);
            mma_perm(wr, au, cu);
            store_tile<T, NX>(img, cx, cnt, eg + e3(p, j0), C);
            store_tile<T, NU>(img, cu, cnt, eg + e4(p, j0), C);
            if (lane < cc) {
                eg[p.E5 + j0 + lane] = T(0.5) * tv;
                eg[p.E6 + j0 + lane] = T(0.5) * tv;
            }
            if (o7 >= 0) {
                // eta7_i = [x_i; u_i] of a boxed parent from the A registers
                store_arow<T, NX>(eg + o7, ax);
                store_arow<T, NU>(eg + o7 + nx, au);
            }
            o7 = o7b;
            _Pragma("unroll") for (int k = 0; k < (NX + 3) / 4; ++k) ax[k] = ax2[k];
            _Pragma("unroll") for (int k = 0; k < (NU + 3) / 4; ++k) au[k] = au2[k];
        }
    } else {
    // child tiles (branching not uniform, C == 0): each child reads its ancestor's rows
    // through its record; eta7 comes from the flat tasks (fbeg = 0). Loads of the wave's
    // next tile are issued before the current tile's MFMAs and stores (vmcnt is in order:
    // loads issued after a store would wait for it)
        int task = gw;
        auto fetch = [&](int tk, Rec& cr, T (&ax)[(NX + 3) / 4], T (&au)[(NU + 3) / 4]) {
            const int ja = 1 + 16 * tk + lo;
            const bool la = tk < Tc && ja < n;
            if (!la) cr = Rec{0, -1, -1, -1};
            else cr = p.crec[ja];
            load_arow<T, NX>(la ? z + p.X0 + (size_t)cr.x * nx : nullptr, ax);
            load_arow<T, NU>(la ? z + p.U0 + (size_t)cr.x * nu : nullptr, au);
        };
        Rec cr;
        T ax[(NX + 3) / 4], au[(NU + 3) / 4];
        if (task < Tc) {
            fetch(task, cr, ax, au);
            // one table over the tiles (host check); lane 0's record is a live child
            wq.load((const T*)p.SQ, __builtin_amdgcn_readfirstlane(cr.y));
            wr.load((const T*)p.SR, __builtin_amdgcn_readfirstlane(cr.z));
        }
        for (; task < Tc; task += nwv) {
            const int j0 = 1 + 16 * task;
            const int cnt = min(16, n - j0);
            const T tv = lane < 2 * cnt ? z[p.T0 + j0 + (lane >> 1)] : T(0);
            Rec cr2;
            T ax2[(NX + 3) / 4], au2[(NU + 3) / 4];
            fetch(task + nwv, cr2, ax2, au2);
            v4 cx[RTX], cu[RTU];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) cx[r] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int r = 0; r < RTU; ++r) cu[r] = v4{0, 0, 0, 0};
            mma_perm<T, NX, NX>(wq, ax, cx);
            mma_perm<T, NU, NU>(wr, au, cu);
            // eta3 / eta4 of consecutive children are contiguous blocks
            store_tile<T, NX>(img, cx, cnt, eg + e3(p, j0));
            store_tile<T, NU>(img, cu, cnt, eg + e4(p, j0));
            if (lane < 2 * cnt) {
                const int j = j0 + (lane >> 1);
                eg[((lane & 1) ? p.E6 : p.E5) + j] = T(0.5) * tv;
            }
            cr = cr2;
            _Pragma("unroll") for (int k = 0; k < (NX + 3) / 4; ++k) ax[k] = ax2[k];
            _Pragma("unroll") for (int k = 0; k < (NU + 3) / 4; ++k) au[k] = au2[k];
        }
    }
    // leaf tiles, pipelined the same way (the wave's tasks continue after the child tiles)
    {
        const int first = ((Tc - gw + nwv - 1) / nwv) * nwv + gw;  // this wave's first task >= Tc
        int task = first;
        // o14: eta14 offset of leaf lo of the tile (-1: unboxed / no leaf)
        auto fetch = [&](int tk, int& o14, T (&ax)[(NX + 3) / 4]) {
            const int la_ = m + 16 * (tk - Tc) + lo;
            const bool la = tk < Tc + Tl && la_ < n;
            o14 = la ? o14_of<NX>(p, la_, bx) : -1;
            load_arow<T, NX>(la ? z + p.X0 + (size_t)la_ * nx : nullptr, ax);
        };
        int o14;
        T ax[(NX + 3) / 4];
        if (task < Tc + Tl) {
            fetch(task, o14, ax);
            wq.load((const T*)p.SP, p.lrec[m + 16 * (task - Tc) - m].x);
        }
        for (; task < Tc + Tl; task += nwv) {
            const int l0 = m + 16 * (task - Tc);
            const int cnt = min(16, n - l0);
            const T sv = lane < 2 * cnt ? z[p.S0 + l0 + (lane >> 1)] : T(0);
            int o14b;
            T ax2[(NX + 3) / 4];
            fetch(task + nwv, o14b, ax2);
            v4 cx[RTX];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) cx[r] = v4{0, 0, 0, 0};
            mma_perm<T, NX, NX>(wq, ax, cx);
            store_tile<T, NX>(img, cx, cnt, eg + e11(p, l0));
            // eta14 = x (boxed leaves; a leaf's eta14 block is its x row), from the A registers
            if (o14 >= 0) store_arow<T, NX>(eg + o14, ax);
            // eta12 = eta13 = s / 2
            if (lane < 2 * cnt) eg[((lane & 1) ? p.E13 : p.E12) + l0 + (lane >> 1)] = T(0.5) * sv;
            o14 = o14b;
            _Pragma("unroll") for (int k = 0; k < (NX + 3) / 4; ++k) ax[k] = ax2[k];
        }
    }
    for (int task = ((Tc + Tl - gw + nwv - 1) / nwv) * nwv + gw; task < Tc + Tl + Tp; task += nwv) {
        // kFlatRowsL flat rows: eta7 (nonleaf [x; u] on boxed nodes) | eta1 = y | eta2 = s - b'y
        const int nD = m * (nx + nu), nF = nD + y1;
        T a1[kFlatRowsL / 64];
        _Pragma("unroll") for (int k = 0; k < kFlatRowsL / 64; ++k) {
            const int q = fbeg + kFlatRowsL * (task - Tc - Tl) + 64 * k + lane;
            a1[k] = z[p.Y0 + (q >= nD && q < nF ? q - nD : 0)];
        }
        _Pragma("unroll") for (int k = 0; k < kFlatRowsL / 64; ++k) {
            const int q = fbeg + kFlatRowsL * (task - Tc - Tl) + 64 * k + lane;
            if (q >= nD && q < nF) {
                eg[p.E1 + q - nD] = a1[k];
            } else if (q < nD) {
                const int i = q / (nx + nu), rr = q - i * (nx + nu);
                const int o7 = o7_of<NX, NU>(p, i, bx);
                if (o7 >= 0) eg[o7 + rr] = rr < nx ? z[p.X0 + (size_t)i * nx + rr] : z[p.U0 + (size_t)i * nu + rr - nx];
            } else if (q < nrow) {
                const int i = q - nF;
                const int c = p.nch[i], yo = p.yrel[i], cs = p.ch_start[i];
                T by = T(0);
                for (int k = 0; k < c; ++k) by = fma(((cglbp<T>)p.cond)[cs + k], z[p.Y0 + yo + k], by);
                for (int k = c; k < 2 * c; ++k) by += T(0) * z[p.Y0 + yo + k];
                by += z[p.Y0 + yo + 2 * c];
                eg[p.E2 + i] = z[p.S0 + i] - by;
            }
        }
    }
}

// L^T (operators.py:55-94) as streaming wave tasks, for trees with one sqrtQ / sqrtR table over
// all children, one sqrtPf over all leaves and a uniform branching factor C <= 4 (BFS: the
// children of parent i are 1 + C i .. C i + C, y_i starts at (2C + 1) i; host-checked).
//
// Tasks (from the task index, no table):
//   [0, Tq)        parent tiles of PT = 4 Q parents (Q = 4 / C): A row lo is child
//                  kA = e_of(lo) % C of parent h_of(lo) + 4 (e_of(lo) / C), so the C children
//                  of one parent land in one lane's accumulator slots and are summed there in
//                  the reference's order: x_i = C7' eta7_i + sum_j sqrtQ eta3_j (same for u)
//   [Tq, + Tl)     leaf tiles of 16 leaves: x_l = sqrtPf eta11_l (+ eta14_l on boxed leaves)
//   [.., + Tf)     flat chunks of 64 rows of [y | s | tau_1..]: y_i = eta1_i - b_i eta2_i,
//                  s_i = eta2_i (nonleaf), s_l = (eta12_l + eta13_l) / 2, tau_j = (eta5_j + eta6_j) / 2
template <class T, int NX, int NU, int QM>  // QM = 4 / C parents per lane (compile time: register arrays)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ELL3_WPE_OF(T, NX))))
k_ellt3(Dev p, const double* __restrict__ eta_, double* __restrict__ z_, int C, int bx) {
    typedef typename MF<T>::v4 v4;
    constexpr int nx = NX, nu = NU, RTX = (NX + 15) / 16, RTU = (NU + 15) / 16;
    const int n = p.n, m = p.m;
    cglbp<T> d = (cglbp<T>)eta_;
    glbp<T> zg = (glbp<T>)z_;
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4;
    const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), nwv = gridDim.x * (blockDim.x >> 6);
    constexpr int Q = QM;
    const int PT = 4 * Q;
    const int Tq = (m + PT - 1) / PT, Tl = (n - m + 15) >> 4;
    const int ny = p.T0 - p.Y0, nrow = ny + n + (n - 1);
    const int Tf = (nrow + kFlatRows - 1) / kFlatRows;
    const int hA = MF<T>::h_of(lo), eA = MF<T>::e_of(lo);
    const int pA = hA + 4 * (eA / C), kA = eA % C;
    const bool slotA = eA < Q * C;
    WPerm<T, NX, NX> wq;  // sqrtQ for parent tiles, sqrtPf for leaf tiles
    WPerm<T, NU, NU> wr;
    {
        int task = gw;
        auto fetch = [&](int tk, T (&ax)[(NX + 3) / 4], T (&au)[(NU + 3) / 4]) {
            const int q = PT * tk + pA;
            const bool la = tk < Tq && slotA && q < m;
            const int j = 1 + C * q + kA;
            load_arow<T, NX>(la ? d + e3(p, j) : nullptr, ax);
            load_arow<T, NU>(la ? d + e4(p, j) : nullptr, au);
        };
        T ax[(NX + 3) / 4], au[(NU + 3) / 4];
        if (task < Tq) {
            fetch(task, ax, au);
            wq.load((const T*)p.SQ, p.crec[1].y);  // one table over the children (host check)
            wr.load((const T*)p.SR, p.crec[1].z);
        }
        for (; task < Tq; task += nwv) {
            const int pb = PT * task;
            // C7' eta7 of this tile's parents (lane: parent h + 4 sl, rows 16 rt + lo)
            T e7x[Q][RTX], e7u[Q][RTU];
            _Pragma("unroll") for (int sl = 0; sl < Q; ++sl) {
                const int q = pb + h + 4 * sl;
                const int o7 = q < m ? o7_of<NX, NU>(p, q, bx) : -1;
                _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt)
                    e7x[sl][rt] = o7 >= 0 && 16 * rt + lo < nx ? d[o7 + 16 * rt + lo] : T(0);
                _Pragma("unroll") for (int rt = 0; rt < RTU; ++rt)
                    e7u[sl][rt] = o7 >= 0 && 16 * rt + lo < nu ? d[o7 + nx + 16 * rt + lo] : T(0);
            }
            T ax2[(NX + 3) / 4], au2[(NU + 3) / 4];
            fetch(task + nwv, ax2, au2);
            v4 cx[RTX], cu[RTU];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) cx[r] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int r = 0; r < RTU; ++r) cu[r] = v4{0, 0, 0, 0};
            mma_perm<T, NX, NX>(wq, ax, cx);
            mma_perm<T, NU, NU>(wr, au, cu);
            _Pragma("unroll") for (int sl = 0; sl < Q; ++sl) {
                const int q = pb + h + 4 * sl;
                if (q >= m) continue;
                _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt) {
                    const int r = 16 * rt + lo;
                    if (r >= nx) continue;
                    T v = e7x[sl][rt];  // the reference starts from C7' eta7 or 0 (operators.py:73-78)
                    _Pragma("unroll") for (int e = 0; e < 4; ++e)
                        if (e / C == sl && e < Q * C) v += cx[rt][e];
                    ostn<ELLT3_NT != 0>(&zg[p.X0 + (size_t)q * nx + r], v);
                }
                _Pragma("unroll") for (int rt = 0; rt < RTU; ++rt) {
                    const int r = 16 * rt + lo;
                    if (r >= nu) continue;
                    T v = e7u[sl][rt];
                    _Pragma("unroll") for (int e = 0; e < 4; ++e)
                        if (e / C == sl && e < Q * C) v += cu[rt][e];
                    ostn<ELLT3_NT != 0>(&zg[p.U0 + (size_t)q * nu + r], v);
                }
            }
            _Pragma("unroll") for (int k = 0; k < (NX + 3) / 4; ++k) ax[k] = ax2[k];
            _Pragma("unroll") for (int k = 0; k < (NU + 3) / 4; ++k) au[k] = au2[k];
        }
    }
    {
        const int first = ((Tq - gw + nwv - 1) / nwv) * nwv + gw;  // this wave's first task >= Tq
        int task = first;
        auto fetch = [&](int tk, T (&ax)[(NX + 3) / 4]) {
            const int la_ = m + 16 * (tk - Tq) + lo;
            const bool la = tk < Tq + Tl && la_ < n;
            load_arow<T, NX>(la ? d + e11(p, la_) : nullptr, ax);
        };
        T ax[(NX + 3) / 4];
        if (task < Tq + Tl) {
            fetch(task, ax);
            wq.load((const T*)p.SP, p.lrec[0].x);
        }
        for (; task < Tq + Tl; task += nwv) {
            const int l0 = m + 16 * (task - Tq);
            // C14' eta14 of this tile's leaves (lane: leaf row(h, e), rows 16 rt + lo)
            T e14[4][RTX];
            bool b14[4];
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                const int l = l0 + MF<T>::row(h, e);
                const int o14 = l < n ? o14_of<NX>(p, l, bx) : -1;
                b14[e] = o14 >= 0;
                _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt)
                    e14[e][rt] = o14 >= 0 && 16 * rt + lo < nx ? d[o14 + 16 * rt + lo] : T(0);
            }
            T ax2[(NX + 3) / 4];
            fetch(task + nwv, ax2);
            v4 cx[RTX];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) cx[r] = v4{0, 0, 0, 0};
            mma_perm<T, NX, NX>(wq, ax, cx);
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                const int l = l0 + MF<T>::row(h, e);
                if (l >= n) continue;
                _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt) {
                    const int r = 16 * rt + lo;
                    if (r >= nx) continue;
                    T v = cx[rt][e];
                    if (b14[e]) v += e14[e][rt];
                    ostn<ELLT3_NT != 0>(&zg[p.X0 + (size_t)l * nx + r], v);
                }
            }
            _Pragma("unroll") for (int k = 0; k < (NX + 3) / 4; ++k) ax[k] = ax2[k];
        }
    }
    const int G = 2 * C + 1;
    // kFlatRows flat rows per task, branch-free loads (every lane loads from valid indices,
    // the row kind selects the formula afterwards) so all rows of a lane are in flight at once
    for (int task = ((Tq + Tl - gw + nwv - 1) / nwv) * nwv + gw; task < Tq + Tl + Tf; task += nwv) {
        constexpr int KR = kFlatRows / 64;
        T va[KR], vb[KR], vc[KR];
        int kind[KR];
        _Pragma("unroll") for (int k = 0; k < KR; ++k) {
            const int q = kFlatRows * (task - Tq - Tl) + 64 * k + lane;
            int ia = 0, ib = 0, ic = 0;
            kind[k] = -1;
            if (q < ny) {  // y_i[k] = eta1 - b_k eta2_i
                const int i = q / G, kk = q - i * G;
                ia = p.E1 + q; ib = p.E2 + i; ic = kk < C ? 1 + C * i + kk : 0;
                kind[k] = kk < C ? 0 : kk < 2 * C ? 1 : 2;
            } else if (q < ny + n) {  // s_i = eta2_i | s_l = (eta12 + eta13) / 2
                const int i = q - ny;
                ia = i < m ? p.E2 + i : p.E12 + i; ib = p.E13 + i;
                kind[k] = i < m ? 3 : 4;
            } else if (q < nrow) {  // tau_j = (eta5 + eta6) / 2
                const int j = q - ny - n + 1;
                ia = p.E5 + j; ib = p.E6 + j;
                kind[k] = 4;
            }
            va[k] = d[ia];
            vb[k] = d[ib];
            vc[k] = ((cglbp<T>)p.cond)[ic];
        }
        _Pragma("unroll") for (int k = 0; k < KR; ++k) {
            const int q = kFlatRows * (task - Tq - Tl) + 64 * k + lane;
            const int kd = kind[k];
            if (kd < 0) continue;
            const T b = kd == 0 ? vc[k] : kd == 1 ? T(0) : T(1);
            const T v = kd <= 2 ? va[k] - b * vb[k] : kd == 3 ? va[k] : T(0.5) * (va[k] + vb[k]);
            const int o = q < ny ? p.Y0 + q : q < ny + n ? p.S0 + (q - ny) : p.T0 + (q - ny - n + 1);
            zg[o] = v;
        }
    }
}
