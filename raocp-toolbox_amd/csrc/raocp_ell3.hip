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

template <class T, int R, int K>
__device__ __forceinline__ void mma_perm(const WPerm<T, R, K>& w, const T (&a)[(K + 3) / 4],
                                         typename MF<T>::v4 (&acc)[(R + 15) / 16]) {
    _Pragma("unroll") for (int s = 0; s < WPerm<T, R, K>::KC; ++s)
        _Pragma("unroll") for (int rt = 0; rt < WPerm<T, R, K>::RT; ++rt) acc[rt] = MF<T>::mma(a[s], w.b[rt][s], acc[rt]);
}

// store a 16-node x R-row tile (accumulators of RT row tiles) to rows dst + node * R + r of
// a contiguous block, through a per-wave LDS image (row stride R + 1: conflict-free writes)
// so every store instruction writes 64 consecutive elements
template <class T, int R>
__device__ __forceinline__ void store_tile(__attribute__((address_space(3))) T* img, const typename MF<T>::v4 (&acc)[(R + 15) / 16],
                                           int cnt, glbp<T> dst) {
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
    const int tot = cnt * R;
    constexpr int V = Vec16<T>::V;
    if constexpr (R % V == 0) {
        // 16 B per lane (a lane's V elements lie in one row): a quarter (fp32) / half (fp64)
        // of the store instructions of one element per lane
        typedef typename Vec16<T>::type vt;
        for (int q = lane * V; q < tot; q += 64 * V) {
            const int a = q / R, r = q - a * R;
            vt w;
            _Pragma("unroll") for (int u = 0; u < V; ++u) w[u] = img[a * S + r + u];
            *(__attribute__((address_space(1))) vt*)(dst + q) = w;
        }
    } else {
        for (int q = lane; q < tot; q += 64) {
            const int a = q / R, r = q - a * R;
            dst[q] = img[a * S + r];
        }
    }
    __builtin_amdgcn_wave_barrier();
}

template <class T, int NX, int NU>
__global__ void __launch_bounds__(256) k_ell3(Dev p, const double* __restrict__ z_, double* __restrict__ eta_) {
    typedef typename MF<T>::v4 v4;
    constexpr int nx = NX, nu = NU, RTX = (NX + 15) / 16, RTU = (NU + 15) / 16;
    const int n = p.n, m = p.m;
    cglbp<T> z = (cglbp<T>)z_;
    glbp<T> eg = (glbp<T>)eta_;
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4;
    const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), nwv = gridDim.x * (blockDim.x >> 6);
    const int Tc = (n - 1 + 15) >> 4, Tl = (n - m + 15) >> 4;
    const int y1 = p.T0 - p.Y0;  // eta1 = y over the whole y segment
    const int nrow = m * (nx + nu) + y1 + m;
    const int Tp = (nrow + 63) >> 6;
    WPerm<T, NX, NX> wq;  // sqrtQ for child tiles, sqrtPf for leaf tiles
    WPerm<T, NU, NU> wr;
    // per-wave LDS image of one output tile (16 nodes x (nx + 1))
    __shared__ T simg[4][16 * (NX + 1)];
    __attribute__((address_space(3))) T* img = (__attribute__((address_space(3))) T*)simg[threadIdx.x >> 6];
    // child tiles: loads of the wave's next tile are issued before the current tile's MFMAs
    // and stores (vmcnt is in order: loads issued after a store would wait for it)
    {
        int task = gw;
        auto fetch = [&](int tk, Rec& cr, T (&ax)[(NX + 3) / 4], T (&au)[(NU + 3) / 4]) {
            const int ja = 1 + 16 * tk + lo;
            const bool la = tk < Tc && ja < n;
            cr = la ? p.crec[ja] : Rec{0, -1, -1, 0};
            load_arow<T, NX>(la ? z + p.X0 + (size_t)cr.x * nx : nullptr, ax);
            load_arow<T, NU>(la ? z + p.U0 + (size_t)cr.x * nu : nullptr, au);
        };
        Rec cr;
        T ax[(NX + 3) / 4], au[(NU + 3) / 4];
        if (task < Tc) {
            fetch(task, cr, ax, au);
            const int tq = __builtin_amdgcn_readfirstlane(cr.y), tr = __builtin_amdgcn_readfirstlane(cr.z);
            wq.load((const T*)p.SQ, tq);  // one table over the tiles (host check)
            wr.load((const T*)p.SR, tr);
        }
        for (; task < Tc; task += nwv) {
            Rec cr2;
            T ax2[(NX + 3) / 4], au2[(NU + 3) / 4];
            fetch(task + nwv, cr2, ax2, au2);
            const int j0 = 1 + 16 * task;
            v4 cx[RTX], cu[RTU];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) cx[r] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int r = 0; r < RTU; ++r) cu[r] = v4{0, 0, 0, 0};
            mma_perm<T, NX, NX>(wq, ax, cx);
            mma_perm<T, NU, NU>(wr, au, cu);
            const int cnt = min(16, n - j0);
            // eta3 / eta4 of consecutive children are contiguous blocks
            store_tile<T, NX>(img, cx, cnt, eg + e3(p, j0));
            store_tile<T, NU>(img, cu, cnt, eg + e4(p, j0));
            if (lane < 2 * cnt) {
                const int j = j0 + (lane >> 1);
                eg[((lane & 1) ? p.E6 : p.E5) + j] = T(0.5) * z[p.T0 + j];
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
        auto fetch = [&](int tk, T (&ax)[(NX + 3) / 4]) {
            const int la_ = m + 16 * (tk - Tc) + lo;
            const bool la = tk < Tc + Tl && la_ < n;
            load_arow<T, NX>(la ? z + p.X0 + (size_t)la_ * nx : nullptr, ax);
        };
        T ax[(NX + 3) / 4];
        if (task < Tc + Tl) {
            fetch(task, ax);
            wq.load((const T*)p.SP, p.lrec[m + 16 * (task - Tc) - m].x);
        }
        for (; task < Tc + Tl; task += nwv) {
            T ax2[(NX + 3) / 4];
            fetch(task + nwv, ax2);
            const int l0 = m + 16 * (task - Tc);
            v4 cx[RTX];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) cx[r] = v4{0, 0, 0, 0};
            mma_perm<T, NX, NX>(wq, ax, cx);
            const int cnt = min(16, n - l0);
            store_tile<T, NX>(img, cx, cnt, eg + e11(p, l0));
            // eta14 = x (boxed leaves; a leaf's eta14 block is its x row), eta12 = eta13 = s / 2
            for (int q = lane; q < cnt * nx; q += 64) {
                const int a = q / nx, r = q - a * nx;
                const int o14 = p.lrec[l0 + a - m].z;
                if (o14 >= 0) eg[o14 + r] = z[p.X0 + (size_t)l0 * nx + q];
            }
            if (lane < 2 * cnt) {
                const int l = l0 + (lane >> 1);
                eg[((lane & 1) ? p.E13 : p.E12) + l] = T(0.5) * z[p.S0 + l];
            }
            _Pragma("unroll") for (int k = 0; k < (NX + 3) / 4; ++k) ax[k] = ax2[k];
        }
    }
    for (int task = ((Tc + Tl - gw + nwv - 1) / nwv) * nwv + gw; task < Tc + Tl + Tp; task += nwv) {
        {
            // 64 flat rows: eta7 (nonleaf [x; u] on boxed nodes) | eta1 = y | eta2 = s - b'y
            const int q = 64 * (task - Tc - Tl) + lane;
            const int nD = m * (nx + nu), nF = nD + y1;
            if (q < nD) {
                const int i = q / (nx + nu), rr = q - i * (nx + nu);
                const int o7 = p.e7off[i];
                if (o7 >= 0) eg[o7 + rr] = rr < nx ? z[p.X0 + (size_t)i * nx + rr] : z[p.U0 + (size_t)i * nu + rr - nx];
            } else if (q < nF) {
                const int e = q - nD;
                eg[p.E1 + e] = z[p.Y0 + e];
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
