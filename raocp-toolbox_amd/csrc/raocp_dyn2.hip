// raocp_dyn2.hip — the dynamics projection (cache.py:259-288) stage by stage, with its
// batched matrix-vector products as 16-node MFMA tiles, in any scalar type T: the sweep of
// fp32 contexts (BASELINE configs[4]: nx = 64, nu = 16, where the per-node products are
// 80 x 64 and fill the MFMA tiles). Included by raocp_kernels.hip after raocp_cp2.hip.
//
// Device form (raocp_dyn.hip header; host tables in raocp_capi.hip):
//   backward, stage t = N-1 .. 0:
//     (A) children j of stage t+1:  P_j = s [B_j' ; A_j'] q_j    (q_j = x_j, s = -1 at the leaves)
//     (B) parents i of stage t:     v = u_i - sum_j P_j[0:nu] ;  d_i = Rinv v ;
//                                   q_i = -x_i + sum_j P_j[nu:] + G v      ([Rinv ; G] one table)
//   forward, stage t = 0 .. N-1 (x_0 = x0bar first):
//     (U) parents i of stage t:     u_i = K x_i + d_i
//     (X) children j of stage t+1:  x_j = [Abar_j | B_j] [x_i ; d_i]
// Each launch is a list of tiles of at most 16 nodes that share one weight table (host:
// nodes of a stage grouped by child kind / class / (kind, class) pair); one wave per tile,
// A operands loaded straight from global (a node's row is contiguous), no LDS.

struct DynTile {
    int first;  // offset into the launch's node list
    int cnt;    // nodes (<= 16)
    int tab;    // weight table
    int pad;
};

// lane l: its tile's node for A row lo (or -1)
__device__ __forceinline__ int tile_node(const DynTile& t, const int* __restrict__ idx, int lo) {
    return lo < t.cnt ? idx[t.first + lo] : -1;
}

template <class T, int RT, int KSM>
__global__ void __launch_bounds__(256) k_d2_prod(Dev p, const Ctl* ctl, const DynTile* __restrict__ tiles,
                                                 int ntiles, const int* __restrict__ idx, const double* __restrict__ W_,
                                                 const double* __restrict__ src_, int src_base, T sign,
                                                 double* __restrict__ pa_) {
    if (ctl && ctl->done) return;
    typedef typename MF<T>::v4 v4;
    const int nx = p.nx, nu = p.nu, R = nx + nu;
    const int wt = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (wt >= ntiles) return;
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4;
    const DynTile t = tiles[wt];
    const int ja = tile_node(t, idx, lo);
    const T* src = (const T*)src_ + src_base;  // x rows (leaves) or q rows
    WFr<T, RT, KSM> wf;
    wf.load_rk((const T*)W_, t.tab, R, nx);
    v4 acc[RT];
    _Pragma("unroll") for (int r = 0; r < RT; ++r) acc[r] = v4{0, 0, 0, 0};
    tile1<T, RT, KSM>(wf, nx, [&](int k, T& a) { if (ja >= 0) a = ((cglbp<T>)src)[(size_t)ja * nx + k]; }, acc);
    glbp<T> pa = (glbp<T>)pa_;
    _Pragma("unroll") for (int e = 0; e < 4; ++e) {
        const int a = MF<T>::row(h, e);
        if (a >= t.cnt) continue;
        const int j = idx[t.first + a];
        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
            const int r = 16 * rt + lo;
            if (r < R) pa[(size_t)j * R + r] = sign * acc[rt][e];
        }
    }
}

template <class T, int RT, int KSM>
__global__ void __launch_bounds__(256) k_d2_node(Dev p, const Ctl* ctl, const DynTile* __restrict__ tiles,
                                                 int ntiles, const int* __restrict__ idx, const double* __restrict__ RG_,
                                                 const double* __restrict__ z_, const double* __restrict__ pa_,
                                                 double* __restrict__ q_, double* __restrict__ d_) {
    if (ctl && ctl->done) return;
    typedef typename MF<T>::v4 v4;
    const int nx = p.nx, nu = p.nu, R = nx + nu;
    const int wt = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (wt >= ntiles) return;
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4;
    const DynTile t = tiles[wt];
    const int ia = tile_node(t, idx, lo);
    cglbp<T> z = (cglbp<T>)z_;
    cglbp<T> pa = (cglbp<T>)pa_;
    int cs = 0, cn = 0;
    if (ia >= 0) {
        cs = p.ch_start[ia];
        cn = p.nch[ia];
    }
    WFr<T, RT, KSM> wf;
    wf.load_rk((const T*)RG_, t.tab, R, nu);
    v4 acc[RT];
    _Pragma("unroll") for (int r = 0; r < RT; ++r) acc[r] = v4{0, 0, 0, 0};
    // A row: v = u_i - sum_j P_j[0:nu]
    tile1<T, RT, KSM>(wf, nu, [&](int k, T& a) {
        if (ia >= 0) {
            T v = z[p.U0 + (size_t)ia * nu + k];
            for (int q = 0; q < cn; ++q) v -= pa[(size_t)(cs + q) * R + k];
            a = v;
        }
    }, acc);
    glbp<T> qo = (glbp<T>)q_;
    glbp<T> dout = (glbp<T>)d_;
    _Pragma("unroll") for (int e = 0; e < 4; ++e) {
        const int a = MF<T>::row(h, e);
        if (a >= t.cnt) continue;
        const int i = idx[t.first + a];
        const int c0 = p.ch_start[i], c1 = c0 + p.nch[i];
        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
            const int r = 16 * rt + lo;
            if (r < nu) {
                dout[(size_t)i * nu + r] = acc[rt][e];
            } else if (r < R) {
                T s = T(0);
                for (int j = c0; j < c1; ++j) s += pa[(size_t)j * R + r];
                qo[(size_t)i * nx + r - nu] = (-z[p.X0 + (size_t)i * nx + r - nu] + s) + acc[rt][e];
            }
        }
    }
}

// forward (U): u_i = K x_i + d_i ; (X): x_j = F [x_anc(j) ; d_anc(j)]
template <class T, int RT, int KSM, bool XROWS>
__global__ void __launch_bounds__(256) k_d2_fwd(Dev p, const Ctl* ctl, const DynTile* __restrict__ tiles,
                                                int ntiles, const int* __restrict__ idx, const double* __restrict__ M_,
                                                double* __restrict__ z_, const double* __restrict__ d_) {
    if (ctl && ctl->done) return;
    typedef typename MF<T>::v4 v4;
    const int nx = p.nx, nu = p.nu;
    const int wt = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (wt >= ntiles) return;
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4;
    const DynTile t = tiles[wt];
    const int na = tile_node(t, idx, lo);
    glbp<T> z = (glbp<T>)z_;
    cglbp<T> dd = (cglbp<T>)d_;
    const int Rr = XROWS ? nx : nu, K = XROWS ? nx + nu : nx;
    const int src = na < 0 ? -1 : (XROWS ? p.anc[na] : na);  // the node whose [x ; d] / x is the A row
    WFr<T, RT, KSM> wf;
    wf.load_rk((const T*)M_, t.tab, Rr, K);
    v4 acc[RT];
    _Pragma("unroll") for (int r = 0; r < RT; ++r) acc[r] = v4{0, 0, 0, 0};
    tile1<T, RT, KSM>(wf, K, [&](int k, T& a) {
        if (src >= 0) a = k < nx ? z[p.X0 + (size_t)src * nx + k] : dd[(size_t)src * nu + k - nx];
    }, acc);
    _Pragma("unroll") for (int e = 0; e < 4; ++e) {
        const int a = MF<T>::row(h, e);
        if (a >= t.cnt) continue;
        const int nd = idx[t.first + a];
        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
            const int r = 16 * rt + lo;
            if (r >= Rr) continue;
            if (XROWS) z[p.X0 + (size_t)nd * nx + r] = acc[rt][e];
            else z[p.U0 + (size_t)nd * nu + r] = acc[rt][e] + dd[(size_t)nd * nu + r];
        }
    }
}

template <class T>
__global__ void k_d2_x0(const Ctl* ctl, double* __restrict__ z_, int X0, const double* __restrict__ x0_,
                        int nx) {
    if (ctl && ctl->done) return;
    if ((int)threadIdx.x < nx) ((T*)z_)[X0 + threadIdx.x] = ((const T*)x0_)[threadIdx.x];
}
