// raocp_cp5.hip — the fused CP iteration (dual half step + prox of g*, the next primal half
// step with the s_0 relaxation and the AVaR kernel projection, the six residual maxima;
// solver.py:27-95, cache.py:248-393) for the LARGE uniform trees (configs 3, 4, 5) as two
// software-pipelined streaming launches. Its own translation unit (host interface: raocp_cp5.h).
//
//   k_cp5_leaf  (a) the AVaR cone rows of every nonleaf node j (eta2_j, 64 nodes per wave task):
//               eta2+_j and s_j of the half step BEFORE the kernel projection (out[S0 + j]; the
//               root: s_0 with its relaxation prox), with their residual terms;
//               (b) tiles of 16 leaves: eta11..eta14 with the leaf SOC and box, x_l of the half
//               step, and s_l of the half step before the kernel projection (out[S0 + l]);
//   k_cp5_fam   tiles of 16 parents (k_cp3's phases 1, 2, 3, 5) that read eta2+_i and their
//               children's s_j from the first launch instead of recomputing them (k_cp3
//               recomputed a nonleaf child's eta2 and a leaf child's SOC in the parent's tile).
//
// Why: k_cp3 runs a family's leaf children inside the family's tile, so its register file is
// the union of the two (468-500 VGPR + AGPR) and every tile waits for about a dozen dependent
// memory round trips (one child slot of prefetch), at one wave per SIMD. Here each launch is a
// persistent grid-stride loop whose waves issue EVERY load of their next tile before the
// current tile's arithmetic (register double buffering, k_cp4's unconditional loads at valid
// clamped addresses), so one tile's memory latency hides behind the previous tile's MFMA and
// VALU work. The per-node scalars are spread over the lane groups (lane group h holds y entry
// q = h + 4 t and child slot h's scalars, broadcast by shuffles where all lanes need them), so
// the prefetch buffer holds each scalar once, not four times. The residual maxima are kept in
// the iterate's type with NaN-propagating maxima (fp32: v_maximum3_f32 with |.| modifiers, two
// entries per instruction) and widened to fp64 per block.
//
// Extra traffic against k_cp3's 3|P| + 2|D|: one store and one load of s per non-root node
// (2 w (n - 1) bytes, 0.2 % at config 4) and one load of eta2+ per parent (w m, 0.1 %).
// The arithmetic of every entry is k_cp3's (sums regrouped: b'y as per-lane-group partial sums,
// L^T accumulators seeded with the box terms), so results agree with k_cp3 at rounding level
// (tests/test_gpu_cp5.py: 1e-12 fp64) and with the oracle (1e-8 per residual trace entry).

#include "raocp_cp5.h"
#include "raocp_cpops.h"

namespace raocp {
namespace {


// ================================ k_cp5_leaf ================================
// the operands of one leaf tile (lane lo = leaf)
template <class T, int NX, int BXL>
struct LeafOps {
    T lz[(NX + 15) / 16][4], lp[(NX + 15) / 16][4], d11[(NX + 15) / 16][4], d14[(NX + 15) / 16][4];
    T d12, d13, sz, sp;
    __device__ __forceinline__ void load(const Dev& p, cglbp<T> zp, cglbp<T> pz, cglbp<T> d, int l, bool live) {
        const int lq = live ? l : p.m;
        ld_rows_o<T, NX>(zp, p.X0 + lq * NX, live, lz);
        ld_rows_o<T, NX>(pz, p.X0 + lq * NX, live, lp);
        ld_rows_o<T, NX>(d, p.E11 + p.m + (lq - p.m) * NX, live, d11);
        if constexpr (BXL == 1) {
            ld_rows_o<T, NX>(d, p.E14 + p.m + (lq - p.m) * NX, live, d14);
        } else {
            _Pragma("unroll") for (int rt = 0; rt < (NX + 15) / 16; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) d14[rt][e] = T(0);
        }
        d12 = ldz_o(d, p.E12 + lq, live);
        d13 = ldz_o(d, p.E13 + lq, live);
        sz = ldz_o(zp, p.S0 + lq, live);
        sp = ldz_o(pz, p.S0 + lq, live);
    }
};

// Tasks of a wave (grid-stride over the waves): the eta2 tasks of the nonleaf ranges of et (64
// per task, lane = node; unsharded [0, m), a shard its own stages and the replicated top), then
// the leaf tiles of [l0, l1) (16 per tile), each tile's loads issued before the previous tile's
// arithmetic.
template <class T, int NX, int C, int BXL, bool LPF>
__global__ void __launch_bounds__(256, LPF ? 1 : 2) k_cp5_leaf(Dev p, Ctl* ctl, Bufs bf, double* __restrict__ part, Cp3Tasks et,
                                                     int l0, int l1, const double* __restrict__ img) {
    typedef typename MF<T>::v4 v4;
    constexpr int RX = (NX + 15) / 16, G = 2 * C + 1;
    typedef WL<T, NX, NX> WP;
    __shared__ __attribute__((aligned(16))) T wlds_[WP::N];
    __shared__ __attribute__((aligned(16))) T blds_[2 * NX];  // one-table trees: [lo_l | hi_l]
    const int m = p.m;
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4, wv = threadIdx.x >> 6;
    const int gw = blockIdx.x * (blockDim.x >> 6) + wv, nwv = gridDim.x * (blockDim.x >> 6);
    cglbp<T> pz = (cglbp<T>)bf.z0;  // p
    cglbp<T> zp = (cglbp<T>)bf.z1;  // z+
    glbp<T> out = (glbp<T>)bf.z2;   // next half step
    cglbp<T> d = (cglbp<T>)bf.e0;   // eta
    glbp<T> eo = (glbp<T>)bf.e1;    // eta+
    cglbp<T> cond = (cglbp<T>)p.cond;
    typedef __attribute__((address_space(3))) T lT;
    lT* bl_ = (lT*)blds_;
    const int nL = (l1 - l0 + 15) >> 4, nE = et.t0[et.nr];  // leaf tiles, eta2 tasks
    // the first leaf tile's operands, in flight during the prologue and the eta2 tasks
    LeafOps<T, NX, BXL> cur;
    if (LPF) cur.load(p, zp, pz, d, l0 + 16 * gw + lo, gw < nL && l0 + 16 * gw + lo < l1);
    {
        lds_fill((lds_d*)wlds_, img, WP::N * (int)sizeof(T) / 16);  // the sqrtPf fragments
        for (int e = threadIdx.x; e < 2 * NX; e += blockDim.x)  // one box table (cp5_supported)
            bl_[e] = BXL == 1 ? (e < NX ? ((cglbp<T>)p.blo_l)[e] : ((cglbp<T>)p.bhi_l)[e - NX]) : T(0);
    }
    const int done = ctl->done;
    Resid<T> rs;
    rs.alpha = (T)ctl->alpha;
    rs.ra = T(1) / rs.alpha;
    const T alpha = rs.alpha, ra = rs.ra;
    dma_wait();
    __syncthreads();
    if (done) return;  // uniform over the grid
    const WP wp{(const lT*)wlds_};
    bool nanf = false;  // a NaN reached a box (Rectangle._constrain raises)
    // ---- (a) eta2 of the nonleaf nodes (cache.py:321-372; raocp_cp3.hip phase 1)
    for (int t = gw; t < nE; t += nwv) {
        int r = 0;
        while (r + 1 < et.nr && t >= et.t0[r + 1]) ++r;
        const int j = et.lo[r] + 64 * (t - et.t0[r]) + lane;
        const bool live = j < et.hi[r];
        const int jq = live ? j : 0, yj = G * jq;
        T cp[C], zy[C], py[C];
        _Pragma("unroll") for (int k = 0; k < C; ++k) {
            cp[k] = ldz_o(cond, 1 + C * jq + k, live);
            zy[k] = ldz_o(zp, p.Y0 + yj + k, live);
            py[k] = ldz_o(pz, p.Y0 + yj + k, live);
        }
        const T zyc = ldz_o(zp, p.Y0 + yj + 2 * C, live), pyc = ldz_o(pz, p.Y0 + yj + 2 * C, live);
        const T zs = ldz_o(zp, p.S0 + jq, live), ps = ldz_o(pz, p.S0 + jq, live), d2 = ldz_o(d, p.E2 + jq, live);
        T bya = T(0), byb = T(0);
        _Pragma("unroll") for (int k = 0; k < C; ++k) {
            bya = fma(cp[k], T(2) * zy[k] - py[k], bya);
            byb = fma(cp[k], zy[k] - py[k], byb);
        }
        bya += T(2) * zyc - pyc;
        byb += zyc - pyc;
        const T av = (T(2) * zs - ps) - bya, bb = (zs - ps) - byb;
        const T v = (d2 + alpha * av) * ra;
        if (live) {
            T ep, x2;
            rs.fin(d2, v, fmax(v, T(0)), bb, ep, x2);
            *elw(eo, p.E2 + j) = ep;
            // s_j of the half step: L^T -> eta2_j; the root's relaxation prox s_0 -= alpha
            // (cache.py:253-257); the others before their parent's kernel projection
            *elw(out, p.S0 + j) = j == 0 ? (zs - alpha * ep) - alpha : zs - alpha * ep;
            rs.account(ps, zs, d2 - ep, x2);
        }
    }
    // ---- (b) leaf tiles
    for (int t = gw; t < nL; t += nwv) {
        const int l = l0 + 16 * t + lo;
        const bool live = l < l1;
        LeafOps<T, NX, BXL> nxt;
        if (LPF) {
            const int tn = t + nwv, ln = l0 + 16 * tn + lo;
            nxt.load(p, zp, pz, d, ln, tn < nL && ln < l1);
        } else {
            cur.load(p, zp, pz, d, l, live);
        }
        // eta14 = x_l (box, cache.py:374-393) seeds the L^T accumulators: x_l = sqrtPf eta11 +
        // eta14 (operators.py:86-94) for the three streams (eta+, d - eta+, xi2)
        v4 gA[RX], gW[RX], gC[RX];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) gA[rt] = gW[rt] = gC[rt] = v4{0, 0, 0, 0};
        if (BXL == 1) {
            T l14[RX][4], h14[RX][4], e14[RX][4];
            ld_rows_lds<T, NX>(bl_, l14);
            ld_rows_lds<T, NX>(bl_ + NX, h14);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                l14[rt][e] = live ? l14[rt][e] : T(0);  // a dead lane's terms stay zero
                h14[rt][e] = live ? h14[rt][e] : T(0);
            }
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                T ep = T(0), x2 = T(0);
                if (tok<NX>(rt, e)) {
                    const T v = (cur.d14[rt][e] + alpha * (T(2) * cur.lz[rt][e] - cur.lp[rt][e])) * ra;
                    rs.fin(cur.d14[rt][e], v, box_sel(v, l14[rt][e], h14[rt][e], nanf), cur.lz[rt][e] - cur.lp[rt][e], ep, x2);
                }
                e14[rt][e] = ep;
                gA[rt][e] = ep;
                gW[rt][e] = cur.d14[rt][e] - ep;
                gC[rt][e] = x2;
            }
            st_rows_o<T, NX>(eo, p.E14 + m + ((live ? l : m) - m) * NX, live, e14);
        }
        // L rows of the leaf: sqrtPf (2 z+ - p), sqrtPf (z+ - p) (operators.py:46-53)
        v4 la[RX], lb[RX];
        {
            T a1[RX][4], a2[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                a1[rt][e] = T(2) * cur.lz[rt][e] - cur.lp[rt][e];
                a2[rt][e] = cur.lz[rt][e] - cur.lp[rt][e];
            }
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) la[rt] = lb[rt] = v4{0, 0, 0, 0};
            mmt(wp.fresh(), a1, la);
            mmt(wp.fresh(), a2, lb);
        }
        // the leaf SOC (eta11, eta12 | eta13) (cache.py:374-393)
        T v11[RX][4];
        T ss = T(0);
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            v11[rt][e] = (cur.d11[rt][e] + alpha * la[rt][e]) * ra;
            if (tok<NX>(rt, e)) ss += v11[rt][e] * v11[rt][e];
        }
        ss = sum_h(ss);
        const T a5 = T(0.5) * (T(2) * cur.sz - cur.sp), b5 = T(0.5) * (cur.sz - cur.sp);
        const T v12 = (cur.d12 + alpha * a5) * ra + T(-0.5);
        const T v13 = (cur.d13 + alpha * a5) * ra + T(0.5);
        ss += v12 * v12;
        const Soc<T> so(sqrt(ss), v13);
        T ep12, x212, ep13, x213;
        rs.fin(cur.d12, v12, so.first(v12), b5, ep12, x212);
        rs.fin(cur.d13, v13, so.last(v13), b5, ep13, x213);
        if (live && h == 0) {
            // s_l of the half step before the kernel projection (k_cp5_fam reads it)
            *elw(out, p.S0 + l) = cur.sz - alpha * (T(0.5) * (ep12 + ep13));
            rs.account(cur.sp, cur.sz, T(0.5) * ((cur.d12 - ep12) + (cur.d13 - ep13)), T(0.5) * (x212 + x213));
            *elw(eo, p.E12 + l) = ep12;
        }
        if (live && h == 1) *elw(eo, p.E13 + l) = ep13;
        if constexpr (LPF) {
            T eA[RX][4], eW[RX][4], eC[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                T ep = T(0), x2 = T(0);
                if (tok<NX>(rt, e)) rs.fin(cur.d11[rt][e], v11[rt][e], so.first(v11[rt][e]), lb[rt][e], ep, x2);
                eA[rt][e] = ep;
                eW[rt][e] = cur.d11[rt][e] - ep;
                eC[rt][e] = x2;
            }
            st_rows_o<T, NX>(eo, p.E11 + m + ((live ? l : m) - m) * NX, live, eA);
            // L^T of the leaf rows: sqrtPf' (eta+, d - eta+, xi2) onto the box terms
            mmt(wp.fresh(), eA, gA);
            mmt(wp.fresh(), eW, gW);
            mmt(wp.fresh(), eC, gC);
            T ox[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                ox[rt][e] = cur.lz[rt][e] - alpha * gA[rt][e];
                if (tok<NX>(rt, e)) rs.account(cur.lp[rt][e], cur.lz[rt][e], gW[rt][e], gC[rt][e]);
            }
            st_rows_o<T, NX>(out, p.X0 + (live ? l : 0) * NX, live, ox);
            cur = nxt;
        } else {
            // two waves per SIMD: one L^T stream at a time, each stream's entries recomputed
            // from (d11, v11, lb) and the SOC selects (the residual maxima taken in the first
            // pass), so only one stream's rows are live at a time
            {
                T eA[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NX>(rt, e)) rs.fin(cur.d11[rt][e], v11[rt][e], so.first(v11[rt][e]), lb[rt][e], ep, x2);
                    eA[rt][e] = ep;
                }
                st_rows_o<T, NX>(eo, p.E11 + m + ((live ? l : m) - m) * NX, live, eA);
                mmt(wp.fresh(), eA, gA);
                T ox[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    ox[rt][e] = cur.lz[rt][e] - alpha * gA[rt][e];
                st_rows_o<T, NX>(out, p.X0 + (live ? l : 0) * NX, live, ox);
            }
            {
                T eW[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    eW[rt][e] = tok<NX>(rt, e) ? cur.d11[rt][e] - alpha * (v11[rt][e] - so.first(v11[rt][e])) : T(0);
                mmt(wp.fresh(), eW, gW);
            }
            {
                T eC[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    const T ep = alpha * (v11[rt][e] - so.first(v11[rt][e]));
                    eC[rt][e] = tok<NX>(rt, e) ? (cur.d11[rt][e] - ep) * ra + lb[rt][e] : T(0);
                }
                mmt(wp.fresh(), eC, gC);
            }
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NX>(rt, e)) rs.account(cur.lp[rt][e], cur.lz[rt][e], gW[rt][e], gC[rt][e]);
        }
    }
    flag_nan(ctl, nanf);
    block_maxima(part, rs);
}

// ================================ k_cp5_fams ================================
// k_cp5_fam's family tiles with the child slots in parallel: one tile per workgroup of C waves
// (k_cp6's role split without the leaf waves; the leaves and eta2 are k_cp5_leaf's), so a
// wave holds one slot's rows instead of all C and two workgroups share a CU, one streaming
// its tile's operands while the other computes:
//
//   wave k < C        child slot k: the parent's L products, the child block SOC (eta3, eta4,
//                     eta5 | eta6), the slot's (eta+, d - eta+, xi2) rows to LDS, tau_j;
//   wave C - 1        also phase 1: eta1 of the parent, y_i of the half step, the children's s;
//   -- barrier --
//   wave 0            L^T of the eta+ stream onto Gamma' eta7 (box), x_i and u_i of the half step;
//   wave 1            the (d - eta+) and xi2 streams and the residual terms of x_i, u_i;
//   wave C - 1        phase 5: the AVaR kernel projection of the family (cache.py:290-317).
//
// The slot rows are summed per parent in slot order (k_cp3's order), so the results equal
// k_cp5_fam's at rounding level (the same entry arithmetic).
template <class T, int NX, int NU, int C, int BXN>
__global__ void __launch_bounds__(64 * C, 2) k_cp5_fams(Dev p, Ctl* ctl, Bufs bf, double* __restrict__ part, Cp3Tasks tk,
                                                        const double* __restrict__ img) {
    typedef typename MF<T>::v4 v4;
    static_assert(C >= 3 && C <= 4, "C waves: two stream waves and a kernel-projection wave after the barrier");
    constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16, G = 2 * C + 1, NQ = (G + 3) / 4;
    typedef WL<T, NX, NX> WQ;
    typedef WL<T, NU, NU> WR;
    __shared__ KpScratch<T> ks_;
    __shared__ __attribute__((aligned(16))) T wlds_[WQ::N + WR::N];
    __shared__ __attribute__((aligned(16))) T blds_[2 * (NX + NU)];  // [lo_nl | hi_nl]
    // one stream of one slot, compacted: [x: 64 lanes x nx / 4 | u: 64 lanes x nu / 4]
    constexpr int SX = NX / 4 * 64, SS = (NX + NU) / 4 * 64;
    __shared__ __attribute__((aligned(16))) T sums_[C * 3 * SS];
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4, wv = threadIdx.x >> 6;
    typedef __attribute__((address_space(3))) T lT;
    typedef __attribute__((address_space(3))) KpScratch<T> lkps;
    lkps& ks = *(lkps*)&ks_;
    lT* sb = (lT*)sums_;
    cglbp<T> pz = (cglbp<T>)bf.z0;  // p
    cglbp<T> zp = (cglbp<T>)bf.z1;  // z+
    glbp<T> out = (glbp<T>)bf.z2;   // next half step
    cglbp<T> d = (cglbp<T>)bf.e0;   // eta
    glbp<T> eo = (glbp<T>)bf.e1;    // eta+
    cglbp<T> cond = (cglbp<T>)p.cond;
    lT* bl_ = (lT*)blds_;
    {
        lds_fill((lds_d*)wlds_, img, (WQ::N + WR::N) * (int)sizeof(T) / 16);  // [sqrtQ | sqrtR]
        for (int e = threadIdx.x; e < 2 * (NX + NU); e += blockDim.x)  // one box table (cp5_supported)
            bl_[e] = BXN == 1 ? (e < NX + NU ? ((cglbp<T>)p.blo_nl)[e] : ((cglbp<T>)p.bhi_nl)[e - (NX + NU)]) : T(0);
    }
    const int done = ctl->done;
    Resid<T> rs;
    rs.alpha = (T)ctl->alpha;
    rs.ra = T(1) / rs.alpha;
    const T alpha = rs.alpha, ra = rs.ra;
    dma_wait();
    __syncthreads();
    if (done) return;  // uniform over the grid
    const WQ wq{(const lT*)wlds_};
    const WR wr{(const lT*)wlds_ + WQ::N};
    bool nanf = false;  // a NaN reached a box (Rectangle._constrain raises)
    const int ntask = tk.t0[tk.nr];
    for (int task = blockIdx.x; task < ntask; task += gridDim.x) {
        int r = 0;
        while (r + 1 < tk.nr && task >= tk.t0[r + 1]) ++r;
        const int i0 = tk.lo[r] + 16 * (task - tk.t0[r]), iend = tk.hi[r];
        const bool live = i0 + lo < iend;
        const int iq = live ? i0 + lo : 0, yo = G * iq;
        {
            // ================= child slot k = wv
            const int k = wv, j = 1 + C * iq + k;
            T xz[RX][4], xp[RX][4], uz[RU][4], up[RU][4];
            ld_rows_o<T, NX>(zp, p.X0 + iq * NX, live, xz);
            ld_rows_o<T, NX>(pz, p.X0 + iq * NX, live, xp);
            ld_rows_o<T, NU>(zp, p.U0 + iq * NU, live, uz);
            ld_rows_o<T, NU>(pz, p.U0 + iq * NU, live, up);
            T d3[RX][4], d4[RU][4];
            ld_rows_o<T, NX>(d, p.E3 + 1 + (j - 1) * NX, live, d3);
            ld_rows_o<T, NU>(d, p.E4 + 1 + (j - 1) * NU, live, d4);
            const T d5 = ldz_o(d, p.E5 + j, live), d6 = ldz_o(d, p.E6 + j, live);
            const T tz = ldz_o(zp, p.T0 + j, live), tp = ldz_o(pz, p.T0 + j, live);
            if (wv == C - 1) {
                // ---------------- phase 1: eta1 of the parent (AVaR cone), y_i of the half step;
                // eta2+_i and the children's s from k_cp5_leaf (cache.py:321-372)
                T yz[NQ], yp[NQ], y1[NQ];
                _Pragma("unroll") for (int t = 0; t < NQ; ++t) {
                    const int q = h + 4 * t;
                    const bool ok = live && q < G;
                    const int qq = q < G ? q : 0;
                    yz[t] = ldz_o(zp, p.Y0 + yo + qq, ok);
                    yp[t] = ldz_o(pz, p.Y0 + yo + qq, ok);
                    y1[t] = ldz_o(d, p.E1 + yo + qq, ok);
                }
                const bool hc = live && h < C;
                const int jh = 1 + C * iq + (h < C ? h : 0);
                const T cph = ldz_o(cond, jh, hc), csl = ldz_o(out, p.S0 + jh, hc);
                const T zs = ldz_o(zp, p.S0 + iq, live), ps = ldz_o(pz, p.S0 + iq, live);
                const T d2 = ldz_o(d, p.E2 + iq, live), e2A = ldz_o(eo, p.E2 + iq, live);
                T pb = T(0);
                if (h < C) pb = cph * (yz[0] - yp[0]);
                _Pragma("unroll") for (int t = 0; t < NQ; ++t)
                    if (h + 4 * t == 2 * C) pb += yz[t] - yp[t];
                const T byb = sum_h(pb);
                const T e2W = d2 - e2A;
                const T e2C = (d2 - e2A) * ra + ((zs - ps) - byb);
                _Pragma("unroll") for (int t = 0; t < NQ; ++t) {
                    const int q = h + 4 * t;
                    if (!live || q >= G) break;
                    const T zy = yz[t], py = yp[t], dv = y1[t];
                    const T v = (dv + alpha * (T(2) * zy - py)) * ra;
                    T ep, x2;
                    rs.fin(dv, v, q < 2 * C ? fmax(v, T(0)) : v, zy - py, ep, x2);
                    *elw(eo, p.E1 + yo + q) = ep;
                    const T b = q < C ? cph : (q < 2 * C ? T(0) : T(1));
                    ks.y[lo][q] = zy - alpha * (ep - b * e2A);
                    rs.account(py, zy, (dv - ep) - b * e2W, x2 - b * e2C);
                }
                if (hc) ks.s[lo][h] = csl;
            }
            // L products of the parent: a = L(2z+ - p), b = L(z+ - p) on the children's rows
            v4 qa[RX], qb[RX], ua[RU], ub[RU];
            {
                T a1[RX][4], a2[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    a1[rt][e] = T(2) * xz[rt][e] - xp[rt][e];
                    a2[rt][e] = xz[rt][e] - xp[rt][e];
                }
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) qa[rt] = qb[rt] = v4{0, 0, 0, 0};
                mmt(wq.fresh(), a1, qa);
                mmt(wq.fresh(), a2, qb);
                T c1[RU][4], c2[RU][4];
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    c1[rt][e] = T(2) * uz[rt][e] - up[rt][e];
                    c2[rt][e] = uz[rt][e] - up[rt][e];
                }
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) ua[rt] = ub[rt] = v4{0, 0, 0, 0};
                mmt(wr.fresh(), c1, ua);
                mmt(wr.fresh(), c2, ub);
            }
            // ---------------- the child block SOC (cache.py:321-372)
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
            const Soc<T> so(sqrt(ss), v6);
            lT* sk = sb + k * 3 * SS;
            {
                T eA[RX][4], eW[RX][4], eC[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NX>(rt, e)) rs.fin(d3[rt][e], v3[rt][e], so.first(v3[rt][e]), qb[rt][e], ep, x2);
                    eA[rt][e] = ep;
                    eW[rt][e] = d3[rt][e] - ep;
                    eC[rt][e] = x2;
                }
                st_rows_o<T, NX>(eo, p.E3 + 1 + (j - 1) * NX, live, eA);
                lds_putc<T, NX>(sk, eA);
                lds_putc<T, NX>(sk + SS, eW);
                lds_putc<T, NX>(sk + 2 * SS, eC);
            }
            {
                T eA[RU][4], eW[RU][4], eC[RU][4];
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NU>(rt, e)) rs.fin(d4[rt][e], v4_[rt][e], so.first(v4_[rt][e]), ub[rt][e], ep, x2);
                    eA[rt][e] = ep;
                    eW[rt][e] = d4[rt][e] - ep;
                    eC[rt][e] = x2;
                }
                st_rows_o<T, NU>(eo, p.E4 + 1 + (j - 1) * NU, live, eA);
                lds_putc<T, NU>(sk + SX, eA);
                lds_putc<T, NU>(sk + SS + SX, eW);
                lds_putc<T, NU>(sk + 2 * SS + SX, eC);
            }
            T ep5, x25, ep6, x26;
            rs.fin(d5, v5, so.first(v5), b5, ep5, x25);
            rs.fin(d6, v6, so.last(v6), b5, ep6, x26);
            if (live && h == 0) {
                *elw(eo, p.E5 + j) = ep5;
                ks.tau[lo][k] = tz - alpha * (T(0.5) * (ep5 + ep6));
                rs.account(tp, tz, T(0.5) * ((d5 - ep5) + (d6 - ep6)), T(0.5) * (x25 + x26));
            }
            if (live && h == 1) *elw(eo, p.E6 + j) = ep6;
        }
        __syncthreads();  // the slots' rows, tau, s and y of the half step are in LDS
        if (wv <= 1) {
            // ---------------- phase 3: L^T = Gamma' eta7 + sqrtQ' / sqrtR' (summed slot rows)
            // (operators.py:73-85); wave 0 the eta+ stream, wave 1 the (d - eta+) and xi2 streams.
            // The parent's rows again (L2 hits: the slot phase read them), so they are not
            // live across the slot phase's SOC
            T xz[RX][4], xp[RX][4], uz[RU][4], up[RU][4], d7x[RX][4], d7u[RU][4];
            ld_rows_o<T, NX>(zp, p.X0 + iq * NX, live, xz);
            ld_rows_o<T, NX>(pz, p.X0 + iq * NX, live, xp);
            ld_rows_o<T, NU>(zp, p.U0 + iq * NU, live, uz);
            ld_rows_o<T, NU>(pz, p.U0 + iq * NU, live, up);
            if (BXN == 1) {
                ld_rows_o<T, NX>(d, p.E7 + iq * (NX + NU), live, d7x);
                ld_rows_o<T, NU>(d, p.E7 + iq * (NX + NU) + NX, live, d7u);
            }
            v4 g0[RX], g1[RX], g2[RX], h0[RU], h1[RU], h2[RU];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) g0[rt] = g1[rt] = g2[rt] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) h0[rt] = h1[rt] = h2[rt] = v4{0, 0, 0, 0};
            if (BXN == 1) {
                T lx[RX][4], hx[RX][4], lu[RU][4], hu[RU][4];
                ld_rows_lds<T, NX>(bl_, lx);
                ld_rows_lds<T, NX>(bl_ + (NX + NU), hx);
                ld_rows_lds<T, NU>(bl_ + NX, lu);
                ld_rows_lds<T, NU>(bl_ + (NX + NU) + NX, hu);
                T e7[RX][4], e7u[RU][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NX>(rt, e)) {
                        const T lv = live ? lx[rt][e] : T(0), hv = live ? hx[rt][e] : T(0);  // dead lanes: zero terms
                        const T v = (d7x[rt][e] + alpha * (T(2) * xz[rt][e] - xp[rt][e])) * ra;
                        rs.fin(d7x[rt][e], v, box_sel(v, lv, hv, nanf), xz[rt][e] - xp[rt][e], ep, x2);
                    }
                    e7[rt][e] = ep;
                    g0[rt][e] = ep;
                    g1[rt][e] = d7x[rt][e] - ep;
                    g2[rt][e] = x2;
                }
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NU>(rt, e)) {
                        const T lv = live ? lu[rt][e] : T(0), hv = live ? hu[rt][e] : T(0);
                        const T v = (d7u[rt][e] + alpha * (T(2) * uz[rt][e] - up[rt][e])) * ra;
                        rs.fin(d7u[rt][e], v, box_sel(v, lv, hv, nanf), uz[rt][e] - up[rt][e], ep, x2);
                    }
                    e7u[rt][e] = ep;
                    h0[rt][e] = ep;
                    h1[rt][e] = d7u[rt][e] - ep;
                    h2[rt][e] = x2;
                }
                if (wv == 0) {
                    const int o7 = p.E7 + iq * (NX + NU);
                    st_rows_o<T, NX>(eo, o7, live, e7);
                    st_rows_o<T, NU>(eo, o7 + NX, live, e7u);
                }
            }
            // the slots' rows of stream q summed per parent in slot order
            auto sums = [&](int q, T (&sx)[RX][4], T (&su)[RU][4]) {
                lds_getc<T, NX>(sb + q * SS, sx);
                lds_getc<T, NU>(sb + q * SS + SX, su);
                _Pragma("unroll") for (int kk = 1; kk < C; ++kk) {
                    T ax[RX][4], au[RU][4];
                    lds_getc<T, NX>(sb + (kk * 3 + q) * SS, ax);
                    lds_getc<T, NU>(sb + (kk * 3 + q) * SS + SX, au);
                    _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) sx[rt][e] += ax[rt][e];
                    _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) su[rt][e] += au[rt][e];
                }
            };
            if (wv == 0) {
                T sx[RX][4], su[RU][4];
                sums(0, sx, su);
                mmt(wq.fresh(), sx, g0);
                mmt(wr.fresh(), su, h0);
                T ox[RX][4], ou[RU][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    ox[rt][e] = xz[rt][e] - alpha * g0[rt][e];
                st_rows_o<T, NX>(out, p.X0 + iq * NX, live, ox);
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    ou[rt][e] = uz[rt][e] - alpha * h0[rt][e];
                st_rows_o<T, NU>(out, p.U0 + iq * NU, live, ou);
            } else {
                {
                    T sx[RX][4], su[RU][4];
                    sums(1, sx, su);
                    mmt(wq.fresh(), sx, g1);
                    mmt(wr.fresh(), su, h1);
                }
                {
                    T sx[RX][4], su[RU][4];
                    sums(2, sx, su);
                    mmt(wq.fresh(), sx, g2);
                    mmt(wr.fresh(), su, h2);
                }
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    if (tok<NX>(rt, e)) rs.account(xp[rt][e], xz[rt][e], g1[rt][e], g2[rt][e]);
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    if (tok<NU>(rt, e)) rs.account(up[rt][e], uz[rt][e], h1[rt][e], h2[rt][e]);
            }
        } else if (wv == C - 1 && live) {
            // ---------------- phase 5: the AVaR kernel projection of the family (cache.py:290-317)
            const T al = ldz_o((cglbp<T>)p.alpha_r, iq, true);
            const T y2c = ks.y[lo][2 * C];
            T rk[C], sr = T(0);
            _Pragma("unroll") for (int k = 0; k < C; ++k) {
                rk[k] = al * ks.y[lo][k] - ks.y[lo][C + k] + y2c - ks.tau[lo][k] - ks.s[lo][k];
                sr += rk[k];
            }
            const T a = al * al + T(3);
            T sw = T(0);
            _Pragma("unroll") for (int k = 0; k < C; ++k) {
                const T w = (rk[k] - sr / (a + (T)C)) / a;
                sw += w;
                if (k == h) {
                    const int j = 1 + C * iq + k;
                    *elw(out, p.Y0 + yo + k) = ks.y[lo][k] - al * w;
                    *elw(out, p.Y0 + yo + C + k) = ks.y[lo][C + k] + w;
                    *elw(out, p.T0 + j) = ks.tau[lo][k] + w;
                    *elw(out, p.S0 + j) = ks.s[lo][k] + w;
                }
            }
            if (h == 0) *elw(out, p.Y0 + yo + 2 * C) = y2c - sw;
        }
        __syncthreads();  // the LDS rows and the scratch are the next tile's
    }
    flag_nan(ctl, nanf);
    block_maxima(part, rs);
}

// ================================ k_cp6 ================================
// The SMALL trees' form (config 2: 8,191 nodes, 256 family tiles, a latency chain on an idle
// chip): one family tile per workgroup of 2 C waves that split the tile's work, so the tile's
// chain is the longest role, not the sum of k_cp4's phases in one or two waves:
//
//   wave k < C        child slot k: the parent's L products, the child block SOC (eta3, eta4,
//                     eta5 | eta6), the slot's (eta+, d - eta+, xi2) rows to LDS, tau_j of the half
//                     step; a nonleaf child's s_j from its eta2 (recomputed, k_cp3's arithmetic);
//   wave 0            also phase 1: eta1, eta2 of the parent, y_i of the half step, s_0;
//   wave C + k        (tiles of leaf parents) leaf child k: eta11..eta14 with the leaf SOC and box,
//                     x_l and s_l of the half step (k_cp5_leaf's arithmetic);
//   -- barrier --
//   wave 0            L^T of the eta+ stream: Gamma' eta7 (box) + sqrtQ' / sqrtR' of the slots'
//                     rows summed in slot order (k_cp3's order), x_i, u_i of the half step;
//   wave 1            the (d - eta+) stream; wave 2 C - 1 the xi2 stream, to LDS;
//   wave C            phase 5: the AVaR kernel projection of the family (cache.py:290-317);
//   -- barrier --
//   wave 1            the residual terms of x_i, u_i from both streams.
//
// Every operand of a role is loaded at the tile's start (k_cp4's unconditional loads), through
// 32-bit saddr offsets. Same arithmetic per entry as k_cp5 (results agree with k_cp4 / k_cp3 at
// rounding level, tests/test_gpu_cp6.py).
template <class T, int NX, int NU, int C, int BXN, int BXL>
__global__ void __launch_bounds__(128 * C) k_cp6(Dev p, Ctl* ctl, Bufs bf, double* __restrict__ part, Cp3Tasks tk,
                                                 const double* __restrict__ img) {
    typedef typename MF<T>::v4 v4;
    static_assert(C >= 2 && C <= 4, "2 C waves: slot waves, leaf waves, two stream waves");
    constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16, G = 2 * C + 1, NQ = (G + 3) / 4;
    typedef WL<T, NX, NX> WQ;
    typedef WL<T, NU, NU> WR;
    typedef WL<T, NX, NX> WP;
    __shared__ KpScratch<T> ks_;
    __shared__ __attribute__((aligned(16))) T wlds_[2 * WQ::N + WR::N];
    __shared__ __attribute__((aligned(16))) T blds_[2 * (NX + NU) + 2 * NX];  // [lo_nl | hi_nl | lo_l | hi_l]
    // the slots' (eta+, d - eta+, xi2) rows: [slot][stream][x chunks RX | u chunks RU] x 64 lanes x 4
    constexpr int SS = (RX + RU) * 256;
    __shared__ __attribute__((aligned(16))) T sums_[C * 3 * SS];
    __shared__ __attribute__((aligned(16))) T xch_[(RX + RU) * 256];  // the xi2 stream's L^T, wave 2 C - 1 -> wave 1
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4, wv = threadIdx.x >> 6;
    typedef __attribute__((address_space(3))) T lT;
    typedef __attribute__((address_space(3))) KpScratch<T> lkps;
    lkps& ks = *(lkps*)&ks_;
    lT* sb = (lT*)sums_;
    cglbp<T> pz = (cglbp<T>)bf.z0;  // p
    cglbp<T> zp = (cglbp<T>)bf.z1;  // z+
    glbp<T> out = (glbp<T>)bf.z2;   // next half step
    cglbp<T> d = (cglbp<T>)bf.e0;   // eta
    glbp<T> eo = (glbp<T>)bf.e1;    // eta+
    cglbp<T> cond = (cglbp<T>)p.cond;
    lT* bl_ = (lT*)blds_;
    const int m = p.m;
    // diagnostics (diagnostic builds, RAOCP_STAMP_KERNEL=c): every wave of the workgroup whose
    // first task is p.cp_dbg stamps [entry, prologue done, role done, barrier, streams done,
    // exit] at stamps[8 wave + q]; every workgroup its [entry, exit] at stamps[64 + 2 block]
    const unsigned long long t_in = kDiag && p.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const bool stp_on = kDiag && p.stamps && (int)blockIdx.x == p.cp_dbg && lane == 0;
    int stp_n = 0;
    auto stamp = [&]() {
        if (kDiag && stp_on && stp_n < 8) p.stamps[8 * wv + stp_n++] = __builtin_amdgcn_s_memrealtime();
    };
    stamp();
    {
        lds_fill((lds_d*)wlds_, img, (2 * WQ::N + WR::N) * (int)sizeof(T) / 16);  // [sqrtQ | sqrtR | sqrtPf]
        for (int e = threadIdx.x; e < 2 * (NX + NU) + 2 * NX; e += blockDim.x) {  // one box table each
            T v = T(0);
            if (e < NX + NU) v = BXN == 1 ? ((cglbp<T>)p.blo_nl)[e] : T(0);
            else if (e < 2 * (NX + NU)) v = BXN == 1 ? ((cglbp<T>)p.bhi_nl)[e - (NX + NU)] : T(0);
            else if (e < 2 * (NX + NU) + NX) v = BXL == 1 ? ((cglbp<T>)p.blo_l)[e - 2 * (NX + NU)] : T(0);
            else v = BXL == 1 ? ((cglbp<T>)p.bhi_l)[e - 2 * (NX + NU) - NX] : T(0);
            bl_[e] = v;
        }
    }
    const int done = ctl->done;
    Resid<T> rs;
    rs.alpha = (T)ctl->alpha;
    rs.ra = T(1) / rs.alpha;
    const T alpha = rs.alpha, ra = rs.ra;
    dma_wait();
    __syncthreads();
    if (done) return;  // uniform over the grid
    stamp();
    const WQ wq{(const lT*)wlds_};
    const WR wr{(const lT*)wlds_ + WQ::N};
    const WP wp{(const lT*)wlds_ + WQ::N + WR::N};
    bool nanf = false;  // a NaN reached a box (Rectangle._constrain raises)
    const int ntask = tk.t0[tk.nr];
    for (int task = blockIdx.x; task < ntask; task += gridDim.x) {
        int r = 0;
        while (r + 1 < tk.nr && task >= tk.t0[r + 1]) ++r;
        const int i0 = tk.lo[r] + 16 * (task - tk.t0[r]), iend = tk.hi[r];
        const bool leafp = tk.lo[r] >= tk.mL;
        const int i = i0 + lo;
        const bool live = i < iend;
        const int iq = live ? i : 0, yo = G * iq;
        if (wv < C) {
            // ================= child slot k = wv (and wave 0: phase 1)
            const int k = wv, j = 1 + C * iq + k;
            T xz[RX][4], xp[RX][4], uz[RU][4], up[RU][4], d3[RX][4], d4[RU][4];
            ld_rows_o<T, NX>(zp, p.X0 + iq * NX, live, xz);
            ld_rows_o<T, NX>(pz, p.X0 + iq * NX, live, xp);
            ld_rows_o<T, NU>(zp, p.U0 + iq * NU, live, uz);
            ld_rows_o<T, NU>(pz, p.U0 + iq * NU, live, up);
            ld_rows_o<T, NX>(d, p.E3 + 1 + (j - 1) * NX, live, d3);
            ld_rows_o<T, NU>(d, p.E4 + 1 + (j - 1) * NU, live, d4);
            const T d5 = ldz_o(d, p.E5 + j, live), d6 = ldz_o(d, p.E6 + j, live);
            const T tz = ldz_o(zp, p.T0 + j, live), tp = ldz_o(pz, p.T0 + j, live);
            // a nonleaf child's s and eta2 inputs (lane group 0 uses them)
            const bool g0 = live && !leafp;
            const T csz = ldz_o(zp, p.S0 + j, g0), csp = ldz_o(pz, p.S0 + j, g0), cdj = ldz_o(d, p.E2 + j, g0);
            T ccp[C], czy[C + 1], cpy[C + 1];
            {
                const int jj = leafp ? 0 : j, yj = G * jj;
                _Pragma("unroll") for (int q = 0; q < C; ++q) {
                    ccp[q] = ldz_o(cond, 1 + C * jj + q, g0);
                    czy[q] = ldz_o(zp, p.Y0 + yj + q, g0);
                    cpy[q] = ldz_o(pz, p.Y0 + yj + q, g0);
                }
                czy[C] = ldz_o(zp, p.Y0 + yj + 2 * C, g0);
                cpy[C] = ldz_o(pz, p.Y0 + yj + 2 * C, g0);
            }
            if (wv == 0) {
                // ---------------- phase 1: the parent's eta2, eta1 (AVaR cone), y_i, s_0
                T cp[C], zyk[C], pyk[C];
                _Pragma("unroll") for (int q = 0; q < C; ++q) {
                    cp[q] = ldz_o(cond, 1 + C * iq + q, live);
                    zyk[q] = ldz_o(zp, p.Y0 + yo + q, live);
                    pyk[q] = ldz_o(pz, p.Y0 + yo + q, live);
                }
                const T zyc = ldz_o(zp, p.Y0 + yo + 2 * C, live), pyc = ldz_o(pz, p.Y0 + yo + 2 * C, live);
                const T zs = ldz_o(zp, p.S0 + iq, live), ps = ldz_o(pz, p.S0 + iq, live), d2 = ldz_o(d, p.E2 + iq, live);
                T qz[NQ], qp[NQ], qd[NQ];
                _Pragma("unroll") for (int t = 0; t < NQ; ++t) {
                    const int q = h + 4 * t;
                    const bool ok = live && q < G;
                    const int qq = q < G ? q : 0;
                    qz[t] = ldz_o(zp, p.Y0 + yo + qq, ok);
                    qp[t] = ldz_o(pz, p.Y0 + yo + qq, ok);
                    qd[t] = ldz_o(d, p.E1 + yo + qq, ok);
                }
                T bya = T(0), byb = T(0);
                _Pragma("unroll") for (int q = 0; q < C; ++q) {
                    bya = fma(cp[q], T(2) * zyk[q] - pyk[q], bya);
                    byb = fma(cp[q], zyk[q] - pyk[q], byb);
                }
                bya += T(2) * zyc - pyc;
                byb += zyc - pyc;
                T e2A, e2C;
                {
                    const T av = (T(2) * zs - ps) - bya, bb = (zs - ps) - byb;
                    const T v = (d2 + alpha * av) * ra;
                    T x2;
                    rs.fin(d2, v, fmax(v, T(0)), bb, e2A, x2);
                    e2C = x2;
                    if (live && h == 0) *elw(eo, p.E2 + i) = e2A;
                }
                const T e2W = d2 - e2A;
                if (live && i == 0 && h == 0) {
                    // root s_0: L^T -> eta2_0, then the relaxation prox s_0 -= alpha (cache.py:253-257)
                    *elw(out, p.S0) = (zs - alpha * e2A) - alpha;
                    rs.account(ps, zs, e2W, e2C);
                }
                _Pragma("unroll") for (int t = 0; t < NQ; ++t) {
                    const int q = h + 4 * t;
                    if (!live || q >= G) break;
                    const T zy = qz[t], py = qp[t], dv = qd[t];
                    const T v = (dv + alpha * (T(2) * zy - py)) * ra;
                    T ep, x2;
                    rs.fin(dv, v, q < 2 * C ? fmax(v, T(0)) : v, zy - py, ep, x2);
                    *elw(eo, p.E1 + yo + q) = ep;
                    T b = T(1);
                    if (q < C) {
                        _Pragma("unroll") for (int kk = 0; kk < C; ++kk) if (kk == q) b = cp[kk];
                    } else if (q < 2 * C) {
                        b = T(0);
                    }
                    ks.y[lo][q] = zy - alpha * (ep - b * e2A);
                    rs.account(py, zy, (dv - ep) - b * e2W, x2 - b * e2C);
                }
            }
            // L products of the parent: a = L(2z+ - p), b = L(z+ - p) on the children's rows
            v4 qa[RX], qb[RX], ua[RU], ub[RU];
            {
                T a1[RX][4], a2[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    a1[rt][e] = T(2) * xz[rt][e] - xp[rt][e];
                    a2[rt][e] = xz[rt][e] - xp[rt][e];
                }
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) qa[rt] = qb[rt] = v4{0, 0, 0, 0};
                mmt(wq.fresh(), a1, qa);
                mmt(wq.fresh(), a2, qb);
                T c1[RU][4], c2[RU][4];
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    c1[rt][e] = T(2) * uz[rt][e] - up[rt][e];
                    c2[rt][e] = uz[rt][e] - up[rt][e];
                }
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) ua[rt] = ub[rt] = v4{0, 0, 0, 0};
                mmt(wr.fresh(), c1, ua);
                mmt(wr.fresh(), c2, ub);
            }
            // ---------------- the child block SOC (cache.py:321-372)
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
            const Soc<T> so(sqrt(ss), v6);
            lT* sk = sb + k * 3 * SS;
            {
                T eA[RX][4], eW[RX][4], eC[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NX>(rt, e)) rs.fin(d3[rt][e], v3[rt][e], so.first(v3[rt][e]), qb[rt][e], ep, x2);
                    eA[rt][e] = ep;
                    eW[rt][e] = d3[rt][e] - ep;
                    eC[rt][e] = x2;
                }
                st_rows_o<T, NX>(eo, p.E3 + 1 + (j - 1) * NX, live, eA);
                lds_put<T, NX>(sk, eA, false);
                lds_put<T, NX>(sk + SS, eW, false);
                lds_put<T, NX>(sk + 2 * SS, eC, false);
            }
            {
                T eA[RU][4], eW[RU][4], eC[RU][4];
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NU>(rt, e)) rs.fin(d4[rt][e], v4_[rt][e], so.first(v4_[rt][e]), ub[rt][e], ep, x2);
                    eA[rt][e] = ep;
                    eW[rt][e] = d4[rt][e] - ep;
                    eC[rt][e] = x2;
                }
                st_rows_o<T, NU>(eo, p.E4 + 1 + (j - 1) * NU, live, eA);
                lds_put<T, NU>(sk + RX * 256, eA, false);
                lds_put<T, NU>(sk + SS + RX * 256, eW, false);
                lds_put<T, NU>(sk + 2 * SS + RX * 256, eC, false);
            }
            T ep5, x25, ep6, x26;
            rs.fin(d5, v5, so.first(v5), b5, ep5, x25);
            rs.fin(d6, v6, so.last(v6), b5, ep6, x26);
            if (live && h == 0) {
                *elw(eo, p.E5 + j) = ep5;
                ks.tau[lo][k] = tz - alpha * (T(0.5) * (ep5 + ep6));
                rs.account(tp, tz, T(0.5) * ((d5 - ep5) + (d6 - ep6)), T(0.5) * (x25 + x26));
                if (!leafp) {
                    // s_j of a nonleaf child: its eta2 recomputed (its own tile's phase 1)
                    T ba = T(0), bb2 = T(0);
                    _Pragma("unroll") for (int q = 0; q < C; ++q) {
                        ba = fma(ccp[q], T(2) * czy[q] - cpy[q], ba);
                        bb2 = fma(ccp[q], czy[q] - cpy[q], bb2);
                    }
                    ba += T(2) * czy[C] - cpy[C];
                    bb2 += czy[C] - cpy[C];
                    const T av = (T(2) * csz - csp) - ba, bb = (csz - csp) - bb2;
                    const T v = (cdj + alpha * av) * ra;
                    const T ep = alpha * (v - fmax(v, T(0)));
                    const T x2 = (cdj - ep) * ra + bb;
                    ks.s[lo][k] = csz - alpha * ep;
                    rs.account(csp, csz, cdj - ep, x2);
                }
            }
            if (live && h == 1) *elw(eo, p.E6 + j) = ep6;
        } else if (leafp) {
            // ================= leaf child k = wv - C of a leaf-parent tile
            const int k = wv - C;
            const int l = 1 + C * iq + k;
            LeafOps<T, NX, BXL> cur;
            cur.load(p, zp, pz, d, l, live);
            v4 gA[RX], gW[RX], gC[RX];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) gA[rt] = gW[rt] = gC[rt] = v4{0, 0, 0, 0};
            if (BXL == 1) {
                T l14[RX][4], h14[RX][4], e14[RX][4];
                ld_rows_lds<T, NX>(bl_ + 2 * (NX + NU), l14);
                ld_rows_lds<T, NX>(bl_ + 2 * (NX + NU) + NX, h14);
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    l14[rt][e] = live ? l14[rt][e] : T(0);  // a dead lane's terms stay zero
                    h14[rt][e] = live ? h14[rt][e] : T(0);
                }
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NX>(rt, e)) {
                        const T v = (cur.d14[rt][e] + alpha * (T(2) * cur.lz[rt][e] - cur.lp[rt][e])) * ra;
                        rs.fin(cur.d14[rt][e], v, box_sel(v, l14[rt][e], h14[rt][e], nanf), cur.lz[rt][e] - cur.lp[rt][e], ep, x2);
                    }
                    e14[rt][e] = ep;
                    gA[rt][e] = ep;
                    gW[rt][e] = cur.d14[rt][e] - ep;
                    gC[rt][e] = x2;
                }
                st_rows_o<T, NX>(eo, p.E14 + m + ((live ? l : m) - m) * NX, live, e14);
            }
            v4 la[RX], lb[RX];
            {
                T a1[RX][4], a2[RX][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    a1[rt][e] = T(2) * cur.lz[rt][e] - cur.lp[rt][e];
                    a2[rt][e] = cur.lz[rt][e] - cur.lp[rt][e];
                }
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) la[rt] = lb[rt] = v4{0, 0, 0, 0};
                mmt(wp.fresh(), a1, la);
                mmt(wp.fresh(), a2, lb);
            }
            T v11[RX][4];
            T ss = T(0);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                v11[rt][e] = (cur.d11[rt][e] + alpha * la[rt][e]) * ra;
                if (tok<NX>(rt, e)) ss += v11[rt][e] * v11[rt][e];
            }
            ss = sum_h(ss);
            const T a5 = T(0.5) * (T(2) * cur.sz - cur.sp), b5 = T(0.5) * (cur.sz - cur.sp);
            const T v12 = (cur.d12 + alpha * a5) * ra + T(-0.5);
            const T v13 = (cur.d13 + alpha * a5) * ra + T(0.5);
            ss += v12 * v12;
            const Soc<T> so(sqrt(ss), v13);
            T ep12, x212, ep13, x213;
            rs.fin(cur.d12, v12, so.first(v12), b5, ep12, x212);
            rs.fin(cur.d13, v13, so.last(v13), b5, ep13, x213);
            if (live && h == 0) {
                ks.s[lo][k] = cur.sz - alpha * (T(0.5) * (ep12 + ep13));
                rs.account(cur.sp, cur.sz, T(0.5) * ((cur.d12 - ep12) + (cur.d13 - ep13)), T(0.5) * (x212 + x213));
                *elw(eo, p.E12 + l) = ep12;
            }
            if (live && h == 1) *elw(eo, p.E13 + l) = ep13;
            T eA[RX][4], eW[RX][4], eC[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                T ep = T(0), x2 = T(0);
                if (tok<NX>(rt, e)) rs.fin(cur.d11[rt][e], v11[rt][e], so.first(v11[rt][e]), lb[rt][e], ep, x2);
                eA[rt][e] = ep;
                eW[rt][e] = cur.d11[rt][e] - ep;
                eC[rt][e] = x2;
            }
            st_rows_o<T, NX>(eo, p.E11 + m + ((live ? l : m) - m) * NX, live, eA);
            mmt(wp.fresh(), eA, gA);
            mmt(wp.fresh(), eW, gW);
            mmt(wp.fresh(), eC, gC);
            T ox[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                ox[rt][e] = cur.lz[rt][e] - alpha * gA[rt][e];
                if (tok<NX>(rt, e)) rs.account(cur.lp[rt][e], cur.lz[rt][e], gW[rt][e], gC[rt][e]);
            }
            st_rows_o<T, NX>(out, p.X0 + (live ? l : 0) * NX, live, ox);
        }
        stamp();
        __syncthreads();  // the slots' rows, tau, s and y of the half step are in LDS
        stamp();
        lT* xch = (lT*)xch_;
        T xp[RX][4], xz[RX][4], up[RU][4], uz[RU][4];  // wave 1: the parent's rows for the residual terms
        v4 g1[RX], h1[RU];
        if (wv <= 1 || wv == 2 * C - 1) {
            // ---------------- phase 3: L^T = Gamma' eta7 + sqrtQ' / sqrtR' (summed slot rows)
            // (operators.py:73-85); wave 0 the eta+ stream, wave 1 the (d - eta+) stream, wave
            // 2 C - 1 the xi2 stream
            ld_rows_o<T, NX>(zp, p.X0 + iq * NX, live, xz);
            ld_rows_o<T, NX>(pz, p.X0 + iq * NX, live, xp);
            ld_rows_o<T, NU>(zp, p.U0 + iq * NU, live, uz);
            ld_rows_o<T, NU>(pz, p.U0 + iq * NU, live, up);
            v4 g0[RX], g2[RX], h0[RU], h2[RU];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) g0[rt] = g1[rt] = g2[rt] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) h0[rt] = h1[rt] = h2[rt] = v4{0, 0, 0, 0};
            if (BXN == 1) {
                T d7x[RX][4], d7u[RU][4], lx[RX][4], hx[RX][4], lu[RU][4], hu[RU][4];
                ld_rows_o<T, NX>(d, p.E7 + iq * (NX + NU), live, d7x);
                ld_rows_o<T, NU>(d, p.E7 + iq * (NX + NU) + NX, live, d7u);
                ld_rows_lds<T, NX>(bl_, lx);
                ld_rows_lds<T, NX>(bl_ + (NX + NU), hx);
                ld_rows_lds<T, NU>(bl_ + NX, lu);
                ld_rows_lds<T, NU>(bl_ + (NX + NU) + NX, hu);
                T e7[RX][4], e7u[RU][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NX>(rt, e)) {
                        const T lv = live ? lx[rt][e] : T(0), hv = live ? hx[rt][e] : T(0);
                        const T v = (d7x[rt][e] + alpha * (T(2) * xz[rt][e] - xp[rt][e])) * ra;
                        rs.fin(d7x[rt][e], v, box_sel(v, lv, hv, nanf), xz[rt][e] - xp[rt][e], ep, x2);
                    }
                    e7[rt][e] = ep;
                    g0[rt][e] = ep;
                    g1[rt][e] = d7x[rt][e] - ep;
                    g2[rt][e] = x2;
                }
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (tok<NU>(rt, e)) {
                        const T lv = live ? lu[rt][e] : T(0), hv = live ? hu[rt][e] : T(0);
                        const T v = (d7u[rt][e] + alpha * (T(2) * uz[rt][e] - up[rt][e])) * ra;
                        rs.fin(d7u[rt][e], v, box_sel(v, lv, hv, nanf), uz[rt][e] - up[rt][e], ep, x2);
                    }
                    e7u[rt][e] = ep;
                    h0[rt][e] = ep;
                    h1[rt][e] = d7u[rt][e] - ep;
                    h2[rt][e] = x2;
                }
                if (wv == 0) {
                    const int o7 = p.E7 + iq * (NX + NU);
                    st_rows_o<T, NX>(eo, o7, live, e7);
                    st_rows_o<T, NU>(eo, o7 + NX, live, e7u);
                }
            }
            // the slots' rows of stream q summed per parent in slot order
            auto sums = [&](int q, T (&sx)[RX][4], T (&su)[RU][4]) {
                lds_get<T, NX>(sb + q * SS, sx);
                lds_get<T, NU>(sb + q * SS + RX * 256, su);
                _Pragma("unroll") for (int k = 1; k < C; ++k) {
                    T ax[RX][4], au[RU][4];
                    lds_get<T, NX>(sb + (k * 3 + q) * SS, ax);
                    lds_get<T, NU>(sb + (k * 3 + q) * SS + RX * 256, au);
                    _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) sx[rt][e] += ax[rt][e];
                    _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) su[rt][e] += au[rt][e];
                }
            };
            if (wv == 0) {
                T sx[RX][4], su[RU][4];
                sums(0, sx, su);
                mmt(wq.fresh(), sx, g0);
                mmt(wr.fresh(), su, h0);
                T ox[RX][4], ou[RU][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    ox[rt][e] = xz[rt][e] - alpha * g0[rt][e];
                st_rows_o<T, NX>(out, p.X0 + iq * NX, live, ox);
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    ou[rt][e] = uz[rt][e] - alpha * h0[rt][e];
                st_rows_o<T, NU>(out, p.U0 + iq * NU, live, ou);
            } else if (wv == 1) {
                T sx[RX][4], su[RU][4];
                sums(1, sx, su);
                mmt(wq.fresh(), sx, g1);
                mmt(wr.fresh(), su, h1);
            } else {
                T sx[RX][4], su[RU][4];
                sums(2, sx, su);
                mmt(wq.fresh(), sx, g2);
                mmt(wr.fresh(), su, h2);
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    xch[(rt * 64 + lane) * 4 + e] = g2[rt][e];
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    xch[((RX + rt) * 64 + lane) * 4 + e] = h2[rt][e];
            }
        } else if (wv == C && live) {
            // ---------------- phase 5: the AVaR kernel projection of the family (cache.py:290-317)
            const T al = ldz_o((cglbp<T>)p.alpha_r, iq, true);
            const T y2c = ks.y[lo][2 * C];
            T rk[C], sr = T(0);
            _Pragma("unroll") for (int k = 0; k < C; ++k) {
                rk[k] = al * ks.y[lo][k] - ks.y[lo][C + k] + y2c - ks.tau[lo][k] - ks.s[lo][k];
                sr += rk[k];
            }
            const T a = al * al + T(3);
            T sw = T(0);
            _Pragma("unroll") for (int k = 0; k < C; ++k) {
                const T w = (rk[k] - sr / (a + (T)C)) / a;
                sw += w;
                if (k == h) {
                    const int j = 1 + C * i + k;
                    *elw(out, p.Y0 + yo + k) = ks.y[lo][k] - al * w;
                    *elw(out, p.Y0 + yo + C + k) = ks.y[lo][C + k] + w;
                    *elw(out, p.T0 + j) = ks.tau[lo][k] + w;
                    *elw(out, p.S0 + j) = ks.s[lo][k] + w;
                }
            }
            if (h == 0) *elw(out, p.Y0 + yo + 2 * C) = y2c - sw;
        }
        __syncthreads();  // the xi2 stream's L^T is in LDS
        if (wv == 1) {
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NX>(rt, e)) rs.account(xp[rt][e], xz[rt][e], g1[rt][e], xch[(rt * 64 + lane) * 4 + e]);
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NU>(rt, e)) rs.account(up[rt][e], uz[rt][e], h1[rt][e], xch[((RX + rt) * 64 + lane) * 4 + e]);
        }
        stamp();
        __syncthreads();  // the LDS rows, the exchange and the scratch are the next tile's
    }
    flag_nan(ctl, nanf);
    block_maxima(part, rs);
    stamp();
    if (kDiag && p.stamps && threadIdx.x == 0 && blockIdx.x < 2000) {
        p.stamps[64 + 2 * blockIdx.x] = t_in;
        p.stamps[65 + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    }
}

// resident grid: one 256-lane workgroup (one wave per SIMD) per CU, fewer when the tasks
// give every wave fewer than `per`
int cu_count() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}
int resident_grid(long tasks, int per) {
    const long wg = (tasks + 4L * per - 1) / (4L * per);
    return (int)std::max(1L, std::min(wg, (long)cu_count()));
}


template <class T, int NX, int NU, int C>
void launch_t(const Dev& p, Ctl* ctl, Bufs bf, double* part, int bx, const Cp3Tasks& et, int l0, int l1, int gl,
              const Cp3Tasks& tk, int gf, const double* img, bool lpf, hipStream_t s) {
    // the sqrtPf fragments follow [sqrtQ | sqrtR] in the image (16-B aligned: N multiples of 64)
    const double* imp = img + (size_t)(WL<T, NX, NX>::N + WL<T, NU, NU>::N) * sizeof(T) / 8;
    if (gl > 0 && lpf) {
        if ((bx & 3) == 1) k_cp5_leaf<T, NX, C, 1, true><<<gl, 256, 0, s>>>(p, ctl, bf, part, et, l0, l1, imp);
        else k_cp5_leaf<T, NX, C, 2, true><<<gl, 256, 0, s>>>(p, ctl, bf, part, et, l0, l1, imp);
    } else if (gl > 0) {
        if ((bx & 3) == 1) k_cp5_leaf<T, NX, C, 1, false><<<gl, 256, 0, s>>>(p, ctl, bf, part, et, l0, l1, imp);
        else k_cp5_leaf<T, NX, C, 2, false><<<gl, 256, 0, s>>>(p, ctl, bf, part, et, l0, l1, imp);
    }
    if ((bx & 3) == 1) k_cp5_fams<T, NX, NU, C, 1><<<gf, 64 * C, 0, s>>>(p, ctl, bf, part + (size_t)gl * 6, tk, img);
    else k_cp5_fams<T, NX, NU, C, 2><<<gf, 64 * C, 0, s>>>(p, ctl, bf, part + (size_t)gl * 6, tk, img);
}

}  // namespace

// compiled: configs 3 (fp64 20 / 8, C = 4), 4 (fp64 32 / 12, C = 3) and 5 (fp32 64 / 16, C = 4),
// every nonleaf and every leaf boxed (bx = 5) or none of them (bx = 10), by one box table each
bool cp5_supported(bool f32, int nx, int nu, int C, int bx, int nbox_nl, int nbox_l) {
    if (bx != 5 && bx != 10) return false;
    if (nbox_nl > 1 || nbox_l > 1) return false;  // one box table per kind (k_cp3 takes several)
    if (!f32) return (nx == 20 && nu == 8 && C == 4) || (nx == 32 && nu == 12 && C == 3);
    return nx == 64 && nu == 16 && C == 4;
}
const char* cp5_name(bool f32, int nx) {
    if (f32) return "k_cp5_leaf<float, 64, 4> x1 + k_cp5_fams<float, 64, 16, 4> x1";
    if (nx == 20) return "k_cp5_leaf<double, 20, 4> x1 + k_cp5_fams<double, 20, 8, 4> x1";
    return "k_cp5_leaf<double, 32, 3> x1 + k_cp5_fams<double, 32, 12, 3> x1";
}
// persistent grids (every workgroup resident, one wave per SIMD): a wave's tiles stream behind
// each other; at most one workgroup per CU
// k_cp5_leaf's default form (raocp_cp5.h): 0 in fp64 (config 3 56.3 -> 53.2 us, config 4 91.3 ->
// 89.7 us for the CP iteration), 1 in fp32 (config 5 327.8 vs 333.0 us; profiles/r05/cp_time_lpf.log)
bool cp5_leaf_pf_default(bool f32) { return f32; }
int cp5_leaf_grid(const Cp3Tasks& et, int l0, int l1, bool lpf) {
    const long tasks = (long)(std::max(l1 - l0, 0) + 15) / 16 + et.t0[et.nr];
    return (lpf ? 1 : 2) * resident_grid(tasks, 2);  // two workgroups per CU without the prefetch
}
// rows of residual partials of the two launches (one per workgroup)
int cp5_rows(int gl, int gf) {
    return gl + gf;
}
int cp5_fam_grid(const Cp3Tasks& tk) {
    return (int)std::max(1L, std::min((long)tk.t0[tk.nr], 2L * cu_count()));  // two workgroups per CU
}
// k_cp6: fp64 at nx = 20, nu = 8 with C = 2 (config 2), boxes as for k_cp5
bool cp6_supported(bool f32, int nx, int nu, int C, int bx, int nbox_nl, int nbox_l) {
    if (bx != 5 && bx != 10) return false;
    if (nbox_nl > 1 || nbox_l > 1) return false;
    return !f32 && nx == 20 && nu == 8 && C == 2;
}
const char* cp6_name() { return "k_cp6<double, 20, 8, 2>"; }
int cp6_rows(int grid) { return grid; }  // a residual row per workgroup
int cp6_grid(const Cp3Tasks& tk) { return (int)std::max(1L, std::min((long)tk.t0[tk.nr], 4096L)); }
void cp6_launch(const Dev& p, Ctl* ctl, Bufs bf, double* part, int bx, const Cp3Tasks& tk, int grid, const double* img,
                hipStream_t s) {
    if ((bx & 3) == 1) k_cp6<double, 20, 8, 2, 1, 1><<<grid, 256, 0, s>>>(p, ctl, bf, part, tk, img);
    else k_cp6<double, 20, 8, 2, 2, 2><<<grid, 256, 0, s>>>(p, ctl, bf, part, tk, img);
}
void cp5_launch(const Dev& p, Ctl* ctl, Bufs bf, double* part, int C, int bx, const Cp3Tasks& et, int l0, int l1, int gl,
                const Cp3Tasks& tk, int gf, const double* img, bool lpf, hipStream_t s) {
    if (p.nx == 20) launch_t<double, 20, 8, 4>(p, ctl, bf, part, bx, et, l0, l1, gl, tk, gf, img, lpf, s);
    else if (p.nx == 32) launch_t<double, 32, 12, 3>(p, ctl, bf, part, bx, et, l0, l1, gl, tk, gf, img, lpf, s);
    else launch_t<float, 64, 16, 4>(p, ctl, bf, part, bx, et, l0, l1, gl, tk, gf, img, lpf, s);
    (void)C;
}

}  // namespace raocp
