// raocp_cp4.hip — the fused CP iteration of raocp_cp3.hip (dual half step + prox of g*, the
// next primal half step with the s_0 relaxation and the AVaR kernel projection, the six
// residual maxima; solver.py:27-95, cache.py:248-393) for trees with one branching factor C,
// with every operand of a tile LOADED AT THE TILE'S START. Its own translation unit (host
// interface: raocp_cp4.h).
//
// Why: k_cp3 issues a tile's loads where the phases use them (the parent's y entries, its
// rows, each child slot, the nonleaf children's eta2 inputs, the eta7 rows and box bounds,
// alpha_r), behind data-dependent control flow (runtime C, `live` guards), so a family tile
// waited for about eleven memory round trips in sequence (37 vmcnt(0) in the fp64 20 / 8
// kernel); at config 2, where every wave has one tile, that chain was the kernel's time
// (≈ 20 us for ≈ 3-4 us of MFMA and VALU work). Here C and the box pattern are compile-time,
// a tile's loads are issued together into registers (FamIn / LeafIn below, ordered by first
// use: vmcnt retires in order), and the arithmetic is k_cp3's, operation for operation; the
// compiler contracts multiply-adds by code shape, so the results agree with k_cp3 at rounding
// level (tests/test_gpu_cp4.py: 1e-12 over 30 iterations).
//
// Layout and products: raocp_cp3.hip (family tiles of 16 parents, lane lo = parent, the
// transposed MFMA form whose L accumulators are directly the L^T B operands; the weight
// fragments [sqrtQ | sqrtR | sqrtPf] in LDS from k_cp3's image). The box bounds of trees with
// one box table per kind (every node the same Rectangle, the benchmark trees) go to LDS once
// per workgroup; other trees read their node's table from global memory at its use.

#include "raocp_cp4.h"
#include "raocp_tile.h"

namespace raocp {
namespace {

// (glbp / cglbp, MF, WL, mmt, ld_rows, ldz, st_rows, ld_rows_lds, sum_h, the cone and box
// projections, KpScratch, dma_wait: raocp_tile.h)

// ---- the operands of one leaf (a leaf tile's lane, or a leaf slot of a leaf-parent family)
template <class T, int NX, int BXL>
struct LeafIn {
    T lz[(NX + 15) / 16][4], lp[(NX + 15) / 16][4], d11[(NX + 15) / 16][4], d14[(NX + 15) / 16][4];
    T d12, d13, sz, sp;
    int bl;  // the leaf's box table (trees with several)
    __device__ __forceinline__ void load(const Dev& p, cglbp<T> zp, cglbp<T> pz, cglbp<T> d, int l, bool live, bool full) {
        const int lq = live ? l : p.m;
        ld_rows<T, NX>(zp + p.X0 + (size_t)lq * NX, live, lz);
        ld_rows<T, NX>(pz + p.X0 + (size_t)lq * NX, live, lp);
        ld_rows<T, NX>(d + p.E11 + p.m + (size_t)(lq - p.m) * NX, live, d11);
        if constexpr (BXL == 1) {  // (eta14 exists only where the leaves are boxed)
            ld_rows<T, NX>(d + p.E14 + p.m + (size_t)(lq - p.m) * NX, full && live, d14);
        } else {
            _Pragma("unroll") for (int rt = 0; rt < (NX + 15) / 16; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) d14[rt][e] = T(0);
        }
        d12 = ldz(d + p.E12 + lq, live);
        d13 = ldz(d + p.E13 + lq, live);
        sz = ldz(zp + p.S0 + lq, live);
        sp = ldz(pz + p.S0 + lq, live);
        bl = 0;
        if (BXL == 1 && full && p.nBl > 1) {
            const int b = p.iBl[lq];
            bl = live ? b : 0;
        }
    }
};

// ---- the operands of one family tile (parent lane lo; lane group h) in first-use order
template <class T, int NX, int NU, int C, int BXN, bool LEAFP>
struct FamIn {
    static constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16, G = 2 * C + 1, NQ = (G + 3) / 4;
    // phase 1: the parent's y entries for b'y, its s, eta2; its eta1 entries q = h + 4 t
    T cp[C], zyk[C], pyk[C], zyc, pyc, zs, ps, d2;
    T qz[NQ], qp[NQ], qd[NQ];
    // the parent's x, u rows (phases 1 and 3), eta7 rows (phase 3)
    T xz[RX][4], xp[RX][4], uz[RU][4], up[RU][4];
    // child slots (phase 2)
    T d3[C][RX][4], d4[C][RU][4], d5[C], d6[C], tz[C], tp[C];
    // nonleaf children (lane group 0): s, eta2 and the child family's y entries (eta2_j recomputed)
    T csz[C], csp[C], cdj[C], ccp[C][C], czy[C][C + 1], cpy[C][C + 1];
    T d7x[RX][4], d7u[RU][4];
    T al;
    int bi;
    __device__ __forceinline__ void load(const Dev& p, cglbp<T> zp, cglbp<T> pz, cglbp<T> d, cglbp<T> cond, int i,
                                         bool live) {
        const int h = (threadIdx.x & 63) >> 4;
        const int iq = live ? i : 0;
        const int yo = G * iq;
        _Pragma("unroll") for (int k = 0; k < C; ++k) {
            cp[k] = ldz(cond + 1 + C * iq + k, live);
            zyk[k] = ldz(zp + p.Y0 + yo + k, live);
            pyk[k] = ldz(pz + p.Y0 + yo + k, live);
        }
        zyc = ldz(zp + p.Y0 + yo + 2 * C, live);
        pyc = ldz(pz + p.Y0 + yo + 2 * C, live);
        zs = ldz(zp + p.S0 + iq, live);
        ps = ldz(pz + p.S0 + iq, live);
        d2 = ldz(d + p.E2 + iq, live);
        _Pragma("unroll") for (int t = 0; t < NQ; ++t) {
            const int q = h + 4 * t;
            const bool ok = live && q < G;
            const int qq = q < G ? q : 0;
            qz[t] = ldz(zp + p.Y0 + yo + qq, ok);
            qp[t] = ldz(pz + p.Y0 + yo + qq, ok);
            qd[t] = ldz(d + p.E1 + yo + qq, ok);
        }
        ld_rows<T, NX>(zp + p.X0 + (size_t)iq * NX, live, xz);
        ld_rows<T, NX>(pz + p.X0 + (size_t)iq * NX, live, xp);
        ld_rows<T, NU>(zp + p.U0 + (size_t)iq * NU, live, uz);
        ld_rows<T, NU>(pz + p.U0 + (size_t)iq * NU, live, up);
        _Pragma("unroll") for (int k = 0; k < C; ++k) {
            const int j = 1 + C * iq + k;
            ld_rows<T, NX>(d + p.E3 + 1 + (size_t)(j - 1) * NX, live, d3[k]);
            ld_rows<T, NU>(d + p.E4 + 1 + (size_t)(j - 1) * NU, live, d4[k]);
            d5[k] = ldz(d + p.E5 + j, live);
            d6[k] = ldz(d + p.E6 + j, live);
            tz[k] = ldz(zp + p.T0 + j, live);
            tp[k] = ldz(pz + p.T0 + j, live);
        }
        if (!LEAFP) {
            const bool g0 = live && h == 0;
            _Pragma("unroll") for (int k = 0; k < C; ++k) {
                const int j = 1 + C * iq + k, yj = G * j;
                csz[k] = ldz(zp + p.S0 + j, g0);
                csp[k] = ldz(pz + p.S0 + j, g0);
                cdj[k] = ldz(d + p.E2 + j, g0);
                _Pragma("unroll") for (int q = 0; q < C; ++q) {
                    ccp[k][q] = ldz(cond + 1 + C * j + q, g0);
                    czy[k][q] = ldz(zp + p.Y0 + yj + q, g0);
                    cpy[k][q] = ldz(pz + p.Y0 + yj + q, g0);
                }
                czy[k][C] = ldz(zp + p.Y0 + yj + 2 * C, g0);
                cpy[k][C] = ldz(pz + p.Y0 + yj + 2 * C, g0);
            }
        }
        if (BXN == 1) {
            ld_rows<T, NX>(d + p.E7 + (size_t)iq * (NX + NU), live, d7x);
            ld_rows<T, NU>(d + p.E7 + (size_t)iq * (NX + NU) + NX, live, d7u);
        }
        al = ldz((cglbp<T>)p.alpha_r + iq, live);
        bi = 0;
        if (BXN == 1 && p.nBnl > 1) {
            const int b = p.iBnl[iq];
            bi = live ? b : 0;
        }
    }
};

template <class T, int NX, int NU, int C, int BXN, int BXL>
__global__ void __launch_bounds__(256) k_cp4(Dev p, Ctl* __restrict__ ctl, Bufs bf, double* __restrict__ part,
                                             Cp3Tasks tk, const double* __restrict__ img) {
    typedef typename MF<T>::v4 v4;
    static_assert(NX % 4 == 0 && NU % 4 == 0, "row layout needs nx, nu multiples of 4");
    constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16, G = 2 * C + 1;
    typedef WL<T, NX, NX> WQ;
    typedef WL<T, NU, NU> WR;
    __shared__ KpScratch<T> kps_[4];
    __shared__ double s_red[6][4];
    __shared__ __attribute__((aligned(16))) T wlds_[2 * WQ::N + WR::N];
    // box bounds of one-table trees: [lo_nl | hi_nl | lo_l | hi_l]
    __shared__ __attribute__((aligned(16))) T blds_[2 * (NX + NU) + 2 * NX];
    const int m = p.m;
    const int lane = threadIdx.x & 63, lo = lane & 15, h = lane >> 4, wv = threadIdx.x >> 6;
    const int gw = blockIdx.x * (blockDim.x >> 6) + wv, nwv = gridDim.x * (blockDim.x >> 6);
    // helper mode (two-wave workgroups, one task each): wave 0 runs the task; on a tile of
    // leaf parents wave 1 runs the leaf children's work (the parent-side s_l into its scratch,
    // read by wave 0 in phase 5), off wave 0's chain. Else one task per wave.
    const bool hm = blockDim.x == 128;
    typedef __attribute__((address_space(3))) KpScratch<T> lkps;
    lkps& ks = *(lkps*)&kps_[wv];
    const lkps& kh = *(const lkps*)&kps_[1];  // helper mode: wave 1's scratch
    cglbp<T> pz = (cglbp<T>)bf.z0;  // p
    cglbp<T> zp = (cglbp<T>)bf.z1;  // z+
    glbp<T> out = (glbp<T>)bf.z2;   // next half step
    cglbp<T> d = (cglbp<T>)bf.e0;   // eta
    glbp<T> eo = (glbp<T>)bf.e1;    // eta+
    cglbp<T> cond = (cglbp<T>)p.cond;
    double m0 = 0.0, m1 = 0.0, m2 = 0.0, m3 = 0.0, m4 = 0.0, m5 = 0.0;
    typedef __attribute__((address_space(3))) T lT;
    lT* wl = (lT*)wlds_;
    lT* bl_ = (lT*)blds_;
    {
        // the weight image by LDS-DMA (whole 16-B chunks; N: multiples of 64)
        const int chunks = (2 * WQ::N + WR::N) * (int)sizeof(T) / 16;
        const int nw = blockDim.x >> 6;
        for (int c0 = wv * 64; c0 < chunks; c0 += nw * 64) {
            const int ch = c0 + lane;
            if (ch < chunks)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) double*)(img + 2 * ch),
                                                 (lds_d*)wlds_ + 2 * c0, 16, 0, 0);
        }
        const bool onen = BXN == 1 && p.nBnl <= 1, onel = BXL == 1 && p.nBl <= 1;
        for (int e = threadIdx.x; e < 2 * (NX + NU) + 2 * NX; e += blockDim.x) {
            T v = T(0);
            if (e < NX + NU) v = onen ? ((cglbp<T>)p.blo_nl)[e] : T(0);
            else if (e < 2 * (NX + NU)) v = onen ? ((cglbp<T>)p.bhi_nl)[e - (NX + NU)] : T(0);
            else if (e < 2 * (NX + NU) + NX) v = onel ? ((cglbp<T>)p.blo_l)[e - 2 * (NX + NU)] : T(0);
            else v = onel ? ((cglbp<T>)p.bhi_l)[e - 2 * (NX + NU) - NX] : T(0);
            bl_[e] = v;
        }
    }
    const int done = ctl->done;
    const T alpha = (T)ctl->alpha, ra = T(1) / alpha;
    dma_wait();
    __syncthreads();
    if (done) return;  // uniform over the grid
    const WQ wq{wl};
    const WR wr{wl + WQ::N};
    const WQ wp{wl + WQ::N + WR::N};
    auto fin = [&](T dv, T v, T pv, T b, T& ep, T& x2) {
        ep = alpha * (v - pv);
        x2 = (dv - ep) * ra + b;
        m2 = nmax(m2, (double)fabs(x2));
        m5 = nmax(m5, (double)fabs(ep - dv));
    };
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
    // one leaf l (lane lo) of slot k: full = the whole leaf (eta11..eta14, x_l of the half step),
    // else only its SOC scalars; pside = the parent's side (s_l into the kernel projection's
    // scratch and its residual terms). raocp_cp3.hip leaf_work, with the operands loaded.
    auto leaf_work = [&](const LeafIn<T, NX, BXL>& cur, int l, int k, bool live, bool full, bool pside) {
        const T(&lz)[RX][4] = cur.lz;
        const T(&lp)[RX][4] = cur.lp;
        const T(&d11)[RX][4] = cur.d11;
        const T(&d14)[RX][4] = cur.d14;
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
        st_rows<T, NX>(eo + p.E11 + m + (size_t)((live ? l : m) - m) * NX, live, eA);
        v4 gA[RX], gW[RX], gC[RX];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) gA[rt] = gW[rt] = gC[rt] = v4{0, 0, 0, 0};
        mmt(wp, eA, gA);
        mmt(wp, eW, gW);
        mmt(wp, eC, gC);
        // eta14 = x_l (box) and x_l = sqrtPf eta11 + eta14 (operators.py:86-94)
        if (BXL == 1 && live) {
            T l14[RX][4], h14[RX][4], e14[RX][4];
            if (p.nBl <= 1) {
                ld_rows_lds<T, NX>(bl_ + 2 * (NX + NU), l14);
                ld_rows_lds<T, NX>(bl_ + 2 * (NX + NU) + NX, h14);
            } else {
                ld_rows<T, NX>((cglbp<T>)p.blo_l + (size_t)cur.bl * NX, true, l14);
                ld_rows<T, NX>((cglbp<T>)p.bhi_l + (size_t)cur.bl * NX, true, h14);
            }
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
            st_rows<T, NX>(eo + p.E14 + m + (size_t)(l - m) * NX, true, e14);
        }
        T ox[RX][4];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            ox[rt][e] = lz[rt][e] - alpha * gA[rt][e];
            if (live && tok<NX>(rt, e)) account(lp[rt][e], lz[rt][e], gW[rt][e], gC[rt][e]);
        }
        st_rows<T, NX>(out + p.X0 + (size_t)(live ? l : 0) * NX, live, ox);
    };
    // one family tile: parents i0 + lo (< iend); LEAFP: the children are leaves
    // diagnostics (p.stamps, RAOCP_STAMP_KERNEL=c): s_memrealtime at the phase boundaries of
    // one family task (lane 0 of the wave that takes task nTL + 200)
    bool stp_on = false;
    int stp_n = 0;
    auto stamp = [&]() {
        if (kDiag && stp_on && (threadIdx.x & 63) == 0 && stp_n < 16) p.stamps[stp_n++] = __builtin_amdgcn_s_memrealtime();
    };
    auto family = [&](auto leafp_tag, int i0, int iend, int split) {
        constexpr bool LEAFP = decltype(leafp_tag)::value;
        stamp();
        const int i = i0 + lo;
        const bool live = i < iend;
        const int yo = G * i;
        FamIn<T, NX, NU, C, BXN, LEAFP> in;
        LeafIn<T, NX, BXL> lf[LEAFP ? C : 1];
        // ---- every operand of the tile, in first-use order (vmcnt retires in issue order)
        if (LEAFP && !hm)
            _Pragma("unroll") for (int k = 0; k < C; ++k) lf[k].load(p, zp, pz, d, 1 + C * i + k, live, !split);
        in.load(p, zp, pz, d, cond, i, live);
        stamp();  // loads issued
        // ---------------- phase 4 (parents of leaves): leaf children; their s_l to the scratch
        // (helper mode: wave 1 of the workgroup)
        if (LEAFP && !hm)
            _Pragma("unroll") for (int k = 0; k < C; ++k) leaf_work(lf[k], 1 + C * i + k, k, live, !split, true);
        stamp();
        // ---------------- phase 1: the parent's rows
        T bya = T(0), byb = T(0);
        if (live) {
            _Pragma("unroll") for (int k = 0; k < C; ++k) {
                bya = fma(in.cp[k], T(2) * in.zyk[k] - in.pyk[k], bya);
                byb = fma(in.cp[k], in.zyk[k] - in.pyk[k], byb);
            }
            bya += T(2) * in.zyc - in.pyc;
            byb += in.zyc - in.pyc;
        }
        const T zs = in.zs, ps = in.ps, d2 = in.d2;
        T e2A, e2C;
        {
            const T av = (T(2) * zs - ps) - bya, bb = (zs - ps) - byb;
            const T v = (d2 + alpha * av) * ra;
            T x2;
            fin(d2, v, fmax(v, T(0)), bb, e2A, x2);
            e2C = x2;
            if (live && h == 0) eo[p.E2 + i] = e2A;
        }
        const T e2W = d2 - e2A;
        if (live && i == 0 && h == 0) {
            // root s_0: L^T -> eta2_0, then the relaxation prox s_0 -= alpha (cache.py:253-257)
            out[p.S0] = (zs - alpha * e2A) - alpha;
            account(ps, zs, e2W, e2C);
        }
        _Pragma("unroll") for (int t = 0; t < FamIn<T, NX, NU, C, BXN, LEAFP>::NQ; ++t) {
            const int q = h + 4 * t;
            if (!live || q >= G) break;
            const T zy = in.qz[t], py = in.qp[t], dv = in.qd[t];
            const T av = T(2) * zy - py, bb = zy - py;
            const T v = (dv + alpha * av) * ra;
            T ep, x2;
            fin(dv, v, q < 2 * C ? fmax(v, T(0)) : v, bb, ep, x2);
            eo[p.E1 + yo + q] = ep;
            T b = T(1);
            if (q < C) {
                _Pragma("unroll") for (int k = 0; k < C; ++k) if (k == q) b = in.cp[k];
            } else if (q < 2 * C) {
                b = T(0);
            }
            ks.y[lo][q] = zy - alpha * (ep - b * e2A);
            account(py, zy, (dv - ep) - b * e2W, x2 - b * e2C);
        }
        // L products of the parent: a = L(2z+ - p), b = L(z+ - p) on the children's rows
        v4 qa[RX], qb[RX], ua[RU], ub[RU];
        {
            T a1[RX][4], a2[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                a1[rt][e] = T(2) * in.xz[rt][e] - in.xp[rt][e];
                a2[rt][e] = in.xz[rt][e] - in.xp[rt][e];
            }
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) qa[rt] = qb[rt] = v4{0, 0, 0, 0};
            mmt(wq, a1, qa);
            mmt(wq, a2, qb);
            T c1[RU][4], c2[RU][4];
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                c1[rt][e] = T(2) * in.uz[rt][e] - in.up[rt][e];
                c2[rt][e] = in.uz[rt][e] - in.up[rt][e];
            }
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) ua[rt] = ub[rt] = v4{0, 0, 0, 0};
            mmt(wr, c1, ua);
            mmt(wr, c2, ub);
        }
        T sxA[RX][4], sxW[RX][4], sxC[RX][4], suA[RU][4], suW[RU][4], suC[RU][4];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
            sxA[rt][e] = sxW[rt][e] = sxC[rt][e] = T(0);
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
            suA[rt][e] = suW[rt][e] = suC[rt][e] = T(0);
        stamp();
        // ---------------- phase 2: child slots (child block SOC, L^T accumulation)
        _Pragma("unroll") for (int k = 0; k < C; ++k) {
            const int j = 1 + C * i + k;
            const T(&d3)[RX][4] = in.d3[k];
            const T(&d4)[RU][4] = in.d4[k];
            const T d5 = in.d5[k], d6 = in.d6[k], tz = in.tz[k], tp = in.tp[k];
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
            T e3A[RX][4], e3W[RX][4], e3C[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                T ep = T(0), x2 = T(0);
                if (live && tok<NX>(rt, e))
                    fin(d3[rt][e], v3[rt][e], soc_apply_t(v3[rt][e], false, nf, tt), qb[rt][e], ep, x2);
                e3A[rt][e] = ep;
                e3W[rt][e] = d3[rt][e] - ep;
                e3C[rt][e] = x2;
            }
            st_rows<T, NX>(eo + p.E3 + 1 + (size_t)((live ? j : 1) - 1) * NX, live, e3A);
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
            st_rows<T, NU>(eo + p.E4 + 1 + (size_t)((live ? j : 1) - 1) * NU, live, e4A);
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                suA[rt][e] += e4A[rt][e];
                suW[rt][e] += e4W[rt][e];
                suC[rt][e] += e4C[rt][e];
            }
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
            if (!LEAFP && live && h == 0) {
                // s_j of a nonleaf child: its eta2 recomputed (the arithmetic of its own tile's
                // phase 1, bit-identical), then the half step
                const T sz = in.csz[k], sp = in.csp[k], dj = in.cdj[k];
                T ba = T(0), bb2 = T(0);
                _Pragma("unroll") for (int q = 0; q < C; ++q) {
                    const T cpq = in.ccp[k][q], zy = in.czy[k][q], py = in.cpy[k][q];
                    ba = fma(cpq, T(2) * zy - py, ba);
                    bb2 = fma(cpq, zy - py, bb2);
                }
                const T zy = in.czy[k][C], py = in.cpy[k][C];
                ba += T(2) * zy - py;
                bb2 += zy - py;
                const T av = (T(2) * sz - sp) - ba, bb = (sz - sp) - bb2;
                const T v = (dj + alpha * av) * ra;
                const T ep = alpha * (v - fmax(v, T(0)));
                const T x2 = (dj - ep) * ra + bb;
                ks.s[lo][k] = sz - alpha * ep;
                account(sp, sz, dj - ep, x2);
            }
        }
        stamp();
        // ---------------- phase 3: eta7 (box on [x_i; u_i]) and x_i, u_i of the half step:
        // L^T = Gamma' eta7 + sqrtQ (sum of the children's eta3) (operators.py:73-85)
        {
            const T(&xz)[RX][4] = in.xz;
            const T(&xp)[RX][4] = in.xp;
            const T(&uz)[RU][4] = in.uz;
            const T(&up)[RU][4] = in.up;
            v4 gxA[RX], gxW[RX], gxC[RX], guA[RU], guW[RU], guC[RU];
            if (BXN == 1) {
                const T(&d7x)[RX][4] = in.d7x;
                const T(&d7u)[RU][4] = in.d7u;
                const int o7 = p.E7 + (live ? i : 0) * (NX + NU);
                T lx[RX][4], hx[RX][4], lu[RU][4], hu[RU][4];
                if (p.nBnl <= 1) {
                    ld_rows_lds<T, NX>(bl_, lx);
                    ld_rows_lds<T, NX>(bl_ + (NX + NU), hx);
                    ld_rows_lds<T, NU>(bl_ + NX, lu);
                    ld_rows_lds<T, NU>(bl_ + (NX + NU) + NX, hu);
                } else {
                    cglbp<T> blo = (cglbp<T>)p.blo_nl + (size_t)in.bi * (NX + NU);
                    cglbp<T> bhi = (cglbp<T>)p.bhi_nl + (size_t)in.bi * (NX + NU);
                    ld_rows<T, NX>(blo, live, lx);
                    ld_rows<T, NX>(bhi, live, hx);
                    ld_rows<T, NU>(blo + NX, live, lu);
                    ld_rows<T, NU>(bhi + NX, live, hu);
                }
                T e7[RX][4], e7u[RU][4];
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (live && tok<NX>(rt, e)) {
                        const T v = (d7x[rt][e] + alpha * (T(2) * xz[rt][e] - xp[rt][e])) * ra;
                        fin(d7x[rt][e], v, box_apply_t(v, lx[rt][e], hx[rt][e], ctl), xz[rt][e] - xp[rt][e], ep, x2);
                    }
                    e7[rt][e] = ep;
                    gxA[rt][e] = ep;
                    gxW[rt][e] = d7x[rt][e] - ep;
                    gxC[rt][e] = x2;
                }
                st_rows<T, NX>(eo + o7, live, e7);
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    T ep = T(0), x2 = T(0);
                    if (live && tok<NU>(rt, e)) {
                        const T v = (d7u[rt][e] + alpha * (T(2) * uz[rt][e] - up[rt][e])) * ra;
                        fin(d7u[rt][e], v, box_apply_t(v, lu[rt][e], hu[rt][e], ctl), uz[rt][e] - up[rt][e], ep, x2);
                    }
                    e7u[rt][e] = ep;
                    guA[rt][e] = ep;
                    guW[rt][e] = d7u[rt][e] - ep;
                    guC[rt][e] = x2;
                }
                st_rows<T, NU>(eo + o7 + NX, live, e7u);
            } else {
                _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) gxA[rt] = gxW[rt] = gxC[rt] = v4{0, 0, 0, 0};
                _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) guA[rt] = guW[rt] = guC[rt] = v4{0, 0, 0, 0};
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
            st_rows<T, NX>(out + p.X0 + (size_t)(live ? i : 0) * NX, live, ox);
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                ou[rt][e] = uz[rt][e] - alpha * guA[rt][e];
                if (live && tok<NU>(rt, e)) account(up[rt][e], uz[rt][e], guW[rt][e], guC[rt][e]);
            }
            st_rows<T, NU>(out + p.U0 + (size_t)(live ? i : 0) * NU, live, ou);
        }
        stamp();
        // ---------------- phase 5: AVaR kernel projection of the family (cache.py:290-317)
        if (hm) {
            __syncthreads();  // the helper's leaf children are done
            if (LEAFP)
                _Pragma("unroll") for (int k = 0; k < C; ++k) ks.s[lo][k] = kh.s[lo][k];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (live) {
            const T al = in.al;
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
        if (hm) __syncthreads();  // the helper's scratch is rewritten by the next task
        stamp();
    };
    const int split = tk.split;
    const int nTL = (tk.l1 - tk.l0 + 15) >> 4;  // leaf tiles (split), then the parent ranges' tiles
    // diagnostics: every wave's [first task start, last task end] at stamps[32 + 2 gw]
    const unsigned long long w_t0 = kDiag && p.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
    for (int tt = hm ? (int)blockIdx.x : gw; tt < nTL + tk.t0[tk.nr]; tt += hm ? (int)gridDim.x : nwv) {
        if (hm && wv == 1) {
            // the helper: a leaf-parent tile's leaf children (phase 4 of the family), then the
            // task's two barriers
            if (tt >= nTL) {
                const int task = tt - nTL;
                int r = 0;
                while (r + 1 < tk.nr && task >= tk.t0[r + 1]) ++r;
                if (tk.lo[r] >= tk.mL) {
                    const int i = tk.lo[r] + 16 * (task - tk.t0[r]) + lo;
                    const bool live = i < tk.hi[r];
                    LeafIn<T, NX, BXL> lf[C];
                    _Pragma("unroll") for (int k = 0; k < C; ++k) lf[k].load(p, zp, pz, d, 1 + C * i + k, live, !split);
                    _Pragma("unroll") for (int k = 0; k < C; ++k) leaf_work(lf[k], 1 + C * i + k, k, live, !split, true);
                }
            }
            __syncthreads();
            __syncthreads();
            continue;
        }
        if (tt < nTL) {
            // a tile of 16 consecutive leaves (split): everything of the leaf but s_l
            const int l = tk.l0 + 16 * tt + lo;
            const bool live = l < tk.l1;
            LeafIn<T, NX, BXL> cur;
            cur.load(p, zp, pz, d, l, live, true);
            leaf_work(cur, l, 0, live, true, false);
            if (hm) {
                __syncthreads();
                __syncthreads();
            }
            continue;
        }
        const int task = tt - nTL;
        stp_on = kDiag && p.stamps != nullptr && task == p.cp_dbg;  // (diagnostics: the stamped task)
        int r = 0;
        while (r + 1 < tk.nr && task >= tk.t0[r + 1]) ++r;
        const int i0 = tk.lo[r] + 16 * (task - tk.t0[r]), iend = tk.hi[r];
        if (tk.lo[r] >= tk.mL) family(std::true_type{}, i0, iend, split);
        else family(std::false_type{}, i0, iend, split);
    }
    if (kDiag && p.stamps && (threadIdx.x & 63) == 0 && gw < 2000) {
        p.stamps[32 + 2 * gw] = w_t0;
        p.stamps[33 + 2 * gw] = __builtin_amdgcn_s_memrealtime();
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

template <class T, int NX, int NU, int C>
void launch_c(const Dev& p, Ctl* ctl, Bufs bf, double* part, int bx, const Cp3Tasks& tk, const double* img, int grid,
              int wpb, hipStream_t s) {
    const int bn = bx & 3, bl = (bx >> 2) & 3;
    const int g = grid, th = 64 * wpb;
    if (bn == 1 && bl == 1) k_cp4<T, NX, NU, C, 1, 1><<<g, th, 0, s>>>(p, ctl, bf, part, tk, img);
    else if (bn == 2 && bl == 2) k_cp4<T, NX, NU, C, 2, 2><<<g, th, 0, s>>>(p, ctl, bf, part, tk, img);
    else if (bn == 2 && bl == 1) k_cp4<T, NX, NU, C, 2, 1><<<g, th, 0, s>>>(p, ctl, bf, part, tk, img);
    else k_cp4<T, NX, NU, C, 1, 2><<<g, th, 0, s>>>(p, ctl, bf, part, tk, img);
}

}  // namespace

// compiled: fp64 at nx = 20, nu = 8 with C = 2 (the benchmark tree; C = 4 spills); every nonleaf and
// every leaf boxed or none of them (bits 0-1 / 2-3 of bx: 1 all, 2 none; mixed: k_cp3)
bool cp4_supported(bool f32, int nx, int nu, int C, int bx) {
    const int bn = bx & 3, bl = (bx >> 2) & 3;
    return !f32 && nx == 20 && nu == 8 && C == 2 && (bn == 1 || bn == 2) && (bl == 1 || bl == 2);
}
const char* cp4_name(bool f32, int nx, int nu) {
    (void)f32;
    (void)nx;
    (void)nu;
    return "k_cp4<double, 20, 8>";
}
void cp4_launch(const Dev& p, Ctl* ctl, Bufs bf, double* part, int C, int bx, const Cp3Tasks& tk, const double* img,
                int grid, int wpb, hipStream_t s) {
    (void)C;
    launch_c<double, 20, 8, 2>(p, ctl, bf, part, bx, tk, img, grid, wpb, s);
}

}  // namespace raocp
