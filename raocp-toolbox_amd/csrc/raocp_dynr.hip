// raocp_dynr.hip — the dynamics projection (cache.py:259-288) of REGULAR trees in two
// launches, as its own translation unit (host interface: raocp_dynr.h).
//
// Regular: one branching factor C (child k of node i is 1 + C i + k, stage t holds nodes
// [(C^t - 1) / (C - 1), (C^(t+1) - 1) / (C - 1))), one offline class per stage and one
// (A, B) pair per child slot of a stage (raocp_capi.hip checks it): the i.i.d. trees of
// BASELINE configs 2, 4, 5. Device form of the recursion (raocp_dyn.hip header), with the
// per-(slot, stage) table WT_k = [-Rinv B_k' ; A_k' - G B_k'] and RG = [Rinv ; G]:
//   backward, node i of stage t, children j = 1 + C i + k (q_j = -x_j at the leaves):
//     [d_i ; q_i + x_i] = RG u_i + sum_k WT_k q_j
//   forward:  u_i = K x_i + d_i ;  x_j = [Abar_k | B_k] [x_i ; d_i]   (x_0 = x0bar)
//
// The tree is cut into tiers at stages 0 = s_0 < s_1 < ... < s_T = N; tier k is C^(s_k)
// subtrees of L_k = s_(k+1) - s_k nonleaf levels, ONE workgroup each, every node address
// computed from (stage, subtree) — no index records. The whole grid is one workgroup per
// subtree of every tier (the host keeps it within the CU count, so every workgroup of a
// launch is resident at once and no wait depends on dispatch order):
//   k_dr_up   [deepest subtrees] .. [tier 1] [top] [stopping test]: a workgroup stages its
//             tables, x and u rows, waits until its C^L child subtrees have arrived (the
//             deepest tier waits for nothing: its boundary is the leaves), reads their
//             published q rows, sweeps its levels backward (d_i to global rows), publishes
//             its root's q row and arrives at its parent subtree's counter; the top bumps
//             the epoch.
//   k_dr_down [top] [tier 1] .. [deepest]: a workgroup stages its tables and [0 | d] rows,
//             waits for its parent subtree's flag (= the epoch), reads its root's x row,
//             sweeps forward (u_i and the children's x rows to the iterate) and sets its
//             own flag.
// A level is ONE workgroup barrier: every output row is a dot product over LDS rows, a
// split-k group of KS lanes per backward row (one per child slot, reduced by DPP), one lane
// per forward row. Tables are staged per tier in the order the lanes read them (16-B
// reads, padded strides spread the banks).
//
// Hand-offs (MI355X_MICROARCH.md, "Valid forms", row 1): the payload (a root's q row, a
// subtree's boundary x rows) is stored write-through (sc1) by every storing wave, which then
// drains (s_waitcnt vmcnt(0)); after a workgroup barrier ONE lane arrives (agent-scope
// atomic add) or stores the flag (sc1). The consumer polls that word with relaxed sc1 loads
// from one lane, joins a workgroup barrier, and reads every payload byte with sc1 loads
// (never through its L1). Every spin is bounded (DrPlan::timeout): a timed-out workgroup
// sets the error word and leaves; every workgroup of a later launch sees the error word at
// its start and leaves at once (the host reports it and clears the words, raocp_capi.hip).
// Counters are reset by their one consumer after its wait; flags carry the projection's
// epoch, so no host reset runs between launches.

#include "raocp_dynr.h"

namespace raocp {
namespace {

typedef double d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) d2v lds2;

__device__ __forceinline__ d2v ld2(const ldsd* p) { return *(const lds2*)p; }

// sum_e a[e] b[e], e < N (N even, both rows 16-B aligned): every load issued first
template <int N>
__device__ __forceinline__ double ldot(const ldsd* a, const ldsd* b) {
    static_assert(N % 2 == 0, "even row lengths");
    d2v x[N / 2], y[N / 2];
    _Pragma("unroll") for (int t = 0; t < N / 2; ++t) {
        x[t] = ld2(a + 2 * t);
        y[t] = ld2(b + 2 * t);
    }
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    _Pragma("unroll") for (int t = 0; t < N / 2; t += 2) {
        s0 = fma(x[t].x, y[t].x, s0);
        s1 = fma(x[t].y, y[t].y, s1);
        if (t + 1 < N / 2) {
            s2 = fma(x[t + 1].x, y[t + 1].x, s2);
            s3 = fma(x[t + 1].y, y[t + 1].y, s3);
        }
    }
    return (s0 + s1) + (s2 + s3);
}

template <int CTRL>
__device__ __forceinline__ double dpp_x(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// sum over the KS consecutive lanes of a split-k group (all live or all idle); every lane
// of the group ends with the same value
template <int KS>
__device__ __forceinline__ double ks_sum(double v) {
    if constexpr (KS >= 2) v += dpp_x<0xB1>(v);  // lane ^ 1
    if constexpr (KS >= 4) v += dpp_x<0x4E>(v);  // lane ^ 2
    return v;
}

// LDS barrier that does not wait for this wave's global stores (s_barrier alone does not
// order LDS: the lgkmcnt wait does)
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// every storing wave drains its global stores, then the workgroup meets (hand-off publish)
__device__ __forceinline__ void drain_sync() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ unsigned ld_u32(const unsigned* p) {
    return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_u32(unsigned* p, unsigned v) {
    __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS-DMA staging (global_load_lds_dwordx4): a wave instruction lands 64 16-B chunks at
// dst + 1 KB * group, each lane reading its own source chunk. Group g of a call goes to wave
// (g + rot) mod nw and rot advances past the call, so the issue of many small ranges is
// spread over the waves.
struct Dma {
    int rot = 0;
    template <class SrcF>
    __device__ __forceinline__ void gen(ldsd* dst, int chunks, SrcF src) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
        const int g0 = ((wave - rot) % nw + nw) % nw;
        for (int c0 = g0 * 64; c0 < chunks; c0 += nw * 64) {
            const int ch = c0 + lane;
            if (ch < chunks) __builtin_amdgcn_global_load_lds((const glbd*)src(ch), dst + 2 * c0, 16, 0, 0);
        }
        rot += (chunks + 63) >> 6;
    }
    // n (even) contiguous doubles, 16-B aligned
    __device__ __forceinline__ void range(ldsd* dst, const double* src, int n) {
        gen(dst, n >> 1, [=](int ch) { return src + 2 * ch; });
    }
    // rows of cols (even) doubles at source stride cols -> LDS rows of w doubles, zero tail
    __device__ __forceinline__ void rows(ldsd* dst, int w, const double* src, int cols, int nrows, const double* zp) {
        const int cpr = w >> 1, cc = cols >> 1;
        gen(dst, nrows * cpr, [=](int ch) {
            const int r = ch / cpr, c = ch - r * cpr;
            return c < cc ? src + (size_t)r * cols + 2 * c : zp;
        });
    }
};

__device__ __forceinline__ int ipow(int b, int e) {
    int v = 1;
    for (int i = 0; i < e; ++i) v *= b;
    return v;
}
// first node of stage t
__device__ __forceinline__ int stage0(int C, int t) { return (ipow(C, t) - 1) / (C - 1); }

// bounded spin of one lane until *w == v; false (error word set) on a timeout
__device__ __forceinline__ bool wait_word(const unsigned* w, unsigned v, const DrPlan& pl, int* s_ok) {
    if (threadIdx.x == 0) {
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        while (ld_u32(w) != v) {
            if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > pl.timeout) {
                *s_ok = 0;
                st_u32(pl.sync + 1, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    return *s_ok != 0;
}

struct Stamps {
    unsigned long long ts[16];
    int n;
};
__device__ __forceinline__ void stamp(const DrPlan& pl, Stamps& s) {
    if (pl.stamps && threadIdx.x == 0 && s.n < 16) s.ts[s.n++] = __builtin_amdgcn_s_memrealtime();
}
// the first subtree of each tier writes its stamps to slots [16 k, 16 k + 16)
__device__ __forceinline__ void stamp_flush(const DrPlan& pl, const Stamps& s, int k, int o) {
    if (pl.stamps && threadIdx.x == 0 && o == 0 && k < 4)
        for (int q = 0; q < 16; ++q) pl.stamps[16 * k + q] = q < s.n ? s.ts[q] : 0ull;
}

// ---- one backward level: nl nodes of stage t (subtree rows xq_l / u_l), their children's
// q rows xq_c (sign -1: the children are leaves, xq_c holds x). Item (node n, row r, slot k),
// KS lanes per row. Rows r < nu are d_i (to global dl), rows r >= nu overwrite x_i in place
// with q_i = acc - x_i.
template <int NX, int NU, int C>
__device__ __forceinline__ void back_level(const ldsd* tb, ldsd* xq_l, const ldsd* xq_c, const ldsd* u_l, int nl,
                                           double sign, glbd* dl) {
    constexpr int R = NX + NU, KS = dr_ks(C), SX = dr_stride(NX), UP = dr_up(NU, C), NUP = dr_nup(NU, C);
    const int items = nl * R * KS;
    for (int it = threadIdx.x; it < items; it += blockDim.x) {
        const int k = it % KS, rq = it / KS, r = rq % R, n = rq / R;
        double acc = 0.0;
        if (C == KS || k < C) acc = sign * ldot<NX>(tb + (r * KS + k) * SX, xq_c + (n * C + k) * SX);
        acc += ldot<UP>(tb + R * KS * SX + r * NUP + k * UP, u_l + n * NUP + k * UP);
        acc = ks_sum<KS>(acc);
        if (k == 0) {
            if (r < NU) {
                dl[(size_t)n * NU + r] = acc;
            } else {
                ldsd* xr = xq_l + n * SX + (r - NU);
                *xr = acc - *xr;
            }
        }
    }
}

// ---- one forward level: nl nodes with rows xd_l = [x_i | d_i]; the children's x rows
// (items n C nx + k nx + r) go to the iterate (zx_c: the first child's row there; sc: the
// children are another tier's roots, stored write-through) and to xd_c when the children
// are nonleaf nodes of this subtree; then the u rows u_i = K x_i + d_i (items after them).
template <int NX, int NU, int C>
__device__ __forceinline__ void fwd_level(const ldsd* tf, const ldsd* xd_l, ldsd* xd_c, int nl, glbd* zx_c, glbd* zu_l,
                                          bool sc) {
    constexpr int SF = dr_stride(NX + NU), SX = dr_stride(NX), CX = C * NX;
    const int nxi = nl * CX, items = nxi + nl * NU;
    for (int it = threadIdx.x; it < items; it += blockDim.x) {
        if (it < nxi) {
            const int n = it / CX, w = it - n * CX, k = w / NX, r = w - k * NX;
            const double v = ldot<NX + NU>(tf + (k * NX + r) * SF, xd_l + n * SF);
            const int j = n * C + k;
            if (xd_c) xd_c[j * SF + r] = v;
            if (sc) st_sc1((double*)(zx_c + (size_t)j * NX + r), v);
            else zx_c[(size_t)j * NX + r] = v;
        } else {
            const int e = it - nxi, n = e / NU, r = e - n * NU;
            const ldsd* xd = xd_l + n * SF;
            zu_l[(size_t)n * NU + r] = ldot<NX>(tf + CX * SF + r * SX, xd) + xd[NX + r];
        }
    }
}

// the tier and subtree of this workgroup from the plan's block ranges
__device__ __forceinline__ void role(const DrPlan& pl, bool up, int& k, int& o) {
    const int b = blockIdx.x;
    k = 0;
    for (int q = 0; q < pl.T; ++q) {
        const int b0 = up ? pl.t[q].bup : pl.t[q].bdn;
        if (b >= b0 && b < b0 + pl.t[q].nsub) k = q;
    }
    o = b - (up ? pl.t[k].bup : pl.t[k].bdn);
}

template <int NX, int NU, int C, int BS>
__global__ void __launch_bounds__(BS) k_dr_up(DrPlan pl, Bufs bf, int zsel, const Ctl* __restrict__ ctl, ChkArg ck) {
    constexpr int R = NX + NU, KS = dr_ks(C), SX = dr_stride(NX), NUP = dr_nup(NU, C), SB1 = dr_back_n(NX, NU, C);
    (void)R;
    (void)KS;
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ Stamps stp;
    __shared__ int s_ok;
    const int tid = threadIdx.x;
    if (ck.on && (int)blockIdx.x == pl.nblk) {  // the previous CP iteration's stopping test
        if (tid < 64) cp_check_wave(ck);
        return;
    }
    if (tid == 0) {
        stp.n = 0;
        s_ok = 1;
    }
    stamp(pl, stp);
    int k, o;
    role(pl, true, k, o);
    const DrTier tt = pl.t[k];
    const int D = pl.T - 1, L = tt.L;
    const bool deepest = k == D;
    glbd* z = pick3(bf, zsel);
    ldsd* sm = (ldsd*)smem_;
    // [TB (L stages) | XQ (levels 0 .. L, SX) | U (levels 0 .. L-1, NUP)]
    const int nnl = (ipow(C, L) - 1) / (C - 1), nall = nnl + ipow(C, L);
    ldsd* TB = sm;
    ldsd* XQ = TB + L * SB1;
    ldsd* U = XQ + nall * SX;
    // prologue: everything this subtree's own data holds, issued at once
    Dma dm;
    dm.range(TB, pl.bimg + (size_t)tt.s0 * SB1, L * SB1);
    for (int l = 0, off = 0; l <= L; ++l) {
        const int cnt = ipow(C, l), g = stage0(C, tt.s0 + l) + o * cnt;
        if (l < L || deepest) dm.rows(XQ + off * SX, SX, (const double*)z + pl.X0 + (size_t)g * NX, NX, cnt, pl.zpage);
        if (l < L) {
            if (NUP == NU) dm.range(U + off * NUP, (const double*)z + pl.U0 + (size_t)g * NU, cnt * NU);
            else dm.rows(U + off * NUP, NUP, (const double*)z + pl.U0 + (size_t)g * NU, NU, cnt, pl.zpage);
        }
        off += cnt;
    }
    const unsigned err = ld_u32(pl.sync + 1);
    const bool work = !(ctl && ctl->done);
    const unsigned ep = k == 0 ? ld_u32(pl.sync) : 0u;
    if (err) {
        dma_wait();
        return;
    }
    if (!deepest) {  // the child subtrees' q rows: arrivals, then sc1 loads
        const int nb = ipow(C, L), gb = stage0(C, tt.s0 + L) + o * nb;
        unsigned* cnt = pl.sync + 2 + tt.w0 + o;
        if (!wait_word(cnt, (unsigned)nb, pl, &s_ok)) {
            dma_wait();
            return;
        }
        if (tid == 0) st_u32(cnt, 0u);
        stamp(pl, stp);
        ldsd* xb = XQ + nnl * SX;
        for (int e = tid; e < nb * NX; e += blockDim.x) {
            const int r = e / NX, c = e - r * NX;
            xb[r * SX + c] = ld_sc1(pl.qbuf + (size_t)(gb + r) * NX + c);
        }
    }
    dma_wait();
    lds_sync();
    stamp(pl, stp);
    if (work) {
        for (int l = L - 1; l >= 0; --l) {
            const int cnt = ipow(C, l), off = (cnt - 1) / (C - 1), offc = off + cnt;
            const int g = stage0(C, tt.s0 + l) + o * cnt;
            back_level<NX, NU, C>(TB + l * SB1, XQ + off * SX, XQ + offc * SX, U + off * NUP, cnt,
                                  (deepest && l == L - 1) ? -1.0 : 1.0, (glbd*)pl.dbuf + (size_t)g * NU);
            lds_sync();
        }
    }
    stamp(pl, stp);
    if (k > 0) {  // publish the root's q row, arrive at the parent subtree's counter
        const int root = stage0(C, tt.s0) + o;
        if (tid < NX) st_sc1(pl.qbuf + (size_t)root * NX + tid, XQ[tid]);
        drain_sync();
        const DrTier& pt = pl.t[k - 1];
        if (tid == 0 && !(pl.fault == 1 && deepest && o == 0))
            __hip_atomic_fetch_add((gu32*)(pl.sync + 2 + pt.w0 + o / ipow(C, pt.L)), 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    } else {  // the top: the projection's epoch for k_dr_down's flags
        drain_sync();
        if (tid == 0) st_u32(pl.sync, ep + 1u);
    }
    stamp(pl, stp);
    stamp_flush(pl, stp, k, o);
}

template <int NX, int NU, int C, int BS>
__global__ void __launch_bounds__(BS) k_dr_down(DrPlan pl, Bufs bf, int zsel, const Ctl* __restrict__ ctl) {
    constexpr int SF = dr_stride(NX + NU), SF1 = dr_fwd_n(NX, NU, C);
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ Stamps stp;
    __shared__ int s_ok;
    const int tid = threadIdx.x;
    if (tid == 0) {
        stp.n = 0;
        s_ok = 1;
    }
    stamp(pl, stp);
    int k, o;
    role(pl, false, k, o);
    const DrTier tt = pl.t[k];
    const int D = pl.T - 1, L = tt.L;
    glbd* z = pick3(bf, zsel);
    ldsd* sm = (ldsd*)smem_;
    // [TF (L stages) | XD (levels 0 .. L-1, SF): [x | d | 0]]
    ldsd* TF = sm;
    ldsd* XD = TF + L * SF1;
    Dma dm;
    dm.range(TF, pl.fimg + (size_t)tt.s0 * SF1, L * SF1);
    constexpr int cpr = SF / 2, cx = NX / 2, cd = (NX + NU) / 2;
    for (int l = 0, off = 0; l < L; ++l) {
        const int cnt = ipow(C, l), g = stage0(C, tt.s0 + l) + o * cnt;
        const double* dl = pl.dbuf + (size_t)g * NU;
        const double* zp = pl.zpage;
        dm.gen(XD + off * SF, cnt * cpr, [=](int ch) {
            const int r = ch / cpr, c = ch - r * cpr;
            return (c >= cx && c < cd) ? dl + (size_t)r * NU + 2 * (c - cx) : zp;
        });
        off += cnt;
    }
    const unsigned err = ld_u32(pl.sync + 1);
    const bool work = !(ctl && ctl->done);
    const unsigned ep = ld_u32(pl.sync);
    if (err) {
        dma_wait();
        return;
    }
    const int root = stage0(C, tt.s0) + o;
    double xr = 0.0;
    if (k == 0) {
        if (tid < NX) {
            xr = ((const glbd*)pl.x0)[tid];
            if (work) z[pl.X0 + tid] = xr;  // x_0 = x0bar (cache.py:282)
        }
    } else {  // the parent subtree's flag, then the root's x row (sc1)
        const DrTier& pt = pl.t[k - 1];
        if (!wait_word(pl.sync + 2 + pl.S + pt.w0 + o / ipow(C, pt.L), ep, pl, &s_ok)) {
            dma_wait();
            return;
        }
        stamp(pl, stp);
        if (tid < NX) xr = ld_sc1((const double*)z + pl.X0 + (size_t)root * NX + tid);
    }
    dma_wait();
    lds_sync();  // (the LDS-DMA rows have landed: the root's x goes into its row after them)
    if (tid < NX) XD[tid] = xr;
    lds_sync();
    stamp(pl, stp);
    if (work) {
        for (int l = 0; l < L; ++l) {
            const int cnt = ipow(C, l), off = (cnt - 1) / (C - 1);
            const int g = stage0(C, tt.s0 + l) + o * cnt, gc = stage0(C, tt.s0 + l + 1) + o * cnt * C;
            const bool last = l + 1 == L;
            fwd_level<NX, NU, C>(TF + l * SF1, XD + off * SF, last ? nullptr : XD + (off + cnt) * SF, cnt,
                                 z + pl.X0 + (size_t)gc * NX, z + pl.U0 + (size_t)g * NU, last && k < D);
            lds_sync();
        }
    }
    stamp(pl, stp);
    if (k < D) {  // the boundary x rows are out: release the child subtrees
        drain_sync();
        if (tid == 0) st_u32(pl.sync + 2 + pl.S + tt.w0 + o, ep);
    }
    stamp(pl, stp);
    stamp_flush(pl, stp, k, o);
}

template <int NX, int NU, int C>
void up_t(const DrPlan& pl, int block, size_t lds, Bufs bf, int zsel, const Ctl* ctl, ChkArg ck, hipStream_t s) {
    const int grid = pl.nblk + (ck.on ? 1 : 0);
    if (block > 512) {
        auto kf = k_dr_up<NX, NU, C, 1024>;
        (void)hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        kf<<<grid, 1024, lds, s>>>(pl, bf, zsel, ctl, ck);
    } else {
        auto kf = k_dr_up<NX, NU, C, 512>;
        (void)hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        kf<<<grid, 512, lds, s>>>(pl, bf, zsel, ctl, ck);
    }
}
template <int NX, int NU, int C>
void down_t(const DrPlan& pl, int block, size_t lds, Bufs bf, int zsel, const Ctl* ctl, hipStream_t s) {
    if (block > 512) {
        auto kf = k_dr_down<NX, NU, C, 1024>;
        (void)hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        kf<<<pl.nblk, 1024, lds, s>>>(pl, bf, zsel, ctl);
    } else {
        auto kf = k_dr_down<NX, NU, C, 512>;
        (void)hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        kf<<<pl.nblk, 512, lds, s>>>(pl, bf, zsel, ctl);
    }
}

}  // namespace

bool dr_supported(int nx, int nu, int C) { return nx == 20 && nu == 8 && (C == 2 || C == 3 || C == 4); }

size_t dr_lds_up(int nx, int nu, int C, int L, bool deepest) {
    (void)deepest;
    long nnl = 0, p = 1;
    for (int l = 0; l < L; ++l, p *= C) nnl += p;
    const long nall = nnl + p;
    return 8 * ((size_t)L * dr_back_n(nx, nu, C) + (size_t)nall * dr_stride(nx) + (size_t)nnl * dr_nup(nu, C));
}
size_t dr_lds_down(int nx, int nu, int C, int L) {
    long nnl = 0, p = 1;
    for (int l = 0; l < L; ++l, p *= C) nnl += p;
    return 8 * ((size_t)L * dr_fwd_n(nx, nu, C) + (size_t)nnl * dr_stride(nx + nu));
}

void dr_launch_up(const DrPlan& pl, int nx, int nu, int block, size_t lds, Bufs bf, int zsel, const Ctl* ctl,
                  ChkArg ck, hipStream_t s) {
    if (nx == 20 && nu == 8) {
        if (pl.C == 2) up_t<20, 8, 2>(pl, block, lds, bf, zsel, ctl, ck, s);
        else if (pl.C == 3) up_t<20, 8, 3>(pl, block, lds, bf, zsel, ctl, ck, s);
        else up_t<20, 8, 4>(pl, block, lds, bf, zsel, ctl, ck, s);
    }
}
void dr_launch_down(const DrPlan& pl, int nx, int nu, int block, size_t lds, Bufs bf, int zsel, const Ctl* ctl,
                    hipStream_t s) {
    if (nx == 20 && nu == 8) {
        if (pl.C == 2) down_t<20, 8, 2>(pl, block, lds, bf, zsel, ctl, s);
        else if (pl.C == 3) down_t<20, 8, 3>(pl, block, lds, bf, zsel, ctl, s);
        else down_t<20, 8, 4>(pl, block, lds, bf, zsel, ctl, s);
    }
}
const char* dr_name_up(int nx, int nu) { return nx == 20 && nu == 8 ? "k_dr_up<20, 8>" : "k_dr_up"; }
const char* dr_name_down(int nx, int nu) { return nx == 20 && nu == 8 ? "k_dr_down<20, 8>" : "k_dr_down"; }

}  // namespace raocp
