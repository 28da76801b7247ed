// raocp_dynr.hip — the dynamics projection (cache.py:259-288) of REGULAR trees in ONE launch,
// as its own translation unit (host interface: raocp_dynr.h).
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
// computed from (stage, subtree). The grid is one workgroup per subtree of every tier (the
// host keeps it within the resident capacity, so every workgroup is resident at once and no
// wait depends on the dispatch order). A workgroup
//   1. stages its x and u rows and its backward tables (LDS-DMA, in the order they are used),
//   2. (above the deepest tier) waits for its C^L child subtrees' q rows,
//   3. sweeps its levels backward: d_i into its [x | d] rows, q_i over x_i in place,
//   4. publishes its root's q row (below the top),
//   5. (below the top) waits for its root's x row from the parent subtree (the top takes x0bar),
//   6. sweeps its levels forward: children's x rows and u_i into LDS,
//   7. publishes its boundary x rows to the child subtrees, then writes x and u to the iterate.
// Nothing is written to global memory during a sweep, and d never leaves the LDS.
//
// A level: lane s of a group holds its table row in registers (one per (row, slot) backward,
// one per child x row or u row forward: the u rows are [K | I] so both are 28-long dots) and
// the group's nodes are read as broadcast 16-B LDS reads. The tables of a workgroup's L stages
// sit in L LDS slots, refilled with the forward tables (LDS-DMA) once the backward sweep is
// done (below the top: during the wait for the root's x row) or, in the top, slot by slot as
// the backward sweep frees them; the top's forward levels wait only for their own table
// (s_waitcnt vmcnt(N), N = the younger table DMAs: every wave issues a fixed count per table).
//
// Hand-offs (MI355X_MICROARCH.md, handoff-1to1): 8-byte granules {32-bit half of a double,
// 32-bit tag} stored with relaxed agent-scope (sc1) stores, polled by the consumer's lanes
// with relaxed agent-scope loads until every granule carries the projection's tag — no
// separate flag, no drain. The tag is sync[0] + 1, read by every workgroup at its start; the
// top stores it to sync[0] when it is done (all workgroups have read it by then: the top's
// backward sweep waited on every one of them). Every wait is bounded (DrPlan::timeout): a
// timed-out workgroup sets the error word and leaves; every workgroup of a later launch sees
// the error word at its start and leaves at once (the host reports it and clears the words
// and the granules, raocp_capi.hip).

#include "raocp_dynr.h"

namespace raocp {
namespace {

typedef double d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) d2v lds2;
typedef __attribute__((address_space(1))) d2v glb2;
typedef __attribute__((address_space(3))) unsigned ldsu;

__device__ __forceinline__ d2v ld2(const ldsd* p) { return *(const lds2*)p; }

// LDS barrier that does not wait for this wave's global memory operations
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }


// {sync[0], sync[1]} by a scalar load (lgkmcnt, outside the vmcnt queue of the counted
// waits; the words were written by earlier launches)
__device__ __forceinline__ unsigned long long sload_pair(const unsigned* p) {
    unsigned long long v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}
__device__ __forceinline__ unsigned ld_u32(const unsigned* p) {
    return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_u32(unsigned* p, unsigned v) {
    __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_gran(const unsigned long long* p) {
    return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_gran(unsigned long long* p, unsigned v, unsigned tag) {
    __hip_atomic_store((gu64*)p, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS-DMA staging (global_load_lds_dwordx4): a wave instruction lands 64 16-B chunks at
// dst + 1 KB * group, each lane reading its own source chunk. gen() spreads the groups of a
// call over the waves from a rotating start (row ranges; TableDma below: tables).
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

// every lane polls granules g = tid + i * blockDim (g < n) of src until each carries tag, and
// puts their halves at dst[g]; false (error word set) on a timeout, or as soon as another
// workgroup has set the error word (a missing hand-off then costs one timeout, not one per tier)
//
// k_dr assumes its grid has the device's CUs to itself: the host checks that the grid is
// resident (occupancy x CUs), which another kernel running beside it on the same device (a
// second context's stream) can break; a workgroup that is never scheduled turns into the
// bounded wait's RAOCP_ERR_STATE, not a hang
//
// Every lane polls its own granules from the start and keeps the ones that carry the tag, so
// the payload is read once, as soon as it is there (round 4 had one wave wait for the last
// granule of each row first and then every lane read its granules: one more dependent round
// trip per hand-off, 1.0 us more per projection at config 2, profiles/r05/dr_poll.log).
__device__ __forceinline__ bool poll_gran(const unsigned long long* src, int n, unsigned tag, ldsu* dst,
                                          long long timeout, unsigned* sync, int& s_ok) {
    const int tid = threadIdx.x, bs = blockDim.x;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    bool bad = false;
    unsigned got = 0;
    for (;;) {
        unsigned long long v[kDrMaxGran];
        _Pragma("unroll") for (int i = 0; i < kDrMaxGran; ++i) {
            const int g = tid + i * bs;
            if (g < n && !((got >> i) & 1u)) v[i] = ld_gran(src + g);
        }
        bool all = true;
        _Pragma("unroll") for (int i = 0; i < kDrMaxGran; ++i) {
            const int g = tid + i * bs;
            if (g < n && !((got >> i) & 1u)) {
                if ((unsigned)(v[i] >> 32) == tag) {
                    dst[g] = (unsigned)v[i];
                    got |= 1u << i;
                } else {
                    all = false;
                }
            }
        }
        if (all) break;
        // another workgroup's timeout (the error word): this wait cannot complete either
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout || ld_u32(sync + 1) != 0u) {
            bad = true;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    if (bad) {
        s_ok = 0;
        st_u32(sync + 1, 1u);
    }
    __syncthreads();
    return s_ok != 0;
}
// granules g < n from the LDS dwords src[g], tag in the high half
__device__ __forceinline__ void publish(unsigned long long* dst, int n, unsigned tag, const ldsu* src) {
    for (int g = threadIdx.x; g < n; g += blockDim.x) st_gran(dst + g, src[g], tag);
}

// diagnostics: up to 30 s_memrealtime stamps of the first subtree of each tier, and its
// shader-clock cycles (s_memtime) over the same span
struct Stamps {
    unsigned long long ts[30];
    unsigned long long c0;
    int n;
};
__device__ __forceinline__ void stamp(const DrPlan& pl, Stamps& s) {
    if (kDiag && pl.stamps && threadIdx.x == 0 && s.n < 30) {
        if (s.n == 0) s.c0 = __builtin_amdgcn_s_memtime();
        s.ts[s.n++] = __builtin_amdgcn_s_memrealtime();
    }
}
// every workgroup (diagnostics, tools/dr_skew.py): slots 1024 + 3 b + {0 start, 1 backward
// sweep done, 2 end}
__device__ __forceinline__ void wg_stamp(const DrPlan& pl, int q) {
    if (kDiag && pl.stamps && threadIdx.x == 0)
        pl.stamps[1024 + 3 * blockIdx.x + q] = __builtin_amdgcn_s_memrealtime();
}
// slots [32 k, 32 k + 30): the stamps; 32 k + 30: the end; 32 k + 31: cycles from the first
// stamp to the end
__device__ __forceinline__ void stamp_flush(const DrPlan& pl, const Stamps& s, int k, int o) {
    if (kDiag && pl.stamps && threadIdx.x == 0 && o == 0 && k < 4) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
        for (int q = 0; q < 30; ++q) pl.stamps[32 * k + q] = q < s.n ? s.ts[q] : 0ull;
        pl.stamps[32 * k + 30] = t1;
        pl.stamps[32 * k + 31] = c1 - s.c0;
    }
}

// node blocks of a level of cnt nodes over NG groups: UN (<= UMAX) consecutive nodes per group
// and pass (two or more once the level has more than two nodes, so fewer waves read the
// level's table), passes of NG UN nodes
template <int cnt, int NG, int UMAX>
struct NodeSplit {
    static constexpr int want = cnt <= 2 ? 1 : ((cnt + NG - 1) / NG > 2 ? (cnt + NG - 1) / NG : 2);
    static constexpr int UN = want < UMAX ? want : UMAX;
};

// ---- one backward level: cnt nodes with [x | d] rows xd (stride NX + NU), their children's
// rows qc (stride qs: q rows, or the leaves' x rows with sign -1), u rows ul. Group g of GS
// lanes takes nodes g UN .. g UN + UN - 1; lane s = (row r, slot k): KS lanes per output row,
// reduced by DPP. Rows r < NU are d_i (into the d part), rows r >= NU overwrite x_i with
// q_i = acc - x_i.
template <int CTRL>
__device__ __forceinline__ double dpp_x(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
template <int KS>
__device__ __forceinline__ double ks_sum(double v) {
    if constexpr (KS >= 2) v += dpp_x<0xB1>(v);  // lane ^ 1
    if constexpr (KS >= 4) v += dpp_x<0x4E>(v);  // lane ^ 2
    return v;
}

template <int NX, int NU, int C, int BS, int UMAX, int cnt>
__device__ __forceinline__ void back_level(const ldsd* tb, ldsd* xd, const ldsd* qc, int qs, const ldsd* ul,
                                           double sign) {
    constexpr int KS = dr_ks(C), UP = dr_up(NU, C), NEB = dr_neb(NX, NU, C), GS = dr_gsb(NX, NU, C);
    constexpr int LB = dr_lb(NX, NU, C), SXD = NX + NU, NG = BS / GS, UN = NodeSplit<cnt, NG, UMAX>::UN;
    const int s = threadIdx.x % GS, g0 = (threadIdx.x / GS) * UN;
    if (g0 >= cnt) return;
    const int r = s / KS, k = s - r * KS;
    const bool live = s < LB;
    d2v w[NEB / 2];
    _Pragma("unroll") for (int p = 0; p < NEB / 2; ++p) w[p] = live ? ld2(tb + 2 * (p * LB + s)) : d2v{0.0, 0.0};
    // a lane of a missing slot (k >= C) reads slot 0's row against its zero table row; a node
    // past the level's end repeats the block's first
    const ldsd* qk = qc + (k < C ? k : 0) * qs;
    const ldsd* uk = ul + k * UP;
    for (int n0 = g0; n0 < cnt; n0 += NG * UN) {
    int nn[UN];
    _Pragma("unroll") for (int h = 0; h < UN; ++h) nn[h] = n0 + h < cnt ? n0 + h : n0;
    d2v q[UN][NX / 2], u[UN][UP / 2];
    double xo[UN];  // x_i entry r - NU (read with the rows: q_i = acc - x_i)
    _Pragma("unroll") for (int p = 0; p < NX / 2; ++p)
        _Pragma("unroll") for (int h = 0; h < UN; ++h) q[h][p] = ld2(qk + nn[h] * C * qs + 2 * p);
    _Pragma("unroll") for (int p = 0; p < UP / 2; ++p)
        _Pragma("unroll") for (int h = 0; h < UN; ++h) u[h][p] = ld2(uk + nn[h] * NU + 2 * p);
    _Pragma("unroll") for (int h = 0; h < UN; ++h) xo[h] = xd[nn[h] * SXD + (r >= NU && live ? r - NU : 0)];
    _Pragma("unroll") for (int h = 0; h < UN; ++h) {
        d2v a = {0.0, 0.0}, b = {0.0, 0.0}, c = {0.0, 0.0};
        _Pragma("unroll") for (int p = 0; p < NX / 2; p += 2) {
            a += w[p] * q[h][p];
            if (p + 1 < NX / 2) b += w[p + 1] * q[h][p + 1];
        }
        _Pragma("unroll") for (int p = 0; p < UP / 2; ++p) c += w[NX / 2 + p] * u[h][p];
        const double acc = ks_sum<KS>(sign * ((a.x + a.y) + (b.x + b.y)) + (c.x + c.y));
        if (live && k == 0 && (h == 0 || n0 + h < cnt)) {
            ldsd* row = xd + nn[h] * SXD;
            if (r < NU) row[NX + r] = acc;
            else row[r - NU] = acc - xo[h];
        }
    }
    }
}

// ---- one forward level: cnt nodes with [x | d] rows xd; lane s < C NX of a group is the
// child x row (slot s / NX, entry s % NX) = [Abar_k | B_k] row . [x ; d] into the children's
// rows xc (stride xs); lanes C NX .. C NX + NU - 1 are u_i = [K | I] row . [x ; d] into ul.
template <int NX, int NU, int C, int BS, int UMAX, int cnt>
__device__ __forceinline__ void fwd_level(const ldsd* tf, const ldsd* xd, ldsd* xc, int xs, ldsd* ul) {
    constexpr int NEF = NX + NU, GS = dr_gsf(NX, NU, C), LF = dr_lf(NX, NU, C), SXD = NX + NU;
    constexpr int NG = BS / GS, UN = NodeSplit<cnt, NG, UMAX>::UN;
    const int s = threadIdx.x % GS, g0 = (threadIdx.x / GS) * UN;
    if (g0 >= cnt || s >= LF) return;
    d2v w[NEF / 2];
    _Pragma("unroll") for (int p = 0; p < NEF / 2; ++p) w[p] = ld2(tf + 2 * (p * LF + s));
    for (int n0 = g0; n0 < cnt; n0 += NG * UN) {
    int nn[UN];
    _Pragma("unroll") for (int h = 0; h < UN; ++h) nn[h] = n0 + h < cnt ? n0 + h : n0;
    d2v v[UN][NEF / 2];
    _Pragma("unroll") for (int p = 0; p < NEF / 2; ++p)
        _Pragma("unroll") for (int h = 0; h < UN; ++h) v[h][p] = ld2(xd + nn[h] * SXD + 2 * p);
    _Pragma("unroll") for (int h = 0; h < UN; ++h) {
        if (h > 0 && n0 + h >= cnt) break;
        d2v a = {0.0, 0.0}, b = {0.0, 0.0};
        _Pragma("unroll") for (int p = 0; p < NEF / 2; p += 2) {
            a += w[p] * v[h][p];
            if (p + 1 < NEF / 2) b += w[p + 1] * v[h][p + 1];
        }
        const double acc = (a.x + a.y) + (b.x + b.y);
        const int m = nn[h];
        if (s < C * NX) {
            const int k = s / NX, r = s - k * NX;
            xc[(m * C + k) * xs + r] = acc;
        } else {
            ul[m * NU + (s - C * NX)] = acc;
        }
    }
    }
}

// the tier and subtree of this workgroup
__device__ __forceinline__ void role(const DrPlan& pl, int& k, int& o) {
    const int b = blockIdx.x;
    k = 0;
    for (int q = 1; q < pl.T; ++q)
        if (b >= pl.t[q].b0 && b < pl.t[q].b0 + pl.t[q].nsub) k = q;
    o = b - pl.t[k].b0;
}

constexpr int cpow(int b, int e) { return e == 0 ? 1 : b * cpow(b, e - 1); }

// f(std::integral_constant<int, I>) for I = A .. B - 1: level indices as constants
template <int A, int B, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (A < B) {
        f(std::integral_constant<int, A>{});
        static_for<A + 1, B>(f);
    }
}

// table DMA with a fixed issue count per wave (IPW instructions of 64 chunks; a wave past the
// table's last group repeats that group: the same bytes to the same LDS place), so every
// counted wait is an immediate
template <int N, int NW>
struct TableDma {
    static constexpr int CH = N / 2, NI = (CH + 63) / 64, IPW = (NI + NW - 1) / NW;
    static __device__ __forceinline__ void issue(ldsd* dst, const double* src) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        _Pragma("unroll") for (int j = 0; j < IPW; ++j) {
            const int gi = wave + j * NW < NI ? wave + j * NW : NI - 1;
            const int ch = gi * 64 + lane;
            if (ch < CH) __builtin_amdgcn_global_load_lds((const glbd*)(src + 2 * ch), dst + 128 * gi, 16, 0, 0);
        }
    }
};

template <int N>
__device__ __forceinline__ void wait_vm_c() {
    static_assert(N >= 0, "count");
    if constexpr (N >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// one tier's subtree o (L nonleaf levels): steps 1-7 of the header
template <int NX, int NU, int C, int BS, int UMAX, int L>
__device__ __forceinline__ void tier_body(const DrPlan& pl, int k, int o, glbd* z, unsigned tag, bool work,
                                          Stamps& stp, int& s_ok, ldsd* sm) {
    constexpr int SXD = NX + NU, TBN = dr_tb_n(NX, NU, C), TFN = dr_tf_n(NX, NU, C), SLOT = dr_slot_n(NX, NU, C);
    constexpr int G = 2 * NX, NW = BS / 64;
    constexpr int NB = cpow(C, L), NNL = (NB - 1) / (C - 1);
    typedef TableDma<TBN, NW> TB;
    typedef TableDma<TFN, NW> TF;
    const int tid = threadIdx.x;
    const DrTier tt = pl.t[k];
    const int s0 = tt.s0;
    const bool deepest = k == pl.T - 1, top = k == 0;
    // LDS: [L table slots | XD: NNL rows [x | d] | XL: NB boundary rows x / q | U: NNL u rows | x0bar]
    ldsd* SL = sm;
    ldsd* XD = SL + L * SLOT;
    ldsd* XL = XD + NNL * SXD;
    ldsd* U = XL + NB * NX;
    ldsd* X0B = U + NNL * NU;
    // first node of each level of this subtree (level L: the boundary)
    int gl[L + 1];
    static_for<0, L + 1>([&](auto lc) { gl[lc.value] = pl.sbase[s0 + lc.value] + o * cpow(C, lc.value); });
    // ---- 1. rows, then the backward tables
    Dma dm;
    if (!(kDiag && (pl.fault & 32))) {
        static_for<0, L>([&](auto lc) {
            constexpr int l = lc.value, cnt = cpow(C, l), off = (cnt - 1) / (C - 1);
            dm.rows(XD + off * SXD, SXD, (const double*)z + pl.X0 + (size_t)gl[l] * NX, NX, cnt, pl.zpage);
            dm.range(U + off * NU, (const double*)z + pl.U0 + (size_t)gl[l] * NU, cnt * NU);
        });
        if (deepest) dm.range(XL, (const double*)z + pl.X0 + (size_t)gl[L] * NX, NB * NX);
    }
    if (top) dm.range(X0B, pl.x0, NX);
    if (!(kDiag && (pl.fault & 4)))
        static_for<0, L>([&](auto ic) {
            constexpr int l = L - 1 - ic.value;
            TB::issue(SL + l * SLOT, pl.bimg + (size_t)(s0 + l) * TBN);
        });
    // ---- 2. the child subtrees' q rows
    if (!deepest) {
        const DrTier& ct = pl.t[k + 1];
        if (!poll_gran(pl.gq + (size_t)(ct.w0 + o * NB) * G, NB * G, tag, (ldsu*)XL, pl.timeout, pl.sync, s_ok)) {
            dma_wait();
            return;
        }
    }
    dma_wait();
    lds_sync();
    stamp(pl, stp);
    // ---- 3. backward sweep; each used slot is refilled with a forward table (table f in slot
    // L - 1 - f)
    static_for<0, L>([&](auto ic) {
        constexpr int i = ic.value, l = L - 1 - i, cnt = cpow(C, l), off = (cnt - 1) / (C - 1);
        if (i > 0) {
            lds_sync();
            stamp(pl, stp);
            if (top && !(kDiag && (pl.fault & 4))) TF::issue(SL + (l + 1) * SLOT, pl.fimg + (size_t)(s0 + i - 1) * TFN);
        }
        if (work && !(kDiag && (pl.fault & 16))) {
            const bool last = l == L - 1;
            back_level<NX, NU, C, BS, UMAX, cnt>(SL + l * SLOT, XD + off * SXD, last ? XL : XD + (off + cnt) * SXD,
                                           last ? NX : SXD, U + off * NU, (deepest && last) ? -1.0 : 1.0);
        }
    });
    lds_sync();
    stamp(pl, stp);
    wg_stamp(pl, 1);
    // ---- 4./5. the root's q row up, its x row down (below the top the forward tables load
    // during that wait; the top issued them as its backward sweep freed the slots)
    if (top && !(kDiag && (pl.fault & 4))) TF::issue(SL, pl.fimg + (size_t)(s0 + L - 1) * TFN);
    if (!top) {
        if (!((pl.fault & 1) && deepest && o == 0)) publish(pl.gq + (size_t)(tt.w0 + o) * G, G, tag, (const ldsu*)XD);
        if (!(kDiag && (pl.fault & 4)))
            static_for<0, L>([&](auto fc) {
                constexpr int f = fc.value;
                TF::issue(SL + (L - 1 - f) * SLOT, pl.fimg + (size_t)(s0 + f) * TFN);
            });
        if (!poll_gran(pl.gx + (size_t)(tt.w0 + o) * G, G, tag, (ldsu*)XD, pl.timeout, pl.sync, s_ok)) {
            dma_wait();
            return;
        }
        stamp(pl, stp);
    } else if (tid < NX) {
        XD[tid] = X0B[tid];  // x_0 = x0bar (cache.py:282)
    }
    // ---- 6. forward sweep: level f waits for its table only (the younger ones stay in flight)
    static_for<0, L>([&](auto fc) {
        constexpr int f = fc.value, cnt = cpow(C, f), off = (cnt - 1) / (C - 1);
        wait_vm_c<(L - 1 - f) * TF::IPW>();
        lds_sync();
        stamp(pl, stp);
        if (work && !(kDiag && (pl.fault & 16))) {
            const bool last = f == L - 1;
            fwd_level<NX, NU, C, BS, UMAX, cnt>(SL + (L - 1 - f) * SLOT, XD + off * SXD, last ? XL : XD + (off + cnt) * SXD,
                                          last ? NX : SXD, U + off * NU);
        }
    });
    lds_sync();
    stamp(pl, stp);
    // ---- 7. the boundary x rows to the child subtrees, then x and u to the iterate
    if (!deepest) publish(pl.gx + (size_t)(pl.t[k + 1].w0 + o * NB) * G, NB * G, tag, (const ldsu*)XL);
    if (work && !(kDiag && (pl.fault & 8))) {
        static_for<0, L + 1>([&](auto lc) {
            constexpr int l = lc.value, cnt = cpow(C, l), off = (cnt - 1) / (C - 1);
            if (l == 0 && !top) return;  // the parent writes this subtree's root row
            glb2* dst = (glb2*)(z + pl.X0 + (size_t)gl[l] * NX);
            if constexpr (l < L) {
                for (int e = tid; e < cnt * (NX / 2); e += BS) {
                    const int r = e / (NX / 2), c = e - r * (NX / 2);
                    dst[e] = ld2(XD + (off + r) * SXD + 2 * c);
                }
            } else {
                for (int e = tid; e < NB * (NX / 2); e += BS) dst[e] = ld2(XL + 2 * e);
            }
        });
        static_for<0, L>([&](auto lc) {
            constexpr int l = lc.value, cnt = cpow(C, l), off = (cnt - 1) / (C - 1);
            glb2* dst = (glb2*)(z + pl.U0 + (size_t)gl[l] * NU);
            for (int e = tid; e < cnt * (NU / 2); e += BS) dst[e] = ld2(U + off * NU + 2 * e);
        });
    }
    if (top && tid == 0) st_u32(pl.sync, tag);  // every workgroup has read the epoch
}

// LMAX: the deepest tier body compiled in (a plan whose subtrees have at most LMAX levels runs
// the instantiation of its largest L: small plans keep the registers of small levels)
// (waves per SIMD: two workgroups per CU at LMAX <= 4, else one; the register budget is then
// 128 / 256 VGPRs and the scheduler keeps a level's LDS reads in flight together)
template <int NX, int NU, int C, int BS, int LMAX>
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(LMAX <= 4 ? 4 : 2, LMAX <= 4 ? 4 : 2)))
k_dr(DrPlan pl, Bufs bf, int zsel, const Ctl* ctl, ChkArg ck) {
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
    // the words this workgroup needs first, written by earlier launches: scalar loads, outside
    // the vmcnt queue the counted waits use
    const unsigned long long sw = sload_pair(pl.sync);
    const unsigned err = (unsigned)(sw >> 32);
    const unsigned tag = (unsigned)sw + 1u;
    const int done = ctl ? ctl->done : 0;
    stamp(pl, stp);
    wg_stamp(pl, 0);
    if (err) return;
    int k, o;
    role(pl, k, o);
    glbd* z = pick3(bf, zsel);
    ldsd* sm = (ldsd*)smem_;
    const int L = pl.t[k].L;
    static_for<1, LMAX + 1>([&](auto lc) {
        // plans of at most 4 levels per tier run two workgroups per CU (<= 128 VGPRs): one node
        // per group and pass
        if (L == lc.value)
            tier_body<NX, NU, C, BS, (LMAX <= 4 ? 1 : (C == 2 ? 4 : 2)), lc.value>(pl, k, o, z, tag, done == 0, stp, s_ok, sm);
    });
    stamp(pl, stp);
    stamp_flush(pl, stp, k, o);
    wg_stamp(pl, 2);
}

template <int NX, int NU, int C, int LMAX>
void launch_t(const DrPlan& pl, size_t lds, Bufs bf, int zsel, const Ctl* ctl, ChkArg ck, hipStream_t s) {
    const int grid = pl.nblk + (ck.on ? 1 : 0);
    auto kf = k_dr<NX, NU, C, 512, LMAX>;
    (void)hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kf<<<grid, 512, lds, s>>>(pl, bf, zsel, ctl, ck);
}
template <int NX, int NU, int C, int LMAX>
int occ_t(size_t lds) {
    int nb = 0;
    const void* kf = (const void*)k_dr<NX, NU, C, 512, LMAX>;
    (void)hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kf, 512, lds) != hipSuccess) return 0;
    return nb;
}
// the compiled LMAX of a plan: 4 (at most 4 levels per tier) or kDrMaxL
template <int NX, int NU, int C, class F>
auto by_lmax(int lmax, F&& f) {
    if (lmax <= 4) return f(std::integral_constant<int, 4>{});
    return f(std::integral_constant<int, kDrMaxL>{});
}

}  // namespace

bool dr_supported(int nx, int nu, int C) { return nx == 20 && nu == 8 && (C == 2 || C == 3 || C == 4); }

size_t dr_lds(int nx, int nu, int C, int L) {
    long nnl = 0, p = 1;
    for (int l = 0; l < L; ++l, p *= C) nnl += p;
    return 8 * ((size_t)L * dr_slot_n(nx, nu, C) + (size_t)nnl * (nx + nu) + (size_t)p * nx + (size_t)nnl * nu + nx);
}

int dr_occupancy(int nx, int nu, int C, int lmax, size_t lds) {
    if (nx == 20 && nu == 8) {
        if (C == 2) return by_lmax<20, 8, 2>(lmax, [&](auto m) { return occ_t<20, 8, 2, m.value>(lds); });
        if (C == 3) return by_lmax<20, 8, 3>(lmax, [&](auto m) { return occ_t<20, 8, 3, m.value>(lds); });
        if (C == 4) return by_lmax<20, 8, 4>(lmax, [&](auto m) { return occ_t<20, 8, 4, m.value>(lds); });
    }
    return 0;
}

void dr_launch(const DrPlan& pl, int nx, int nu, size_t lds, Bufs bf, int zsel, const Ctl* ctl, ChkArg ck,
               hipStream_t s) {
    int lmax = 0;
    for (int k = 0; k < pl.T; ++k) lmax = pl.t[k].L > lmax ? pl.t[k].L : lmax;
    if (nx == 20 && nu == 8) {
        if (pl.C == 2) by_lmax<20, 8, 2>(lmax, [&](auto m) { launch_t<20, 8, 2, m.value>(pl, lds, bf, zsel, ctl, ck, s); return 0; });
        else if (pl.C == 3) by_lmax<20, 8, 3>(lmax, [&](auto m) { launch_t<20, 8, 3, m.value>(pl, lds, bf, zsel, ctl, ck, s); return 0; });
        else by_lmax<20, 8, 4>(lmax, [&](auto m) { launch_t<20, 8, 4, m.value>(pl, lds, bf, zsel, ctl, ck, s); return 0; });
    }
}
const char* dr_name(int nx, int nu) { return nx == 20 && nu == 8 ? "k_dr<20, 8>" : "k_dr"; }

}  // namespace raocp
