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
#define RAOCP_AMAX_BITS
// sum_h by shuffles here: the row-swap form (raocp_tile.h) spills 4 VGPRs in k_drc and measured
// 0.25 us per iteration slower (profiles/r06/drc_variants.log)
#define RAOCP_SUMH_SHFL
#include "raocp_cpops.h"

namespace raocp {
namespace {

typedef double d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) d2v lds2;
typedef __attribute__((address_space(1))) d2v glb2;
typedef __attribute__((address_space(3))) unsigned ldsu;

__device__ __forceinline__ d2v ld2(const ldsd* p) { return *(const lds2*)p; }

// LDS barrier that does not wait for this wave's global memory operations
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


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
// every workgroup (diagnostics, tools/dr_skew.py): slots 1024 + 4 b + {0 start, 1 backward
// sweep done, 2 end, 3 forward sweep done (k_drc: the CP step's start)}; the host checks the
// buffer holds them (raocp_debug_dyn_stamps)
__device__ __forceinline__ void wg_stamp(const DrPlan& pl, int q) {
    if (kDiag && pl.stamps && threadIdx.x == 0)
        pl.stamps[1024 + 4 * blockIdx.x + q] = __builtin_amdgcn_s_memrealtime();
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

// ================================ k_drc: the fused CP step ================================
// A workgroup of the sweep owns the CP families whose parent is one of its subtree's nonleaf
// nodes (solver.py:27-95 with cache.py:248-393): the family of node i reads the projection only
// at i (x+_i, u+_i: eta3 / eta4 of a child are sqrtQ / sqrtR of the PARENT's rows,
// operators.py:19-53), and a leaf's rows only its own x+. So right behind its forward sweep, with
// x+ and u+ still in LDS, a workgroup runs the CP iteration of its 15 families (one 16-lane MFMA
// tile, lane lo = subtree-local BFS index, lo = 15 dead) and, in the deepest tier, of its 16
// leaves (lane lo = leaf), with k_cp6's entry arithmetic (raocp_cp5.hip) split over the waves:
//   wave 0, 1    child slot k: the parent's L products, the child block SOC (eta3..eta6), the
//                slot's (eta+, d - eta+, xi2) rows to LDS, tau_j; a nonleaf child's s_j from its
//                eta2 (recomputed, k_cp6's arithmetic)
//   wave 2       phase 1: eta1, eta2 of the parent, y_i of the half step, s_0
//   wave 3       (deepest) the leaf tile: eta11..eta14 with the leaf SOC and box, x_l of the half
//                step by the eta+ stream, s_l; the (d - eta+) and xi2 rows to LDS
//   -- barrier --
//   wave 0       L^T of the eta+ stream (Gamma' eta7 + slot sums in slot order): x_i, u_i
//   wave 1       the (d - eta+) and xi2 streams and the residual terms of x_i, u_i
//   wave 2       the AVaR kernel projection of the family (cache.py:290-317)
//   wave 4       (deepest) the leaves' (d - eta+) and xi2 streams and their residual terms
// Every operand that does not depend on the projection is in LDS before the forward sweep ends:
// gathered by 4-B LDS-DMA (Cpa) while the workgroup waits for its root's x row (the top: behind
// its forward sweep, off the critical path); the MFMA weight fragments and box tables land in the
// table slots the forward levels free (slot 3 after level 0, slot 2 after level 1).
//
// Global index of the subtree-local node lc (C = 2): (R0 << level(lc)) + lc, R0 the root.
__device__ __forceinline__ int lev2(int lc) { return 31 - __builtin_clz((unsigned)lc + 1u); }
__device__ __forceinline__ int gnode(int R0, int lc) { return (R0 << lev2(lc)) + lc; }

// the CP operand region (doubles): rows of the 15 families lo (row 15 zero), their 30 children
// c = 2 lo + 1 + k (row c - 1; rows 30, 31 zero), the deepest tier's 16 leaves q. The child
// rows are padded (strides D3S, D4S, SCS, zeros in the padding) so that the 16 lanes lo, whose
// child rows lie two rows apart, read distinct LDS banks: unpadded, the child scalars' stride
// of 256 B put all 16 on one bank and eta4's on two
struct Cpa {
    static constexpr int D3S = 22, D4S = 10, SCS = 18;
    static constexpr int PX = 0;      // [16][20] x of p (the previous z+) at the parents
    static constexpr int PU = 320;    // [16][8]  u of p
    static constexpr int D3 = 448;    // [32][D3S] eta3 of the children
    static constexpr int D4 = 1152;   // [32][D4S] eta4
    static constexpr int SC = 1472;   // [32][SCS] eta5, eta6, tau of z+ / p; a nonleaf child's s of z+ / p,
                                      //           eta2, cond of its children, y of z+ / p (entries 0, 1, 2C)
    static constexpr int PS = 2048;   // [16][24] y of z+ / p (5 + 5), eta1 (5), s of z+ / p, eta2,
                                      //          cond of the children (2), AVaR alpha
    static constexpr int D7 = 2432;   // [16][28] eta7 (boxed nonleaf nodes)
    static constexpr int LP = 2880;   // [16][20] x of p at the leaves (deepest tier)
    static constexpr int D11 = 3200;  // [16][20] eta11
    static constexpr int D14 = 3520;  // [16][20] eta14 (boxed leaves)
    static constexpr int LS = 3840;   // [16][4]  eta12, eta13, s of z+ / p
    static constexpr int N = 3904;
    // after barrier A2 (k_drc cp_phase): the families' box seeds of the (d - eta+) and xi2 streams
    // over the dead eta3 / eta4 rows ([16][28] each), the xi2 stream's L^T over the child scalars
    static constexpr int SDW = D3, SDC = D3 + 448;
    static_assert(SDC + 448 <= SC && 448 <= SCS * 32, "reuse of the dead child rows");
};
static_assert(Cpa::N == kDrcCpa, "CP operand region");
// scratch in the table slots once the forward sweep is done (doubles from the first slot; slot
// s at s * 1344): the weight image in slots 2 and 3 as the forward levels free them; slots 0-1
// first hold the L products that waves exchange (qa, qb, lb, ua, ub), then (after barrier A2)
// the child slots' stream rows [slot k][stream q][x 320 | u 128]; the leaves' (d - eta+) and xi2
// rows, the kernel-projection scratch and the residual maxima in the slots' tails
struct Cps {
    static constexpr int WA = kDrcWa;  // doubles of the first image part ([sqrtQ | sqrtR])
    static constexpr int WB = kDrcWb;  // the second ([sqrtPf | lo_nl | hi_nl | lo_l | hi_l])
    static constexpr int SLOT = 1344;
    static constexpr int QA = 0, QB = 512, LB = 1024, UA = 1536, UB = 1792;  // products (row-layout v4 x 64 lanes)
    static constexpr int SB = 0, SX = 320, SS = 448;                          // stream rows (compacted)
    static constexpr int WP = 2 * SLOT, BX = 2 * SLOT + 640, LEW = 2 * SLOT + 736, KPS = 2 * SLOT + 1056;
    // MX2: the deepest leaf wave's lane maxima for wave 0's residual row ([m2 64 | m5 64 | m0, m1,
    // m3, m4 of lanes 0..15])
    static constexpr int WQ = 3 * SLOT, WR = 3 * SLOT + 640, LEC = 3 * SLOT + 768, MX2 = 3 * SLOT + 1088;
};
static_assert(Cps::UB + 256 <= 2 * Cps::SLOT && 6 * Cps::SS <= 2 * Cps::SLOT, "slots 0-1");
static_assert(Cps::KPS + 272 <= 3 * Cps::SLOT && Cps::MX2 + 192 <= 4 * Cps::SLOT, "slot tails");

// The CP operands through registers: every lane loads up to four pairs of the region (pair f =
// doubles 2 f, 2 f + 1 of Cpa, f = tid + 512 s) with 8-byte loads at valid addresses (zeros from
// the zero page where a row is dead), before the wait they hide behind; once they have landed,
// the pairs go to LDS with 16-B stores (cpa_commit). 16 VGPRs across the wait, 8 load
// instructions per lane, no per-dword DMA.
constexpr int kCpaPairs = Cpa::N / 2;
constexpr int kCpaSlots = (kCpaPairs + 511) / 512;
struct CpaStage {
    d2v v[kCpaSlots];
};
template <int NX, int NU, int BXN>
__device__ __forceinline__ void cpa_issue(const DrcArg& a, const DrPlan& pl, const Bufs& bf, int R0, bool deepest,
                                          CpaStage& st) {
    const double* pz = bf.z0;  // p
    const double* zp = bf.z1;  // z+ (y, tau, s: not written by this launch)
    const double* dd = bf.e0;  // eta
    const double* zpg = pl.zpage;
    const int l0 = 16 * R0 + 15;  // the first leaf of the subtree (deepest tier)
    _Pragma("unroll") for (int sl = 0; sl < kCpaSlots; ++sl) {
        const int f = threadIdx.x + 512 * sl, e = 2 * f;
        const double* s0 = zpg;
        const double* s1 = zpg;
        bool pair = true;  // the two doubles are adjacent in global memory (s1 = s0 + 1)
        if (e < Cpa::PU) {
            const int r = e / NX;
            if (r < 15) s0 = pz + pl.X0 + (size_t)gnode(R0, r) * NX + (e - r * NX);
        } else if (e < Cpa::D3) {
            const int q = e - Cpa::PU, r = q / NU;
            if (r < 15) s0 = pz + pl.U0 + (size_t)gnode(R0, r) * NU + (q - r * NU);
        } else if (e < Cpa::D4) {
            const int q = e - Cpa::D3, r = q / Cpa::D3S, c = q - r * Cpa::D3S;
            if (r < 30 && c < NX) s0 = dd + a.E3 + 1 + (size_t)(gnode(R0, r + 1) - 1) * NX + c;
        } else if (e < Cpa::SC) {
            const int q = e - Cpa::D4, r = q / Cpa::D4S, c = q - r * Cpa::D4S;
            if (r < 30 && c < NU) s0 = dd + a.E4 + 1 + (size_t)(gnode(R0, r + 1) - 1) * NU + c;
        } else if (e < Cpa::PS) {
            // child scalars (Cpa::SC): eta5, eta6 | tau z+, p | a nonleaf child's s z+, p | eta2,
            // cond k=0 | cond k=1, y0 z+ | y1 z+, y4 z+ | y0 p, y1 p | y4 p, -
            pair = false;
            const int q = e - Cpa::SC, r = q / Cpa::SCS, c = q - r * Cpa::SCS;
            if (r < 30 && c < 16) {
                const int j = gnode(R0, r + 1);
                const bool nl = !(deepest && r + 1 >= 15);
                switch (c) {
                    case 0: s0 = dd + a.E5 + j; s1 = dd + a.E6 + j; break;
                    case 2: s0 = zp + a.T0 + j; s1 = pz + a.T0 + j; break;
                    case 4: if (nl) { s0 = zp + a.S0 + j; s1 = pz + a.S0 + j; } break;
                    case 6: if (nl) { s0 = dd + a.E2 + j; s1 = a.cond + 1 + 2 * j; } break;
                    case 8: if (nl) { s0 = a.cond + 2 + 2 * j; s1 = zp + a.Y0 + 5 * j; } break;
                    case 10: if (nl) { s0 = zp + a.Y0 + 5 * j + 1; s1 = zp + a.Y0 + 5 * j + 4; } break;
                    case 12: if (nl) { s0 = pz + a.Y0 + 5 * j; s1 = pz + a.Y0 + 5 * j + 1; } break;
                    default: if (nl) s0 = pz + a.Y0 + 5 * j + 4; break;
                }
            }
        } else if (e < Cpa::D7) {
            // parent scalars (Cpa::PS): y z+ (5), y p (5), eta1 (5), s z+, s p, eta2, cond (2), alpha, -
            pair = false;
            const int q = e - Cpa::PS, r = q / 24, c = q - r * 24;
            if (r < 15) {
                const int g = gnode(R0, r);
                auto src = [&](int cc) -> const double* {
                    if (cc < 5) return zp + a.Y0 + 5 * g + cc;
                    if (cc < 10) return pz + a.Y0 + 5 * g + (cc - 5);
                    if (cc < 15) return dd + a.E1 + 5 * g + (cc - 10);
                    switch (cc) {
                        case 15: return zp + a.S0 + g;
                        case 16: return pz + a.S0 + g;
                        case 17: return dd + a.E2 + g;
                        case 18: return a.cond + 1 + 2 * g;
                        case 19: return a.cond + 2 + 2 * g;
                        case 20: return a.alpha_r + g;
                        default: return zpg;
                    }
                };
                s0 = src(c);
                s1 = src(c + 1);
            }
        } else if (e < Cpa::LP) {
            const int q = e - Cpa::D7, r = q / (NX + NU);
            if (BXN == 1 && r < 15) s0 = dd + a.E7 + (size_t)gnode(R0, r) * (NX + NU) + (q - r * (NX + NU));
        } else if (e < Cpa::D11) {
            if (deepest) s0 = pz + pl.X0 + (size_t)l0 * NX + (e - Cpa::LP);
        } else if (e < Cpa::D14) {
            if (deepest) s0 = dd + a.E11 + a.m + (size_t)(l0 - a.m) * NX + (e - Cpa::D11);
        } else if (e < Cpa::LS) {
            if (deepest && a.box == 1) s0 = dd + a.E14 + a.m + (size_t)(l0 - a.m) * NX + (e - Cpa::D14);
        } else if (e < Cpa::N) {
            pair = false;
            const int q = e - Cpa::LS, ll = l0 + (q >> 2);
            if (deepest) {
                if ((q & 3) == 0) {
                    s0 = dd + a.E12 + ll;
                    s1 = dd + a.E13 + ll;
                } else {
                    s0 = zp + a.S0 + ll;
                    s1 = pz + a.S0 + ll;
                }
            }
        }
        if (pair) s1 = s0 == zpg ? zpg : s0 + 1;
        st.v[sl] = d2v{*(const glbd*)s0, *(const glbd*)s1};
    }
}
__device__ __forceinline__ void cpa_commit(ldsd* A, const CpaStage& st) {
    _Pragma("unroll") for (int sl = 0; sl < kCpaSlots; ++sl) {
        const int f = threadIdx.x + 512 * sl;
        if (f < kCpaPairs) *(lds2*)(A + 2 * f) = st.v[sl];
    }
}

// a wave's maximum of non-negative doubles (NaN above +inf) by their bit patterns as unsigned
// integers: wave_nmax's DPP steps with one 64-bit compare and two selects per step; lane 63
// ends with it
__device__ __forceinline__ double bmax(double a, double b) {
    return (unsigned long long)__double_as_longlong(a) > (unsigned long long)__double_as_longlong(b) ? a : b;
}
// (the steps whose rows and banks are all written take no "old" operand: no copy per step)
template <int CTRL>
__device__ __forceinline__ double dpp_full(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// N maxima at once, step by step (independent chains interleaved: the DPP hazards of one value
// are filled with the others' work)
template <int N>
__device__ __forceinline__ void wave_bmax_n(double (&v)[N]) {
#ifdef RAOCP_BMAX_SEQ
    _Pragma("unroll") for (int q = 0; q < N; ++q) {
        v[q] = bmax(v[q], dpp_full<0xB1>(v[q]));
        v[q] = bmax(v[q], dpp_full<0x4E>(v[q]));
        v[q] = bmax(v[q], dpp_full<0x141>(v[q]));
        v[q] = bmax(v[q], dpp_full<0x140>(v[q]));
        v[q] = bmax(v[q], dpp_d<0x142, 0xA>(v[q]));
        v[q] = bmax(v[q], dpp_d<0x143, 0xC>(v[q]));
    }
    return;
#endif
    _Pragma("unroll") for (int q = 0; q < N; ++q) v[q] = bmax(v[q], dpp_full<0xB1>(v[q]));   // lane ^ 1
    _Pragma("unroll") for (int q = 0; q < N; ++q) v[q] = bmax(v[q], dpp_full<0x4E>(v[q]));   // lane ^ 2
    _Pragma("unroll") for (int q = 0; q < N; ++q) v[q] = bmax(v[q], dpp_full<0x141>(v[q]));  // row half-mirror
    _Pragma("unroll") for (int q = 0; q < N; ++q) v[q] = bmax(v[q], dpp_full<0x140>(v[q]));  // row mirror
    _Pragma("unroll") for (int q = 0; q < N; ++q) v[q] = bmax(v[q], dpp_d<0x142, 0xA>(v[q]));  // row_bcast15
    _Pragma("unroll") for (int q = 0; q < N; ++q) v[q] = bmax(v[q], dpp_d<0x143, 0xC>(v[q]));  // row_bcast31
}
__device__ __forceinline__ double wave_bmax(double v) {
    double a[1] = {v};
    wave_bmax_n<1>(a);
    return a[0];
}

// an R-row node vector from an LDS row in the tile's row layout (raocp_tile.h ld_rows), zero
// when !live (row must be a valid LDS row either way)
template <int R>
__device__ __forceinline__ void ld_lr(const ldsd* row, bool live, double (&a)[(R + 15) / 16][4]) {
    constexpr int KC = R / 4;
    const ldsd* b = row + KC * ((threadIdx.x & 63) >> 4);
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
        double w = 0.0;
        if (tok<R>(rt, e)) w = b[4 * rt + e];
        a[rt][e] = live ? w : 0.0;
    }
}

// slot (rt, e) of a lane's R-row vector: its row index KC h + 4 rt + e (tok<R>(rt, e)), and its
// place in a compacted LDS image (lds_putc: lane's KC values at base + lane KC)
template <int R>
__device__ __forceinline__ int row_of(int rt, int e) {
    return (R / 4) * ((threadIdx.x & 63) >> 4) + 4 * rt + e;
}
template <int R>
__device__ __forceinline__ int cpos(int rt, int e) {
    return (threadIdx.x & 63) * (R / 4) + 4 * rt + e;
}

// a store of the CP step (stv false: timing probes of diagnostic builds skip them)
__device__ __forceinline__ void gput(bool stv, glbp<double> b, unsigned o, double v) {
    if (stv) *elw(b, o) = v;
}

// wo(t0, nt): the sweep's write-out of the projected x / u rows, run by waves 3 and 4 in their
// wait between barriers A2 and B
template <int NX, int NU, int BXN, int BXL, class WO>
__device__ __forceinline__ void cp_phase(const DrcArg& a, const Bufs& bf, double alpha_in, int X0, int U0, int R0,
                                         bool deepest, const ldsd* XD, const ldsd* XL, const ldsd* U, ldsd* A,
                                         ldsd* SL, unsigned long long* dstamps, int nblk, const WO& wo, bool stv = true) {
    typedef double T;
    typedef MF<T>::v4 v4;
    constexpr int C = 2, RX = (NX + 15) / 16, RU = (NU + 15) / 16, G = 2 * C + 1, NQ = (G + 3) / 4;
    constexpr int SXD = NX + NU, SS = Cps::SS, SX = Cps::SX;
    static_assert(NX == 20 && NU == 8, "the scratch layout (Cps) is sized for nx = 20, nu = 8");
    typedef WL<T, NX, NX> WQ;
    typedef WL<T, NU, NU> WR;
    typedef __attribute__((address_space(3))) KpScratch<T> lkps;
    // (the wave index as a lane value: with it in a scalar register the role branches become
    // scalar ones and the allocator overlaps the roles' live ranges, 91 VGPRs spilled)
    const int tid = threadIdx.x, lane = tid & 63, lo = lane & 15, h = lane >> 4, wv = tid >> 6;
    // diagnostics: per-wave stamps of the first (deepest) and the last (top) workgroup at
    // 3072 + {0, 64} + 8 wave + {0 start, 1 first role done, 2 second role done, 3 third role
    // done, 5 last role done, 4 end; slot waves: 6 after barrier A2, 7 their block's SOC}
    auto dstamp = [&](int q) {
        if (kDiag && dstamps && lane == 0 && (blockIdx.x == 0 || (int)blockIdx.x == nblk - 1))
            dstamps[3072 + ((int)blockIdx.x == 0 ? 0 : 64) + 8 * wv + q] = __builtin_amdgcn_s_memrealtime();
    };
    dstamp(0);
    const WQ wq{SL + Cps::WQ};
    const WR wr{SL + Cps::WR};
    const WQ wp{SL + Cps::WP};
    const ldsd* BX = SL + Cps::BX;  // [lo_nl | hi_nl | lo_l | hi_l]
    lkps& ks = *(lkps*)(SL + Cps::KPS);
    glbp<T> out = (glbp<T>)bf.z2;  // next half step
    glbp<T> eo = (glbp<T>)bf.e1;   // eta+
    const int m = a.m;
    Resid<T> rs;
    rs.alpha = alpha_in;
    rs.ra = T(1) / rs.alpha;
    const T alpha = rs.alpha, ra = rs.ra;
    bool nanf = false;  // a NaN reached a box (Rectangle._constrain raises)
    // the wave's residual row (its six maxima by DPP; lanes 58..63 hold all six and store one
    // each), written by every wave once its terms are final: in the idle time of its role where
    // it has one, so that only waves 1 and 4 reduce (one maximum) behind the last barrier
    // (lane 63 stores the row as three 16-B stores: a per-lane pick of one of six values became
    // an indexed private array in scratch, whose load waited for every store of the wave)
    auto put_row = [&](const double (&mm)[6]) {
        if (lane == 63) {
            glb2* row = (glb2*)(a.part + ((size_t)blockIdx.x * 8 + wv) * 6);
            row[0] = d2v{mm[0], mm[1]};
            row[1] = d2v{mm[2], mm[3]};
            row[2] = d2v{mm[4], mm[5]};
        }
    };
    auto emit_row = [&]() {
        double mm[6] = {rs.m0.get(), rs.m1.get(), rs.m2.get(), rs.m3.get(), rs.m4.get(), rs.m5.get()};
        wave_bmax_n<6>(mm);
        put_row(mm);
    };
    // rows of waves whose terms feed only some maxima: the others stay zero (wave 6 accounts s_j
    // only: xi0, xi1, delta0, delta1; wave 7 the box entries only: xi2, delta2)
    auto emit_acc_row = [&]() {
        double m4[4] = {rs.m0.get(), rs.m1.get(), rs.m3.get(), rs.m4.get()};
        wave_bmax_n<4>(m4);
        const double mm[6] = {m4[0], m4[1], 0, m4[2], m4[3], 0};
        put_row(mm);
    };
    auto emit_fin_row = [&]() {
        double m2[2] = {rs.m2.get(), rs.m5.get()};
        wave_bmax_n<2>(m2);
        const double mm[6] = {0, 0, m2[0], 0, 0, m2[1]};
        put_row(mm);
    };
    auto zero_row = [&]() {
        const double mm[6] = {0, 0, 0, 0, 0, 0};
        put_row(mm);
    };
    const bool live = lo < 15;
    const int lq = live ? lo : 0;
    const int i = gnode(R0, lq), yo = G * i;  // this lane's parent (global)
    const int l = 16 * R0 + 15 + lo;           // this lane's leaf (deepest tier)
    // ============ Ia: the L products, one MFMA chain per wave (waves w, w + 4 share a SIMD)
    v4 pk[RX];  // wave 0: qa = sqrtQ (2 x+ - p); wave 1: qb = sqrtQ (x+ - p); wave 2: la; wave 3: lb
    if (wv < 2 || (wv < 4 && deepest)) {
        T b[RX][4];
        {
            T z[RX][4], pp[RX][4];
            if (wv < 2) {
                ld_lr<NX>(XD + lq * SXD, live, z);
                ld_lr<NX>(A + Cpa::PX + lq * NX, live, pp);
            } else {
                ld_lr<NX>(XL + lo * NX, true, z);
                ld_lr<NX>(A + Cpa::LP + lo * NX, true, pp);
            }
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                b[rt][e] = (wv & 1) ? z[rt][e] - pp[rt][e] : T(2) * z[rt][e] - pp[rt][e];
        }
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) pk[rt] = v4{0, 0, 0, 0};
        if (wv < 2) mmt(wq.fresh(), b, pk);
        else mmt(wp.fresh(), b, pk);
        if (wv != 2) {  // qa, qb, lb to LDS (la stays in wave 2's registers)
            ldsd* dst = SL + (wv == 0 ? Cps::QA : (wv == 1 ? Cps::QB : Cps::LB));
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                dst[(rt * 64 + lane) * 4 + e] = pk[rt][e];
        }
    } else if (wv == 4) {
        T c1[RU][4], c2[RU][4];
        {
            T uz[RU][4], up[RU][4];
            ld_lr<NU>(U + lq * NU, live, uz);
            ld_lr<NU>(A + Cpa::PU + lq * NU, live, up);
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                c1[rt][e] = T(2) * uz[rt][e] - up[rt][e];
                c2[rt][e] = uz[rt][e] - up[rt][e];
            }
        }
        v4 ua[RU], ub[RU];
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) ua[rt] = ub[rt] = v4{0, 0, 0, 0};
        mmt(wr.fresh(), c1, ua);
        mmt(wr.fresh(), c2, ub);
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            SL[Cps::UA + (rt * 64 + lane) * 4 + e] = ua[rt][e];
            SL[Cps::UB + (rt * 64 + lane) * 4 + e] = ub[rt][e];
        }
    } else if (wv == 5) {
        // ================= phase 1: the parent's eta2, eta1 (AVaR cone), y_i, s_0
        const ldsd* ps = A + Cpa::PS + lq * 24;
        T cp[C], zyk[C], pyk[C];
        _Pragma("unroll") for (int q = 0; q < C; ++q) {
            cp[q] = live ? ps[18 + q] : T(0);
            zyk[q] = live ? ps[q] : T(0);
            pyk[q] = live ? ps[5 + q] : T(0);
        }
        const T zyc = live ? ps[2 * C] : T(0), pyc = live ? ps[5 + 2 * C] : T(0);
        const T zs = live ? ps[15] : T(0), pps = live ? ps[16] : T(0), d2 = live ? ps[17] : T(0);
        T qz[NQ], qp[NQ], qd[NQ];
        _Pragma("unroll") for (int t = 0; t < NQ; ++t) {
            const int q = h + 4 * t;
            const bool ok = live && q < G;
            const int qq = q < G ? q : 0;
            qz[t] = ok ? ps[qq] : T(0);
            qp[t] = ok ? ps[5 + qq] : T(0);
            qd[t] = ok ? ps[10 + qq] : T(0);
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
            const T av = (T(2) * zs - pps) - bya, bb = (zs - pps) - byb;
            const T v = (d2 + alpha * av) * ra;
            T x2;
            rs.fin(d2, v, fmax(v, T(0)), bb, e2A, x2);
            e2C = x2;
            if (live && h == 0) gput(stv, eo, a.E2 + i, e2A);
        }
        const T e2W = d2 - e2A;
        if (live && i == 0 && h == 0) {
            // root s_0: L^T -> eta2_0, then the relaxation prox s_0 -= alpha (cache.py:253-257)
            gput(stv, out, a.S0, (zs - alpha * e2A) - alpha);
            rs.account(pps, zs, e2W, e2C);
        }
        _Pragma("unroll") for (int t = 0; t < NQ; ++t) {
            const int q = h + 4 * t;
            if (!live || q >= G) break;
            const T zy = qz[t], py = qp[t], dv = qd[t];
            const T v = (dv + alpha * (T(2) * zy - py)) * ra;
            T ep, x2;
            rs.fin(dv, v, q < 2 * C ? fmax(v, T(0)) : v, zy - py, ep, x2);
            gput(stv, eo, a.E1 + yo + q, ep);
            T bq = T(1);
            if (q < C) {
                _Pragma("unroll") for (int kk = 0; kk < C; ++kk) if (kk == q) bq = cp[kk];
            } else if (q < 2 * C) {
                bq = T(0);
            }
            ks.y[lo][q] = zy - alpha * (ep - bq * e2A);
            rs.account(py, zy, (dv - ep) - bq * e2W, x2 - bq * e2C);
        }
    } else if (wv == 6) {
        // ================= s_j of the nonleaf children (k = h < C): its eta2 recomputed (its own
        // family's phase 1, k_cp6's arithmetic)
        const int k = h, cl = 2 * lq + 1 + (h & 1);
        if (live && h < C && !(deepest && cl >= 15)) {
            const ldsd* sc = A + Cpa::SC + (cl - 1) * Cpa::SCS;
            const T csz = sc[4], csp = sc[5], cdj = sc[6];
            const T ccp[C] = {sc[7], sc[8]}, czy[C + 1] = {sc[9], sc[10], sc[11]}, cpy[C + 1] = {sc[12], sc[13], sc[14]};
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
    dstamp(1);
    lds_sync();  // A: the products in LDS
    // ============ Ib: the SOC of each child block (wave k: slot k) and of the leaves (wave 2);
    // every operand read into registers before barrier A2, after which the stream rows overwrite
    // the products' LDS
    if (wv < 2) {
        const int k = wv, cl = 2 * lq + 1 + k, j = gnode(R0, cl);
        v4 qa[RX], qb[RX], ua[RU], ub[RU];
        {
            const ldsd* o = SL + (k == 0 ? Cps::QB : Cps::QA);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) {
                v4 w;
                _Pragma("unroll") for (int e = 0; e < 4; ++e) w[e] = o[(rt * 64 + lane) * 4 + e];
                if (k == 0) {
                    qa[rt] = pk[rt];
                    qb[rt] = w;
                } else {
                    qa[rt] = w;
                    qb[rt] = pk[rt];
                }
            }
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                ua[rt][e] = SL[Cps::UA + (rt * 64 + lane) * 4 + e];
                ub[rt][e] = SL[Cps::UB + (rt * 64 + lane) * 4 + e];
            }
        }
        T d3[RX][4], d4[RU][4];
        ld_lr<NX>(A + Cpa::D3 + (cl - 1) * Cpa::D3S, live, d3);
        ld_lr<NU>(A + Cpa::D4 + (cl - 1) * Cpa::D4S, live, d4);
        const ldsd* sc = A + Cpa::SC + (cl - 1) * Cpa::SCS;
        const T d5 = live ? sc[0] : T(0), d6 = live ? sc[1] : T(0), tz = live ? sc[2] : T(0), tp = live ? sc[3] : T(0);
        lds_sync();  // A2
        dstamp(6);
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
        dstamp(7);
        // each entry's (eta+, d - eta+, xi2) straight to the slot's stream rows and eta+ to the dual
        ldsd* sk = SL + Cps::SB + k * 3 * SS;
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            if (!tok<NX>(rt, e)) continue;
            T ep, x2;
            rs.fin(d3[rt][e], v3[rt][e], so.first(v3[rt][e]), qb[rt][e], ep, x2);
            const int q = cpos<NX>(rt, e);
            sk[q] = ep;
            sk[SS + q] = d3[rt][e] - ep;
            sk[2 * SS + q] = x2;
            if (live) gput(stv, eo, a.E3 + 1 + (j - 1) * NX + row_of<NX>(rt, e), ep);
        }
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            if (!tok<NU>(rt, e)) continue;
            T ep, x2;
            rs.fin(d4[rt][e], v4_[rt][e], so.first(v4_[rt][e]), ub[rt][e], ep, x2);
            const int q = SX + cpos<NU>(rt, e);
            sk[q] = ep;
            sk[SS + q] = d4[rt][e] - ep;
            sk[2 * SS + q] = x2;
            if (live) gput(stv, eo, a.E4 + 1 + (j - 1) * NU + row_of<NU>(rt, e), ep);
        }
        T ep5, x25, ep6, x26;
        rs.fin(d5, v5, so.first(v5), b5, ep5, x25);
        rs.fin(d6, v6, so.last(v6), b5, ep6, x26);
        if (live && h == 0) {
            gput(stv, eo, a.E5 + j, ep5);
            ks.tau[lo][k] = tz - alpha * (T(0.5) * (ep5 + ep6));
            rs.account(tp, tz, T(0.5) * ((d5 - ep5) + (d6 - ep6)), T(0.5) * (x25 + x26));
        }
        if (live && h == 1) gput(stv, eo, a.E6 + j, ep6);
    } else if (wv == 2 && deepest) {
        // ================= the leaf tile (lane lo = leaf lo of the subtree; k_cp6's leaf waves)
        v4 lb[RX];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
            lb[rt][e] = SL[Cps::LB + (rt * 64 + lane) * 4 + e];
        T d11[RX][4];
        ld_lr<NX>(A + Cpa::D11 + lo * NX, true, d11);
        const ldsd* ls = A + Cpa::LS + lo * 4;
        const T d12 = ls[0], d13 = ls[1], sz = ls[2], sp = ls[3];
        lds_sync();  // A2
        T v11[RX][4];
        T ss = T(0);
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            v11[rt][e] = (d11[rt][e] + alpha * pk[rt][e]) * ra;
            if (tok<NX>(rt, e)) ss += v11[rt][e] * v11[rt][e];
        }
        ss = sum_h(ss);
        const T a5 = T(0.5) * (T(2) * sz - sp), b5 = T(0.5) * (sz - sp);
        const T v12 = (d12 + alpha * a5) * ra + T(-0.5);
        const T v13 = (d13 + alpha * a5) * ra + T(0.5);
        ss += v12 * v12;
        const Soc<T> so(sqrt(ss), v13);
        T ep12, x212, ep13, x213;
        rs.fin(d12, v12, so.first(v12), b5, ep12, x212);
        rs.fin(d13, v13, so.last(v13), b5, ep13, x213);
        if (h == 0) {
            ks.s[7 + (lo >> 1)][lo & 1] = sz - alpha * (T(0.5) * (ep12 + ep13));
            rs.account(sp, sz, T(0.5) * ((d12 - ep12) + (d13 - ep13)), T(0.5) * (x212 + x213));
            gput(stv, eo, a.E12 + l, ep12);
        }
        if (h == 1) gput(stv, eo, a.E13 + l, ep13);
        T eA[RX][4];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            T ep = T(0), x2 = T(0);
            if (tok<NX>(rt, e)) {
                rs.fin(d11[rt][e], v11[rt][e], so.first(v11[rt][e]), lb[rt][e], ep, x2);
                const int q = cpos<NX>(rt, e);
                SL[Cps::LEW + q] = d11[rt][e] - ep;
                SL[Cps::LEC + q] = x2;
                gput(stv, eo, a.E11 + m + (l - m) * NX + row_of<NX>(rt, e), ep);
            }
            eA[rt][e] = ep;
        }
        // its terms are final here (the leaf box terms are wave 4's): the lane maxima to LDS for
        // wave 0's row (m2, m5 of every lane; m0, m1, m3, m4 of the lanes h = 0 that account s_l)
        {
            ldsd* mx = SL + Cps::MX2;
            mx[lane] = rs.m2.get();
            mx[64 + lane] = rs.m5.get();
            if (h == 0) {
                mx[128 + lo] = rs.m0.get();
                mx[144 + lo] = rs.m1.get();
                mx[160 + lo] = rs.m3.get();
                mx[176 + lo] = rs.m4.get();
            }
        }
        zero_row();
        // the eta+ stream (after barrier B, the same wave): sqrtPf' eta11+ onto the box term
        lds_sync();  // B
        dstamp(2);
        v4 gA[RX];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) gA[rt] = v4{0, 0, 0, 0};
        if (BXL == 1) {
            // eta14 = x_l (box, cache.py:374-393) seeds the eta+ stream's L^T accumulator
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) {
                _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    if (!tok<NX>(rt, e)) continue;
                    const int r = row_of<NX>(rt, e);
                    const T lzv = XL[lo * NX + r], lpv = A[Cpa::LP + lo * NX + r], d14 = A[Cpa::D14 + lo * NX + r];
                    const T v = (d14 + alpha * (T(2) * lzv - lpv)) * ra;
                    T ep, x2;
                    Resid<T> dup = rs;  // (the terms are wave 4's: the same entries)
                    dup.fin(d14, v, box_sel(v, BX[2 * (NX + NU) + r], BX[2 * (NX + NU) + NX + r], nanf), lzv - lpv, ep, x2);
                    gA[rt][e] = ep;
                    gput(stv, eo, a.E14 + m + (l - m) * NX + r, ep);
                }
                __builtin_amdgcn_sched_barrier(0);  // a row block at a time: bounded live operands
            }
        }
        mmt(wp.fresh(), eA, gA);
        const ldsd* xl = XL;
        asm volatile("" : "+v"(xl));  // x+_l read again: not kept live across the SOC
        T lz[RX][4], ox[RX][4];
        ld_lr<NX>(xl + lo * NX, true, lz);
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
            ox[rt][e] = lz[rt][e] - alpha * gA[rt][e];
        if (stv) st_rows_o<T, NX>(out, X0 + l * NX, true, ox);
    }
    if (!(wv < 2 || (wv == 2 && deepest))) lds_sync();  // A2
    if (wv == 3 || wv == 4) wo(tid - 192, 128);  // the sweep's write-out
    // rows final at A, written in the waves' idle time up to barrier B (not before A2, which the
    // slot waves wait for): wave 5 (phase 1), wave 6 (the children's s); none: wave 3, and
    // waves 2, 4 outside the deepest tier
    if (wv == 5) emit_row();
    else if (wv == 6) emit_acc_row();
    else if (wv == 3 || ((wv == 2 || wv == 4) && !deepest)) zero_row();
    if (BXN == 1 && wv == 7) {
        // ================= the box rows of the families (Rectangle on eta7 = [x_i | u_i],
        // cache.py:374-393): eta7+ to the dual, and per entry the three streams' seeds
        // (eta7+ over eta7 in place, d - eta7+ and xi2 over the dead eta3 / eta4 rows)
        // lane group h takes the entries r = 4 t + h, t < 7 (x rows for t < 5); the operands of
        // entry t + 1 are read before entry t's stores (the in-place stores would otherwise
        // order each entry's reads behind the previous entry's writes)
        constexpr int NT = (NX + NU) / 4;
        auto opnd = [&](int t, T (&o5)[5]) {
            const int r = 4 * t + h;
            const bool xr = 4 * t < NX;
            o5[0] = xr ? XD[lq * SXD + r] : U[lq * NU + (xr ? 0 : r - NX)];
            o5[1] = xr ? A[Cpa::PX + lq * NX + r] : A[Cpa::PU + lq * NU + (xr ? 0 : r - NX)];
            o5[2] = A[Cpa::D7 + lq * (NX + NU) + r];
            o5[3] = BX[r];
            o5[4] = BX[(NX + NU) + r];
            _Pragma("unroll") for (int q = 0; q < 5; ++q) o5[q] = live ? o5[q] : T(0);  // dead lanes: zero terms
        };
        T cur[5], nxt[5];
        opnd(0, cur);
        _Pragma("unroll") for (int t = 0; t < NT; ++t) {
            if (t + 1 < NT) opnd(t + 1, nxt);
            const int r = 4 * t + h, o = lq * (NX + NU) + r;
            const T zv = cur[0], pv = cur[1], d7 = cur[2];
            const T v = (d7 + alpha * (T(2) * zv - pv)) * ra;
            T ep, x2;
            rs.fin(d7, v, box_sel(v, cur[3], cur[4], nanf), zv - pv, ep, x2);
            if (live) {
                gput(stv, eo, a.E7 + i * (NX + NU) + r, ep);
                A[Cpa::D7 + o] = ep;
                A[Cpa::SDW + o] = d7 - ep;
                A[Cpa::SDC + o] = x2;
            }
            _Pragma("unroll") for (int q = 0; q < 5; ++q) cur[q] = nxt[q];
        }
    }
    if (!(wv == 2 && deepest)) {
        dstamp(2);
        lds_sync();  // B: the stream rows, tau, s, y of the half step are in LDS
    }
    if (wv == 7) emit_fin_row();  // its box terms (zeros when unboxed)
    // ============ II: the L^T streams (operators.py:73-94), one MFMA chain per wave
    if (wv == 0 || wv == 1 || wv == 3) {
        // families: wave 0 the eta+ stream onto Gamma' eta7 (box) -> x_i, u_i of the half step;
        // wave 1 the (d - eta+) stream, wave 3 the xi2 stream (to LDS for wave 1's residual terms)
        const int q = wv == 0 ? 0 : (wv == 1 ? 1 : 2);
        v4 g[RX], hh[RU];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) g[rt] = v4{0, 0, 0, 0};
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) hh[rt] = v4{0, 0, 0, 0};
        if (BXN == 1) {
            // the box terms of the stream (wave 7's seeds: eta7+, d - eta7+ or xi2 per entry of
            // [x | u]) seed the accumulator
            const ldsd* sd = A + (q == 0 ? Cpa::D7 : (q == 1 ? Cpa::SDW : Cpa::SDC)) + lq * (NX + NU);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NX>(rt, e)) g[rt][e] = live ? sd[row_of<NX>(rt, e)] : T(0);
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NU>(rt, e)) hh[rt][e] = live ? sd[NX + row_of<NU>(rt, e)] : T(0);
        }
        {
            // the slots' rows of stream q summed per parent in slot order
            const ldsd* sb = SL + Cps::SB;
            T sx[RX][4], su[RU][4], ax[RX][4], au[RU][4];
            lds_getc<T, NX>(sb + q * SS, sx);
            lds_getc<T, NU>(sb + q * SS + SX, su);
            lds_getc<T, NX>(sb + (3 + q) * SS, ax);
            lds_getc<T, NU>(sb + (3 + q) * SS + SX, au);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) sx[rt][e] += ax[rt][e];
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) su[rt][e] += au[rt][e];
            mmt(wq.fresh(), sx, g);
            mmt(wr.fresh(), su, hh);
        }
        if (wv == 0) {
            T xz[RX][4], uz[RU][4], ox[RX][4], ou[RU][4];
            ld_lr<NX>(XD + lq * SXD, live, xz);
            ld_lr<NU>(U + lq * NU, live, uz);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                ox[rt][e] = xz[rt][e] - alpha * g[rt][e];
            if (stv) st_rows_o<T, NX>(out, X0 + i * NX, live, ox);
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                ou[rt][e] = uz[rt][e] - alpha * hh[rt][e];
            if (stv) st_rows_o<T, NU>(out, U0 + i * NU, live, ou);
            if (deepest) {  // the leaf wave's lane maxima join this wave's row
                const ldsd* mx = SL + Cps::MX2;
                const T v2 = mx[lane], v5 = mx[64 + lane];
                const T v0 = mx[128 + lo], v1 = mx[144 + lo], v3 = mx[160 + lo], v4 = mx[176 + lo];
                rs.m2.add(v2);
                rs.m5.add(v5);
                rs.m0.add(h == 0 ? v0 : T(0));
                rs.m1.add(h == 0 ? v1 : T(0));
                rs.m3.add(h == 0 ? v3 : T(0));
                rs.m4.add(h == 0 ? v4 : T(0));
            }
            emit_row();
            dstamp(3);
            lds_sync();  // C
        } else if (wv == 3) {
            // xi2 stream to LDS, compacted (the child scalars are dead after barrier A2)
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NX>(rt, e)) A[Cpa::SC + cpos<NX>(rt, e)] = g[rt][e];
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NU>(rt, e)) A[Cpa::SC + SX + cpos<NU>(rt, e)] = hh[rt][e];
            dstamp(3);
            lds_sync();  // C
        } else {
            // ============ III: the residual terms of x_i, u_i from both streams; all but the xi2
            // stream's (xi0 = xi1 + L^T xi2) before barrier C, with the row's other five maxima
            T xz[RX][4], xp[RX][4], uz[RU][4], up[RU][4];
            ld_lr<NX>(XD + lq * SXD, live, xz);
            ld_lr<NX>(A + Cpa::PX + lq * NX, live, xp);
            ld_lr<NU>(U + lq * NU, live, uz);
            ld_lr<NU>(A + Cpa::PU + lq * NU, live, up);
            T x1x[RX][4], x1u[RU][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NX>(rt, e)) x1x[rt][e] = rs.account_pre(xp[rt][e], xz[rt][e], g[rt][e]);
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NU>(rt, e)) x1u[rt][e] = rs.account_pre(up[rt][e], uz[rt][e], hh[rt][e]);
            double m5[5] = {rs.m1.get(), rs.m2.get(), rs.m3.get(), rs.m4.get(), rs.m5.get()};
            wave_bmax_n<5>(m5);
            dstamp(3);
            lds_sync();  // C
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NX>(rt, e)) rs.account_post(x1x[rt][e], A[Cpa::SC + cpos<NX>(rt, e)]);
            _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NU>(rt, e)) rs.account_post(x1u[rt][e], A[Cpa::SC + SX + cpos<NU>(rt, e)]);
            const double mm[6] = {wave_bmax(rs.m0.get()), m5[0], m5[1], m5[2], m5[3], m5[4]};
            put_row(mm);
        }
    } else if ((wv == 4 || wv == 5) && deepest) {
        // leaves: wave 4 the (d - eta+) stream, wave 5 the xi2 stream (to LDS for wave 4's terms)
        v4 g[RX];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) g[rt] = v4{0, 0, 0, 0};
        if (BXL == 1) {
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) {
                _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                    if (!tok<NX>(rt, e)) continue;
                    const int r = row_of<NX>(rt, e);
                    const T lzv = XL[lo * NX + r], lpv = A[Cpa::LP + lo * NX + r], d14 = A[Cpa::D14 + lo * NX + r];
                    const T v = (d14 + alpha * (T(2) * lzv - lpv)) * ra;
                    T ep, x2;
                    Resid<T> dup = rs;  // the entry's terms: wave 4's (waves 2 and 5 compute the same entries)
                    dup.fin(d14, v, box_sel(v, BX[2 * (NX + NU) + r], BX[2 * (NX + NU) + NX + r], nanf), lzv - lpv, ep, x2);
                    if (wv == 4) {
                        rs.m2.add(x2);
                        rs.m5.add(ep - d14);
                    }
                    g[rt][e] = wv == 4 ? d14 - ep : x2;
                }
                __builtin_amdgcn_sched_barrier(0);  // a row block at a time: bounded live operands
            }
        }
        {
            T ew[RX][4];
            lds_getc<T, NX>(SL + (wv == 4 ? Cps::LEW : Cps::LEC), ew);
            mmt(wp.fresh(), ew, g);
        }
        if (wv == 5) {
            // compacted; the eta11 operand rows are dead after barrier A2
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NX>(rt, e)) A[Cpa::D11 + cpos<NX>(rt, e)] = g[rt][e];
            dstamp(3);
            lds_sync();  // C
        } else {
            // the leaves' residual terms as wave 1's: all but xi0 before barrier C
            T lz[RX][4], lp[RX][4], x1x[RX][4];
            ld_lr<NX>(XL + lo * NX, true, lz);
            ld_lr<NX>(A + Cpa::LP + lo * NX, true, lp);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NX>(rt, e)) x1x[rt][e] = rs.account_pre(lp[rt][e], lz[rt][e], g[rt][e]);
            double m5[5] = {rs.m1.get(), rs.m2.get(), rs.m3.get(), rs.m4.get(), rs.m5.get()};
            wave_bmax_n<5>(m5);
            dstamp(3);
            lds_sync();  // C
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<NX>(rt, e)) rs.account_post(x1x[rt][e], A[Cpa::D11 + cpos<NX>(rt, e)]);
            const double mm[6] = {wave_bmax(rs.m0.get()), m5[0], m5[1], m5[2], m5[3], m5[4]};
            put_row(mm);
        }
    } else if (wv == 6 && live) {
        // ================= the AVaR kernel projection of the family (cache.py:290-317)
        const T al = A[Cpa::PS + lq * 24 + 20];
        const T y2c = ks.y[lo][2 * C];
        T rk[C], sr = T(0);
        _Pragma("unroll") for (int k = 0; k < C; ++k) {
            rk[k] = al * ks.y[lo][k] - ks.y[lo][C + k] + y2c - ks.tau[lo][k] - ks.s[lo][k];
            sr += rk[k];
        }
        const T aa = al * al + T(3);
        T sw = T(0);
        _Pragma("unroll") for (int k = 0; k < C; ++k) {
            const T w = (rk[k] - sr / (aa + (T)C)) / aa;
            sw += w;
            if (k == h) {
                const int j = 1 + C * i + k;
                gput(stv, out, a.Y0 + yo + k, ks.y[lo][k] - al * w);
                gput(stv, out, a.Y0 + yo + C + k, ks.y[lo][C + k] + w);
                gput(stv, out, a.T0 + j, ks.tau[lo][k] + w);
                gput(stv, out, a.S0 + j, ks.s[lo][k] + w);
            }
        }
        if (h == 0) gput(stv, out, a.Y0 + yo + 2 * C, y2c - sw);
    }
    if (!(wv == 0 || wv == 1 || wv == 3 || ((wv == 4 || wv == 5) && deepest))) {
        dstamp(3);
        lds_sync();  // C
    }
    dstamp(5);
    flag_nan(a.ctl, nanf, a.nanbit);
    dstamp(4);
}

// one tier's subtree o (L nonleaf levels): steps 1-7 of the header. BX > 0 (k_drc): the CP
// iteration of the subtree's families follows (cp_phase; BX = 1 every node boxed, 2 none)
template <int NX, int NU, int C, int BS, int UMAX, int L, int BX = 0>
__device__ __forceinline__ void tier_body(const DrPlan& pl, int k, int o, glbd* z, unsigned tag, bool work,
                                          Stamps& stp, int& s_ok, ldsd* sm, const DrcArg* ca = nullptr,
                                          const Bufs* bfp = nullptr, double alpha = 0.0) {
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
    constexpr bool CPF = BX > 0;
    static_assert(!CPF || (C == 2 && L == 4), "k_drc: binary trees, tiers of 4 levels");
    ldsd* CPA = X0B + NX;  // k_drc: the CP operand region (Cpa)
    const int R0 = pl.sbase[s0] + o;  // the subtree's root
    const bool gat = !(kDiag && (pl.fault & 128));  // timing probes (diagnostic builds)
    if constexpr (CPF)
        if (kDiag && (pl.fault & 512)) {  // the CP step alone
            if (work) {
                CpaStage cs;
                if (gat) cpa_issue<NX, NU, BX>(*ca, pl, *bfp, R0, deepest, cs);
                TableDma<Cps::WA, BS / 64>::issue(SL + 3 * SLOT, ca->img);
                TableDma<Cps::WB, BS / 64>::issue(SL + 2 * SLOT, ca->img + Cps::WA);
                dma_wait();
                if (gat) cpa_commit(CPA, cs);
                lds_sync();
                if (!(pl.fault & 64))
                    cp_phase<NX, NU, BX, BX>(*ca, *bfp, alpha, pl.X0, pl.U0, R0, deepest, XD, XL, U, CPA, SL, nullptr, pl.nblk,
                                             [](int, int) {},
                                         !(pl.fault & 1024));
            }
            return;
        }
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
        // k_drc: the CP operands are loaded (older than the forward tables) and go to LDS once
        // they have landed, still inside the wait below
        CpaStage cs;
        if constexpr (CPF)
            if (work && gat) cpa_issue<NX, NU, BX>(*ca, pl, *bfp, R0, deepest, cs);
        if (!(kDiag && (pl.fault & 4)))
            static_for<0, L>([&](auto fc) {
                constexpr int f = fc.value;
                TF::issue(SL + (L - 1 - f) * SLOT, pl.fimg + (size_t)(s0 + f) * TFN);
            });
        if constexpr (CPF)
            if (work && gat) {
                wait_vm_c<L * TF::IPW>();  // the operands have landed (the forward tables stay in flight)
                cpa_commit(CPA, cs);
            }
        if (!poll_gran(pl.gx + (size_t)(tt.w0 + o) * G, G, tag, (ldsu*)XD, pl.timeout, pl.sync, s_ok)) {
            dma_wait();
            return;
        }
        stamp(pl, stp);
    } else if (tid < NX) {
        XD[tid] = X0B[tid];  // x_0 = x0bar (cache.py:282)
    }
    // ---- 6. forward sweep: level f waits for its table only (the younger ones stay in flight).
    // k_drc: the CP weight image lands in the slots levels 0 and 1 free (issued behind their
    // barriers, so level f >= 2 also lets those younger DMAs stay in flight)
    typedef TableDma<Cps::WA, NW> WAD;
    typedef TableDma<Cps::WB, NW> WBD;
    static_for<0, L>([&](auto fc) {
        constexpr int f = fc.value, cnt = cpow(C, f), off = (cnt - 1) / (C - 1);
        constexpr int XW = CPF ? (f >= 2 ? WAD::IPW : 0) + (f >= 3 ? WBD::IPW : 0) : 0;
        wait_vm_c<(L - 1 - f) * TF::IPW + XW>();
        lds_sync();
        stamp(pl, stp);
#ifndef DRC_NO_WDMA  // (timing probe builds only)
        if constexpr (CPF && f == 1) WAD::issue(SL + 3 * SLOT, ca->img);
        if constexpr (CPF && f == 2) WBD::issue(SL + 2 * SLOT, ca->img + Cps::WA);
#endif
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
    if constexpr (CPF) {
        if (work && gat && top) {  // the top has no wait to hide its operands behind
            CpaStage ct;
            cpa_issue<NX, NU, BX>(*ca, pl, *bfp, R0, deepest, ct);
            dma_wait();
            cpa_commit(CPA, ct);
        }
        dma_wait();
        lds_sync();  // operands, weights and boxes in LDS for every wave
    }
    // the write-out of the projected rows by lanes t0, t0 + nt, ...: by the whole workgroup here,
    // or (k_drc) inside the CP step by two waves that wait there anyway, so that the CP step
    // starts right behind the forward sweep
    auto writeout = [&](int t0, int nt) {
        if (!(work && !(kDiag && (pl.fault & 8)))) return;
        static_for<0, L + 1>([&](auto lc) {
            constexpr int l = lc.value, cnt = cpow(C, l), off = (cnt - 1) / (C - 1);
            if (l == 0 && !top) return;  // the parent writes this subtree's root row
            glb2* dst = (glb2*)(z + pl.X0 + (size_t)gl[l] * NX);
            if constexpr (l < L) {
                for (int e = t0; e < cnt * (NX / 2); e += nt) {
                    const int r = e / (NX / 2), c = e - r * (NX / 2);
                    dst[e] = ld2(XD + (off + r) * SXD + 2 * c);
                }
            } else {
                for (int e = t0; e < NB * (NX / 2); e += nt) dst[e] = ld2(XL + 2 * e);
            }
        });
        static_for<0, L>([&](auto lc) {
            constexpr int l = lc.value, cnt = cpow(C, l), off = (cnt - 1) / (C - 1);
            glb2* dst = (glb2*)(z + pl.U0 + (size_t)gl[l] * NU);
            for (int e = t0; e < cnt * (NU / 2); e += nt) dst[e] = ld2(U + off * NU + 2 * e);
        });
    };
    if constexpr (!CPF) writeout(tid, BS);
    if constexpr (CPF) {
        wg_stamp(pl, 3);
#ifndef DRC_NO_CPCODE  // (timing probe builds only)
        if (work && !(kDiag && (pl.fault & 64)))
            cp_phase<NX, NU, BX, BX>(*ca, *bfp, alpha, pl.X0, pl.U0, R0, deepest, XD, XL, U, CPA, SL,
                                     kDiag ? pl.stamps : nullptr, pl.nblk, writeout, !(kDiag && (pl.fault & 1024)));
        else
            writeout(tid, BS);
#else
        writeout(tid, BS);
#endif
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

// the previous iteration's stopping test (solver.py:137-161) by k_drc's extra workgroup: the
// residual rows (one per sweep wave) spread over all its lanes (a few loads each, issued
// together), the maxima by DPP per wave and through LDS across the waves
__device__ __forceinline__ void cp_check_block(const ChkArg& ck, ldsd* red) {
    Ctl* ctl = ck.ctl;
    if (ctl->done) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nt = blockDim.x;
    double m[6] = {0, 0, 0, 0, 0, 0};
    _Pragma("unroll") for (int j = 0; j < 8; ++j) {
        const int r = tid + j * nt;
        if (r < ck.rows) _Pragma("unroll") for (int q = 0; q < 6; ++q) m[q] = bmax(m[q], ck.part[(size_t)r * 6 + q]);
    }
    for (int r = tid + 8 * nt; r < ck.rows; r += nt)
        _Pragma("unroll") for (int q = 0; q < 6; ++q) m[q] = bmax(m[q], ck.part[(size_t)r * 6 + q]);
    wave_bmax_n<6>(m);
    if (lane == 63) _Pragma("unroll") for (int q = 0; q < 6; ++q) red[q * 16 + wv] = m[q];
    __syncthreads();
    if (tid != 0) return;
    _Pragma("unroll") for (int q = 0; q < 6; ++q) {
        double b = red[q * 16];
        for (int w = 1; w < (nt >> 6); ++w) b = bmax(b, red[q * 16 + w]);
        m[q] = b;
    }
    const int k = ctl->k;
    for (int q = 0; q < 6; ++q) ck.hist[(size_t)k * 6 + q] = m[q];
    const double err = nmax(nmax(m[0], m[1]), m[2]);
    if (ctl->flags & ck.nanbit) ctl->flags |= 1;
    if (k >= ctl->max_iters || err <= ctl->tol || (ctl->flags & 1)) {
        ctl->done = 1;
        ctl->final_k = k;
    } else {
        ctl->k = k + 1;
    }
}

// k_drc: k_dr's sweep with each subtree's CP families behind its forward sweep (every tier of 4
// levels, binary trees at nx / nu = 20 / 8; the host checks the plan). One launch per CP
// iteration; the extra workgroup runs the previous iteration's stopping test (its residual rows
// are the other of the two alternating row sets, ck.part).
template <int NX, int NU, int C, int BX>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4)))
k_drc(DrPlan pl, const DrcArg* __restrict__ cap, Bufs bf, ChkArg ck) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ Stamps stp;
    __shared__ int s_ok;
    const int tid = threadIdx.x;
    if (ck.on && (int)blockIdx.x == pl.nblk) {  // the previous CP iteration's stopping test
        cp_check_block(ck, (ldsd*)smem_);
        return;
    }
    if (tid == 0) {
        stp.n = 0;
        s_ok = 1;
    }
    const unsigned long long sw = sload_pair(pl.sync);
    const unsigned err = (unsigned)(sw >> 32);
    const unsigned tag = (unsigned)sw + 1u;
    // the CP arguments are read from device memory where the CP step uses them (as kernel
    // arguments they were loaded at the start and kept in scalar registers across the sweep,
    // which then spilled scalars inside its levels)
    Ctl* ctl = cap->ctl;
    const int done = ctl->done;
    const double alpha = ctl->alpha;  // the CP step size, read at the start (not on the CP path)
    stamp(pl, stp);
    wg_stamp(pl, 0);
    if (err) return;
    int k, o;
    role(pl, k, o);
    glbd* z = pick3(bf, 1);
    if (pl.t[k].L == 4)
        tier_body<NX, NU, C, 512, 1, 4, BX>(pl, k, o, z, tag, done == 0, stp, s_ok, (ldsd*)smem_, cap, &bf, alpha);
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

bool drc_supported(int nx, int nu, int C) { return nx == 20 && nu == 8 && C == 2; }
size_t drc_lds(int nx, int nu, int C) { return dr_lds(nx, nu, C, 4) + 8 * (size_t)kDrcCpa; }
int drc_occupancy(size_t lds) {
    int nb = 0;
    const void* kf = (const void*)k_drc<20, 8, 2, 1>;
    (void)hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kf, 512, lds) != hipSuccess) return 0;
    int nb2 = 0;
    const void* kf2 = (const void*)k_drc<20, 8, 2, 2>;
    (void)hipFuncSetAttribute(kf2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb2, kf2, 512, lds) != hipSuccess) return 0;
    return nb < nb2 ? nb : nb2;
}
void drc_launch(const DrPlan& pl, const DrcArg* dca, int box, size_t lds, Bufs bf, ChkArg ck, hipStream_t s) {
    const int grid = pl.nblk + (ck.on ? 1 : 0);
    if (box == 1) {
        (void)hipFuncSetAttribute((const void*)k_drc<20, 8, 2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        k_drc<20, 8, 2, 1><<<grid, 512, lds, s>>>(pl, dca, bf, ck);
    } else {
        (void)hipFuncSetAttribute((const void*)k_drc<20, 8, 2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        k_drc<20, 8, 2, 2><<<grid, 512, lds, s>>>(pl, dca, bf, ck);
    }
}
const char* drc_name() { return "k_drc<20, 8, 2>"; }
bool dr_diag_build() { return kDiag; }

}  // namespace raocp
