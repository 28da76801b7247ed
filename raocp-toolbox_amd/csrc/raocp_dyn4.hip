// raocp_dyn4.hip — the dynamics projection (cache.py:259-288) of the regular trees k_dy3 takes,
// in ONE launch (host interface: raocp_dyn4.h).
//
// Device form of the recursion (raocp_dyn3.hip header): backward, a tile of 16 parents i of
// stage t (children j = 1 + C i + k; q_j = -x_j at the leaves):
//     h = sum_k B_k' q_j,  a = sum_k A_k' q_j,  v = u_i - h,  d_i = Rinv v,  q_i = (-x_i + a) + G v
// forward (x_0 = x0bar):  u_i = K x_i + d_i,  x_j = A_k x_i + B_k u_i
// with k_dy3's per-stage table images (k_dy3_image) and MFMA tile arithmetic (the transposed
// form of raocp_cp3.hip: a product's accumulators are the next product's B operand).
//
// k_dy3 runs a launch per stage and direction (12-14 at configs 4 / 5): each small stage costs
// a dispatch, an image fill and a drain for a few microseconds of MFMA work. Here every tile
// is a task of one persistent launch, a workgroup of 4 waves per task (child slot k on wave k,
// the slot sums through LDS to wave 0 in slot order -- k_dy3's slot-parallel arithmetic), and
// tasks wait only for the tiles they read:
//   backward tile (t, b): the C child tiles (t + 1, C b .. C b + C - 1) have stored their q rows;
//   the top task (stages ts-1 .. 0 back, 0 .. ts-1 forward in one workgroup): every tile of ts;
//   forward tile (t, b): its parents' tile (t - 1, b / C) (or the top) has stored their x rows.
// Flags carry the projection's epoch (sync[0] + 1). Rows another workgroup of the launch reads
// are written with agent-scope (sc1, write-through) stores and read with agent-scope loads; a
// producer waits for its stores (vmcnt(0) on every wave), a barrier, then one lane stores the
// flag (sc1); a consumer's wave 0 polls the flags (bounded), a barrier, then its loads
// (MI355X_MICROARCH.md handoff-flag / publish-large: no L2 write-back or invalidate per task).
// Stages of many tiles run as tasks of 4 tiles, a wave per tile with its C slots in sequence
// (k_dy3's wide-stage arithmetic); stages of few tiles a tile per task, a wave per slot.
// The last workgroup to finish advances the epoch. Every wait is bounded: a timed-out
// workgroup sets the error word and leaves, later waits see it and leave, the host reports
// RAOCP_ERR_STATE and clears the words (raocp_capi.hip fuse_err).
//
// Every workgroup walks its tasks in order (task = blockIdx.x + r * nwg) and a task waits only
// for earlier tasks, so with the whole grid resident (host check: occupancy x CUs) the
// earliest unfinished task can always run: no deadlock. Like k_dr, k_dy4 assumes its grid has
// the device's CUs to itself (raocp_dynr.hip).

#include "raocp_dyn4.h"
#include "raocp_tile.h"

namespace raocp {
namespace {

__device__ __forceinline__ unsigned ld_u32(const unsigned* p) {
    return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_u32(unsigned* p, unsigned v) {
    __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// row-layout loads / stores (raocp_tile.h ld_rows / st_rows) of rows other workgroups of the
// launch write or read: agent-scope relaxed accesses (global_load / global_store ... sc1),
// 8 bytes each (an fp32 pair where a lane's run is 8-B aligned)
template <class T>
struct Sc1;
template <>
struct Sc1<double> {
    static __device__ __forceinline__ double ld(const double* p) { return ld_sc1(p); }
    static __device__ __forceinline__ void st(double* p, double v) { st_sc1(p, v); }
};
template <>
struct Sc1<float> {
    static __device__ __forceinline__ float ld(const float* p) {
        return __uint_as_float(__hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    static __device__ __forceinline__ void st(float* p, float v) {
        __hip_atomic_store((gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
};
template <class T, int R>
__device__ __forceinline__ void ld_rows_c(const T* v, bool live, T (&a)[(R + 15) / 16][4]) {
    constexpr int KC = R / 4;
    const T* b = v + KC * ((threadIdx.x & 63) >> 4);
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) {
        if constexpr (sizeof(T) == 4 && KC % 2 == 0) {
            _Pragma("unroll") for (int e = 0; e < 4; e += 2) {
                if (!tok<R>(rt, e)) {
                    a[rt][e] = a[rt][e + 1] = T(0);
                    continue;
                }
                const unsigned long long w =
                    __hip_atomic_load((const gu64*)(b + 4 * rt + e), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                a[rt][e] = live ? __uint_as_float((unsigned)w) : T(0);
                a[rt][e + 1] = live ? __uint_as_float((unsigned)(w >> 32)) : T(0);
            }
        } else {
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                T w = T(0);
                if (tok<R>(rt, e)) w = Sc1<T>::ld(b + 4 * rt + e);
                a[rt][e] = live ? w : T(0);
            }
        }
    }
}
template <class T, int R>
__device__ __forceinline__ void st_rows_c(T* v, bool live, const T (&a)[(R + 15) / 16][4]) {
    constexpr int KC = R / 4;
    T* b = v + KC * ((threadIdx.x & 63) >> 4);
    if (!live) return;
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) {
        if constexpr (sizeof(T) == 4 && KC % 2 == 0) {
            _Pragma("unroll") for (int e = 0; e < 4; e += 2) {
                if (!tok<R>(rt, e)) continue;
                const unsigned long long w =
                    (unsigned long long)__float_as_uint(a[rt][e]) | ((unsigned long long)__float_as_uint(a[rt][e + 1]) << 32);
                __hip_atomic_store((gu64*)(b + 4 * rt + e), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<R>(rt, e)) Sc1<T>::st(b + 4 * rt + e, a[rt][e]);
        }
    }
}

// wave 0's lanes poll flags f[0, n) until each carries tag (bounded; the error word of another
// workgroup ends the wait too), then an agent-scope acquire and a barrier; false on a timeout
__device__ __forceinline__ bool wait_flags(const unsigned* f, int n, unsigned tag, const Dy4Plan& pl, int& s_ok) {
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        bool bad = false;
        for (int r0 = 0; r0 < n && !bad; r0 += 64) {
            const int r = r0 + lane;
            for (;;) {
                const bool ok = r >= n || ld_u32(f + r) == tag;
                if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > pl.timeout || ld_u32(pl.sync + 1) != 0u) {
                    bad = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (bad && lane == 0) {
            s_ok = 0;
            st_u32(pl.sync + 1, 1u);
        }
    }
    __syncthreads();
    return s_ok != 0;
}
// the workgroup's (write-through) stores, then flags f[0, n): every wave waits for its own
// stores (vmcnt(0): the barrier alone does not), the barrier, then lanes of wave 0 store the
// flags (sc1)
__device__ __forceinline__ void release_flags(unsigned* f, int n, unsigned tag) {
    dma_wait();
    __syncthreads();
    if ((int)threadIdx.x < n) st_u32(f + threadIdx.x, tag);
}

// the stage images (k_dy3_image: raocp_dyn3.hip Dy3Lds), the same fragment tables as WL
template <class T, int NX, int NU, int C>
struct Dy4 {
    typedef WL<T, NU, NX> WB;   // B_k'
    typedef WL<T, NX, NX> WA;   // A_k' (backward) / A_k (forward)
    typedef WL<T, NU, NU> WRI;  // Rinv
    typedef WL<T, NX, NU> WG;   // G (backward) / B_k (forward)
    typedef WL<T, NU, NX> WK;   // K
    static constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16;
    static constexpr int BN = C * (WB::N + WA::N) + WRI::N + WG::N;  // [B_k' | A_k']_k [Rinv | G]
    static constexpr int FN = WK::N + C * (WA::N + WG::N);           // K [A_k | B_k]_k
    static constexpr int IMG = BN > FN ? BN : FN;
    static constexpr int RED = C * (RU + RX) * 4 * 64;  // the slot sums [slot][RU + RX][4][64]
    static constexpr size_t lds() { return (size_t)(IMG + RED) * sizeof(T); }
};

template <class T, int NX, int NU, int C>
__global__ void __launch_bounds__(256) k_dy4(Dy4Plan pl, Dev p, const Ctl* ctl, ChkArg ck, double* z_, double* q_,
                                             double* d_, const double* x0_) {
    typedef Dy4<T, NX, NU, C> D;
    typedef typename MF<T>::v4 v4;
    static_assert(C >= 2 && C <= 4, "a wave per child slot");
    constexpr int RX = D::RX, RU = D::RU;
    extern __shared__ __attribute__((aligned(16))) double dsm_[];
    __shared__ int s_ok;
    const int tid = threadIdx.x;
    if (ck.on && (int)blockIdx.x == pl.nwg) {  // the previous CP iteration's stopping test
        if (tid < 64) cp_check_wave(ck);
        return;
    }
    typedef __attribute__((address_space(3))) T lT;
    lT* wl = (lT*)dsm_;
    lT* red = wl + D::IMG;
    const unsigned tag = ld_u32(pl.sync) + 1u;
    if (ld_u32(pl.sync + 1)) return;  // an earlier projection timed out: the host resets the words
    // (the stopping test of this launch's extra workgroup may set done meanwhile: a workgroup
    // that saw it skips its arithmetic, never the protocol, as k_dr)
    const bool work = !(ctl && ctl->done);
    if (tid == 0) s_ok = 1;
    __syncthreads();
    glbp<T> z = (glbp<T>)z_;
    const int lane = tid & 63, lo = lane & 15, wv = tid >> 6;
    int cur = -1;  // the image in LDS: 2 t (backward) or 2 t + 1 (forward)
    auto image = [&](int t, bool fwd) {
        const int key = 2 * t + (fwd ? 1 : 0);
        if (key == cur) return;
        __syncthreads();  // every read of the previous image is done
        // the child-slot tables depend on the slots' kinds only: with the same kinds at every
        // stage a stage change within a direction reloads the class part alone
        const bool part = pl.same_kinds && cur >= 0 && (cur & 1) == (fwd ? 1 : 0);
        if (!fwd) {
            const double* src = pl.bimg + (size_t)t * pl.bstride;
            constexpr int off = C * (D::WB::N + D::WA::N);  // [Rinv | G] (a multiple of 64 elements)
            if (part) lds_fill((lds_d*)(wl + off), src + (size_t)off * sizeof(T) / 8, (D::BN - off) * (int)sizeof(T) / 16);
            else lds_fill((lds_d*)wl, src, D::BN * (int)sizeof(T) / 16);
        } else {
            const double* src = pl.fimg + (size_t)t * pl.fstride;
            lds_fill((lds_d*)wl, src, (part ? D::WK::N : D::FN) * (int)sizeof(T) / 16);
        }
        dma_wait();
        __syncthreads();
        cur = key;
    };
    // the parents' (d, q) of a tile from the slot sums ha = sum_k B_k' q_j, aa = sum_k A_k' q_j
    auto back_finish = [&](int iq, bool live, const T (&u)[RU][4], const T (&x)[RX][4], const v4 (&ha)[RU],
                           const v4 (&aa)[RX]) {
        lT* wr = wl + C * (D::WB::N + D::WA::N);
        const typename D::WRI wri{wr};
        const typename D::WG wg{wr + D::WRI::N};
        T v[RU][4];
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) v[rt][e] = u[rt][e] - ha[rt][e];
        v4 dv[RU], gv[RX];
        _Pragma("unroll") for (int r = 0; r < RU; ++r) dv[r] = v4{0, 0, 0, 0};
        _Pragma("unroll") for (int r = 0; r < RX; ++r) gv[r] = v4{0, 0, 0, 0};
        mmt(wri, v, dv);
        mmt(wg, v, gv);
        T dd[RU][4], qq[RX][4];
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) dd[rt][e] = dv[rt][e];
        _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e)
            qq[rt][e] = (-x[rt][e] + aa[rt][e]) + gv[rt][e];
        st_rows_c<T, NU>((T*)d_ + (size_t)iq * NU, live, dd);
        st_rows_c<T, NX>((T*)q_ + (size_t)iq * NX, live, qq);
    };
    // child slot k's rows of parent iq: q_j, or -x_j at the leaves (stage N - 1)
    auto load_q = [&](int t, int iq, bool live, int k, T (&qj)[RX][4]) {
        const int j = 1 + C * iq + k;
        if (t == pl.N - 1) {
            ld_rows<T, NX>((cglbp<T>)z + pl.X0 + (size_t)j * NX, live, qj);
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) qj[rt][e] = -qj[rt][e];
        } else {
            ld_rows_c<T, NX>((const T*)q_ + (size_t)j * NX, live, qj);
        }
    };
    // ---- backward tile b of stage t, a wave per child slot: wave k < C slot k's products, the
    // slot sums through LDS to wave 0 in slot order, wave 0 the parents (k_dy3's slot-parallel
    // arithmetic)
    auto back_tile = [&](int t, int b) {
        const int i0 = pl.i0[t] + 16 * b, i = i0 + lo;
        const bool live = i < pl.i0[t + 1];
        const int iq = live ? i : i0;
        T u[RU][4], x[RX][4];
        if (wv == 0) {
            ld_rows<T, NU>((cglbp<T>)z + pl.U0 + (size_t)iq * NU, live, u);
            ld_rows<T, NX>((cglbp<T>)z + pl.X0 + (size_t)iq * NX, live, x);
        }
        v4 ha[RU], aa[RX];
        _Pragma("unroll") for (int r = 0; r < RU; ++r) ha[r] = v4{0, 0, 0, 0};
        _Pragma("unroll") for (int r = 0; r < RX; ++r) aa[r] = v4{0, 0, 0, 0};
        if (wv < C) {
            T qj[RX][4];
            load_q(t, iq, live, wv, qj);
            const typename D::WB wb{wl + wv * (D::WB::N + D::WA::N)};
            const typename D::WA wa{wl + wv * (D::WB::N + D::WA::N) + D::WB::N};
            mmt(wb, qj, ha);
            mmt(wa, qj, aa);
            if (wv > 0) {
                lT* rd = red + (size_t)wv * (RU + RX) * 4 * 64;
                _Pragma("unroll") for (int r = 0; r < RU; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    rd[(r * 4 + e) * 64 + lane] = ha[r][e];
                _Pragma("unroll") for (int r = 0; r < RX; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    rd[((RU + r) * 4 + e) * 64 + lane] = aa[r][e];
            }
        }
        __syncthreads();
        if (wv == 0) {
            _Pragma("unroll") for (int kk = 1; kk < C; ++kk) {
                const lT* rd = red + (size_t)kk * (RU + RX) * 4 * 64;
                _Pragma("unroll") for (int r = 0; r < RU; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    ha[r][e] += rd[(r * 4 + e) * 64 + lane];
                _Pragma("unroll") for (int r = 0; r < RX; ++r) _Pragma("unroll") for (int e = 0; e < 4; ++e)
                    aa[r][e] += rd[((RU + r) * 4 + e) * 64 + lane];
            }
            back_finish(iq, live, u, x, ha, aa);
        }
    };
    // ---- backward tiles b0 .. b0 + cnt - 1 of a wide stage, a wave per tile: the C slots'
    // products accumulate in the MFMA registers (k_dy3's wide-stage arithmetic)
    auto back_wide = [&](int t, int b0, int cnt) {
        if (wv >= cnt) return;
        const int i0 = pl.i0[t] + 16 * (b0 + wv), i = i0 + lo;
        const bool live = i < pl.i0[t + 1];
        const int iq = live ? i : i0;
        T qj[C][RX][4], u[RU][4], x[RX][4];
        _Pragma("unroll") for (int k = 0; k < C; ++k) load_q(t, iq, live, k, qj[k]);
        ld_rows<T, NU>((cglbp<T>)z + pl.U0 + (size_t)iq * NU, live, u);
        ld_rows<T, NX>((cglbp<T>)z + pl.X0 + (size_t)iq * NX, live, x);
        v4 ha[RU], aa[RX];
        _Pragma("unroll") for (int r = 0; r < RU; ++r) ha[r] = v4{0, 0, 0, 0};
        _Pragma("unroll") for (int r = 0; r < RX; ++r) aa[r] = v4{0, 0, 0, 0};
        _Pragma("unroll") for (int k = 0; k < C; ++k) {
            const typename D::WB wb{wl + k * (D::WB::N + D::WA::N)};
            const typename D::WA wa{wl + k * (D::WB::N + D::WA::N) + D::WB::N};
            mmt(wb, qj[k], ha);
            mmt(wa, qj[k], aa);
        }
        back_finish(iq, live, u, x, ha, aa);
    };
    // ---- forward: slot k's children of the tile's parents, u = K x + d (wave 0 of a tile
    // stores u), x_j = A_k x + B_k u
    auto fwd_rows = [&](int t, int b, int k0, int k1, bool su) {
        const int i0 = pl.i0[t] + 16 * b, i = i0 + lo;
        const bool live = i < pl.i0[t + 1];
        const int iq = live ? i : i0;
        T x[RX][4], dc[RU][4];
        if (i == 0) ld_rows<T, NX>((cglbp<T>)x0_, true, x);  // x_0 = x0bar (cache.py:282)
        else ld_rows_c<T, NX>((const T*)z_ + pl.X0 + (size_t)iq * NX, live, x);
        ld_rows_c<T, NU>((const T*)d_ + (size_t)iq * NU, live, dc);
        if (i == 0 && su) st_rows<T, NX>(z + pl.X0, true, x);
        const typename D::WK wk{wl};
        v4 ku[RU];
        _Pragma("unroll") for (int r = 0; r < RU; ++r) ku[r] = v4{0, 0, 0, 0};
        mmt(wk, x, ku);
        T u[RU][4];
        _Pragma("unroll") for (int rt = 0; rt < RU; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) u[rt][e] = ku[rt][e] + dc[rt][e];
        if (su) st_rows<T, NU>(z + pl.U0 + (size_t)iq * NU, live, u);
        for (int k = k0; k < k1; ++k) {
            lT* wf = wl + D::WK::N + k * (D::WA::N + D::WG::N);
            const typename D::WA wa{wf};
            const typename D::WG wb{wf + D::WA::N};
            v4 xa[RX];
            _Pragma("unroll") for (int r = 0; r < RX; ++r) xa[r] = v4{0, 0, 0, 0};
            mmt(wa, x, xa);
            mmt(wb, u, xa);
            T xj[RX][4];
            _Pragma("unroll") for (int rt = 0; rt < RX; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) xj[rt][e] = xa[rt][e];
            st_rows_c<T, NX>((T*)z_ + pl.X0 + (size_t)(1 + C * iq + k) * NX, live, xj);
        }
    };
    for (int task = blockIdx.x; task < pl.ntask; task += pl.nwg) {
        if (task < pl.ttop) {
            int t = pl.N - 1;
            while (task >= pl.tb[t] + pl.nk[t]) --t;
            const int kt = task - pl.tb[t];
            const int b0 = pl.wide[t] ? 4 * kt : kt, cnt = pl.wide[t] ? min(4, pl.nt[t] - b0) : 1;
            if (t < pl.N - 1) {
                const int c0 = C * b0, cn = min(C * cnt, pl.nt[t + 1] - c0);
                if (!wait_flags(pl.flags + pl.fb[t + 1] + c0, cn, tag, pl, s_ok)) return;
            }
            image(t, false);
            if (work) {
                if (pl.wide[t]) back_wide(t, b0, cnt);
                else back_tile(t, b0);
            }
            if (pl.fault == 1 && t == pl.N - 1 && b0 == 0) continue;  // test hook: never released
            release_flags(pl.flags + pl.fb[t] + b0, cnt, tag);
        } else if (task == pl.ttop) {
            if (!wait_flags(pl.flags + pl.fb[pl.ts], pl.nt[pl.ts], tag, pl, s_ok)) return;
            if (work) {
                for (int t = pl.ts - 1; t >= 0; --t) {
                    image(t, false);
                    for (int b = 0; b < pl.nt[t]; ++b) {
                        back_tile(t, b);
                        dma_wait();  // the stage's q rows are out before the next stage reads them
                        __syncthreads();
                    }
                }
                for (int t = 0; t < pl.ts; ++t) {
                    image(t, true);
                    if (wv < C)
                        for (int b = 0; b < pl.nt[t]; ++b) fwd_rows(t, b, wv, wv + 1, wv == 0);
                    dma_wait();  // the children's x rows are out before the next stage reads them
                    __syncthreads();
                }
            }
            release_flags(pl.flags + pl.ftop, 1, tag);
        } else {
            int t = pl.ts;
            while (task >= pl.tf[t] + pl.nk[t]) ++t;
            const int kt = task - pl.tf[t];
            const int b0 = pl.wide[t] ? 4 * kt : kt, cnt = pl.wide[t] ? min(4, pl.nt[t] - b0) : 1;
            const bool ok = t == pl.ts ? wait_flags(pl.flags + pl.ftop, 1, tag, pl, s_ok)
                                       : wait_flags(pl.flags + pl.ff[t - 1] + b0 / C, (b0 + cnt - 1) / C - b0 / C + 1, tag, pl, s_ok);
            if (!ok) return;
            image(t, true);
            if (work) {
                if (pl.wide[t]) {
                    if (wv < cnt) fwd_rows(t, b0 + wv, 0, C, true);
                } else if (wv < C) {
                    fwd_rows(t, b0, wv, wv + 1, wv == 0);
                }
            }
            release_flags(pl.flags + pl.ff[t] + b0, cnt, tag);
        }
    }
    // the last workgroup to finish advances the epoch (every workgroup has read it by then)
    __syncthreads();
    if (tid == 0) {
        const unsigned prev = atomicAdd(pl.sync + 2, 1u);
        if (prev == (unsigned)pl.nwg - 1u) {
            st_u32(pl.sync + 2, 0u);
            st_u32(pl.sync, tag);
        }
    }
}

template <class T, int NX, int NU, int C>
void launch_t(const Dy4Plan& pl, const Dev& p, const Ctl* ctl, ChkArg ck, double* z, double* q, double* d,
              const double* x0, size_t lds, hipStream_t s) {
    auto kf = k_dy4<T, NX, NU, C>;
    (void)hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kf<<<pl.nwg + (ck.on ? 1 : 0), 256, lds, s>>>(pl, p, ctl, ck, z, q, d, x0);
}
template <class T, int NX, int NU, int C>
int occ_t(size_t lds) {
    int nb = 0;
    const void* kf = (const void*)k_dy4<T, NX, NU, C>;
    (void)hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kf, 256, lds) != hipSuccess) return 0;
    return nb;
}

// f(type, nx, nu, C) for the compiled combinations: fp64 20 / 8 (C = 2, 3, 4) and 32 / 12 (C = 3);
// fp32 20 / 8 (C = 2), 32 / 12 (C = 3) and 64 / 16 (C = 4)
template <class F>
bool dispatch(bool f32, int nx, int nu, int C, F&& f) {
    if (!f32) {
        if (nx == 20 && nu == 8 && C == 2) return f(Dy4<double, 20, 8, 2>{}), true;
        if (nx == 20 && nu == 8 && C == 3) return f(Dy4<double, 20, 8, 3>{}), true;
        if (nx == 20 && nu == 8 && C == 4) return f(Dy4<double, 20, 8, 4>{}), true;
        if (nx == 32 && nu == 12 && C == 3) return f(Dy4<double, 32, 12, 3>{}), true;
        return false;
    }
    if (nx == 20 && nu == 8 && C == 2) return f(Dy4<float, 20, 8, 2>{}), true;
    if (nx == 32 && nu == 12 && C == 3) return f(Dy4<float, 32, 12, 3>{}), true;
    if (nx == 64 && nu == 16 && C == 4) return f(Dy4<float, 64, 16, 4>{}), true;
    return false;
}
}  // namespace

bool dy4_supported(bool f32, int nx, int nu, int C) {
    return dispatch(f32, nx, nu, C, [](auto) {});
}
size_t dy4_lds(bool f32, int nx, int nu, int C) {
    size_t v = 0;
    dispatch(f32, nx, nu, C, [&](auto d) { v = decltype(d)::lds(); });
    return v;
}
int dy4_occupancy(bool f32, int nx, int nu, int C, size_t lds) {
    (void)nu;
    if (!f32) {
        if (nx == 20 && C == 2) return occ_t<double, 20, 8, 2>(lds);
        if (nx == 20 && C == 3) return occ_t<double, 20, 8, 3>(lds);
        if (nx == 20 && C == 4) return occ_t<double, 20, 8, 4>(lds);
        if (nx == 32) return occ_t<double, 32, 12, 3>(lds);
        return 0;
    }
    if (nx == 20) return occ_t<float, 20, 8, 2>(lds);
    if (nx == 32) return occ_t<float, 32, 12, 3>(lds);
    if (nx == 64) return occ_t<float, 64, 16, 4>(lds);
    return 0;
}
void dy4_launch(const Dy4Plan& pl, bool f32, int nx, int nu, const Dev& p, const Ctl* ctl, ChkArg ck, double* z,
                double* q, double* d, const double* x0, size_t lds, hipStream_t s) {
    (void)nu;
    const int C = pl.C;
    if (!f32) {
        if (nx == 20 && C == 2) launch_t<double, 20, 8, 2>(pl, p, ctl, ck, z, q, d, x0, lds, s);
        else if (nx == 20 && C == 3) launch_t<double, 20, 8, 3>(pl, p, ctl, ck, z, q, d, x0, lds, s);
        else if (nx == 20 && C == 4) launch_t<double, 20, 8, 4>(pl, p, ctl, ck, z, q, d, x0, lds, s);
        else launch_t<double, 32, 12, 3>(pl, p, ctl, ck, z, q, d, x0, lds, s);
        return;
    }
    if (nx == 20) launch_t<float, 20, 8, 2>(pl, p, ctl, ck, z, q, d, x0, lds, s);
    else if (nx == 32) launch_t<float, 32, 12, 3>(pl, p, ctl, ck, z, q, d, x0, lds, s);
    else launch_t<float, 64, 16, 4>(pl, p, ctl, ck, z, q, d, x0, lds, s);
}
const char* dy4_name(bool f32, int nx, int nu) {
    (void)nu;
    if (!f32) return nx == 20 ? "k_dy4<double, 20, 8> x1" : "k_dy4<double, 32, 12> x1";
    return nx == 20 ? "k_dy4<float, 20, 8> x1" : (nx == 32 ? "k_dy4<float, 32, 12> x1" : "k_dy4<float, 64, 16> x1");
}

}  // namespace raocp
