// raocp_tile.h — device helpers of the streaming CP tiles shared by the translation units
// raocp_cp4.hip and raocp_cp5.hip (the layout is raocp_cp3.hip's: family / leaf tiles of 16
// nodes, lane lo = node, lane group h = lane >> 4 holding rows KC h .. KC h + KC - 1 of an
// R-row vector, R = 4 KC; products in the transposed MFMA form D = W V with the weights as the
// A operand from the k_cp3_image fragments in LDS). Header-only, anonymous namespace: each
// translation unit gets its own copies.
#pragma once

#include "raocp_common.h"

namespace raocp {
namespace {

template <class U>
using glbp = __attribute__((address_space(1))) U*;
template <class U>
using cglbp = const __attribute__((address_space(1))) U*;
typedef __attribute__((address_space(3))) double lds_d;

// ---- 16x16x4 MFMA in T ----------------------------------------------------------------
template <class T>
struct MF;
template <>
struct MF<double> {
    typedef double v4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ v4 mma(double a, double b, v4 c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
};
template <>
struct MF<float> {
    typedef float v4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ v4 mma(float a, float b, v4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
};

// weight fragments of one R x K table in LDS (k_cp3_image order, raocp_cp3.hip WL):
// lds[(ro KS + s) 64 + lane]
template <class T, int R, int K>
struct WL {
    static constexpr int RO = (R / 4 + 3) / 4, KS = K / 4, N = RO * KS * 64;
    const __attribute__((address_space(3))) T* base;
    __device__ __forceinline__ T get(int ro, int s) const { return base[(ro * KS + s) * 64 + (threadIdx.x & 63)]; }
    // the same table behind an opaque base: a product through it re-reads its fragments from
    // LDS instead of keeping an earlier product's (RO KS registers) live in between
    __device__ __forceinline__ WL fresh() const {
        const __attribute__((address_space(3))) T* b = base;
        asm volatile("" : "+v"(b));
        return WL{b};
    }
};
// acc[ro] += W b (b in row layout over K)
template <class T, int R, int K>
__device__ __forceinline__ void mmt(const WL<T, R, K>& W, const T (&b)[(K + 15) / 16][4],
                                    typename MF<T>::v4 (&acc)[(R + 15) / 16]) {
    _Pragma("unroll") for (int s = 0; s < WL<T, R, K>::KS; ++s)
        _Pragma("unroll") for (int ro = 0; ro < WL<T, R, K>::RO; ++ro)
            acc[ro] = MF<T>::mma(W.get(ro, s), b[s >> 2][s & 3], acc[ro]);
}

template <class T>
struct V4a {
    typedef T type __attribute__((ext_vector_type(4), aligned(sizeof(T))));
};
// slot (rt, e) of an R-row vector holds a row (t = 4 rt + e < R / 4)
template <int R>
__device__ __forceinline__ constexpr bool tok(int rt, int e) {
    return 4 * rt + e < R / 4;
}
// row-layout load of an R-row node vector: a[rt][e] = v[R/4 h + 4 rt + e] (0 past R/4).
// v must be a valid row address even when !live: every load is issued unconditionally and
// the value selected after it -- a load under a runtime condition makes the compiler branch
// around it and wait for it on its own, one memory round trip per load
template <class T, int R>
__device__ __forceinline__ void ld_rows(cglbp<T> v, bool live, T (&a)[(R + 15) / 16][4]) {
    typedef typename V4a<T>::type vt;
    constexpr int KC = R / 4;
    cglbp<T> b = v + KC * ((threadIdx.x & 63) >> 4);
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) {
        if (4 * rt + 3 < KC) {
            const vt w = *(const __attribute__((address_space(1))) vt*)(b + 4 * rt);
            _Pragma("unroll") for (int e = 0; e < 4; ++e) a[rt][e] = live ? w[e] : T(0);
        } else {
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                T w = T(0);
                if (tok<R>(rt, e)) w = b[4 * rt + e];
                a[rt][e] = live ? w : T(0);
            }
        }
    }
}
// one scalar at a valid address, zero when !live (unconditional load, see ld_rows)
template <class T>
__device__ __forceinline__ T ldz(cglbp<T> v, bool live) {
    const T w = *v;
    return live ? w : T(0);
}
template <class T, int R>
__device__ __forceinline__ void st_rows(glbp<T> v, bool live, const T (&a)[(R + 15) / 16][4]) {
    typedef typename V4a<T>::type vt;
    constexpr int KC = R / 4;
    glbp<T> b = v + KC * ((threadIdx.x & 63) >> 4);
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) {
        if (!live) continue;
        if (4 * rt + 3 < KC) {
            vt w;
            _Pragma("unroll") for (int e = 0; e < 4; ++e) w[e] = a[rt][e];
            *(__attribute__((address_space(1))) vt*)(b + 4 * rt) = w;
        } else {
            _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<R>(rt, e)) b[4 * rt + e] = a[rt][e];
        }
    }
}
// the same from LDS rows (the box bounds of one-table trees)
template <class T, int R>
__device__ __forceinline__ void ld_rows_lds(const __attribute__((address_space(3))) T* v, T (&a)[(R + 15) / 16][4]) {
    constexpr int KC = R / 4;
    const __attribute__((address_space(3))) T* b = v + KC * ((threadIdx.x & 63) >> 4);
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt)
        _Pragma("unroll") for (int e = 0; e < 4; ++e) a[rt][e] = tok<R>(rt, e) ? b[4 * rt + e] : T(0);
}

// 32-bit element offsets from a wave-uniform base: loads and stores through el() / elw()
// address with the SGPR base and a 32-bit VGPR byte offset (global_* saddr), so no 64-bit
// per-lane pointer has to stay live across a tile loop (byte offsets below 4 GiB)
template <class T>
__device__ __forceinline__ cglbp<T> el(cglbp<T> b, unsigned o) {
    return (cglbp<T>)((const __attribute__((address_space(1))) char*)b + o * (unsigned)sizeof(T));
}
template <class T>
__device__ __forceinline__ glbp<T> elw(glbp<T> b, unsigned o) {
    return (glbp<T>)((__attribute__((address_space(1))) char*)b + o * (unsigned)sizeof(T));
}
// ld_rows / st_rows / ldz at element offset off from base
template <class T, int R>
__device__ __forceinline__ void ld_rows_o(cglbp<T> base, unsigned off, bool live, T (&a)[(R + 15) / 16][4]) {
    typedef typename V4a<T>::type vt;
    constexpr int KC = R / 4;
    const unsigned o = off + KC * ((threadIdx.x & 63) >> 4);
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) {
        if (4 * rt + 3 < KC) {
            const vt w = *(const __attribute__((address_space(1))) vt*)el(base, o + 4 * rt);
            _Pragma("unroll") for (int e = 0; e < 4; ++e) a[rt][e] = live ? w[e] : T(0);
        } else {
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                T w = T(0);
                if (tok<R>(rt, e)) w = *el(base, o + 4 * rt + e);
                a[rt][e] = live ? w : T(0);
            }
        }
    }
}
template <class T, int R>
__device__ __forceinline__ void st_rows_o(glbp<T> base, unsigned off, bool live, const T (&a)[(R + 15) / 16][4]) {
    typedef typename V4a<T>::type vt;
    constexpr int KC = R / 4;
    const unsigned o = off + KC * ((threadIdx.x & 63) >> 4);
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) {
        if (!live) continue;
        if (4 * rt + 3 < KC) {
            vt w;
            _Pragma("unroll") for (int e = 0; e < 4; ++e) w[e] = a[rt][e];
            *(__attribute__((address_space(1))) vt*)elw(base, o + 4 * rt) = w;
        } else {
            _Pragma("unroll") for (int e = 0; e < 4; ++e)
                if (tok<R>(rt, e)) *elw(base, o + 4 * rt + e) = a[rt][e];
        }
    }
}
template <class T>
__device__ __forceinline__ T ldz_o(cglbp<T> base, unsigned off, bool live) {
    const T w = *el(base, off);
    return live ? w : T(0);
}

// sum over the 4 lane groups (the rows of one node)
template <class T>
__device__ __forceinline__ T sum_h(T v) {
#ifdef RAOCP_SUMH_SHFL
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    return v;
#endif
    // lanes l ^ 16 and l ^ 32 by gfx950's row swaps (v_permlane16_swap / v_permlane32_swap: VALU
    // moves, no LDS round trip as ds_bpermute); every lane adds its own value and its partner's,
    // so the four lane groups end with the same sum, as with the shuffles
    if constexpr (sizeof(T) == 8) {
        auto sw16 = [](T x) {
            const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(x), false, false);
            const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(x), false, false);
            return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
        };
        auto sw32 = [](T x) {
            const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(x), false, false);
            const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(x), false, false);
            return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
        };
        return sw32(sw16(v));
    } else {
        const auto a = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
        const T w = __int_as_float(a[0]) + __int_as_float(a[1]);
        const auto b = __builtin_amdgcn_permlane32_swap(__float_as_int(w), __float_as_int(w), false, false);
        return __int_as_float(b[0]) + __int_as_float(b[1]);
    }
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

// per-wave scratch of the kernel projection (raocp_cp3.hip KpScratch): the family's y
// (2C + 1 <= 9) and the children's tau, s after the half step
template <class T>
struct KpScratch {
    T y[16][9];
    T tau[16][4];
    T s[16][4];
};

__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// the weight image (or a part of it) by LDS-DMA: `chunks` 16-B pieces from src to dst, every
// wave of the workgroup issuing its share (the caller waits with dma_wait + a barrier)
__device__ __forceinline__ void lds_fill(lds_d* dst, const double* src, int chunks) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int c0 = wv * 64; c0 < chunks; c0 += nw * 64) {
        const int ch = c0 + lane;
        if (ch < chunks)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) double*)(src + 2 * ch), dst + 2 * c0,
                                             16, 0, 0);
    }
}

}  // namespace
}  // namespace raocp
