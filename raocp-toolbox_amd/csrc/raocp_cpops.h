// raocp_cpops.h — entry arithmetic and reductions of the fused CP tiles shared by the
// translation units raocp_cp5.hip (k_cp5, k_cp6) and raocp_dynr.hip (k_drc): the residual maxima
// with numpy's NaN propagation, the second-order-cone and box projections as selects, the
// per-workgroup residual row and the LDS forms of a row-layout vector. Header-only, anonymous
// namespace (each translation unit gets its own copies).
#pragma once

#include "raocp_tile.h"

namespace raocp {
namespace {

// One residual maximum of |terms| with numpy's NaN propagation (solver.py:137-161): fp32 by the
// NaN-propagating v_maximum3_f32 (|.| modifiers, two terms per instruction); fp64 by v_max_f64
// plus a NaN mask (v_cmp_u_f64 into a scalar lane mask), folded in at the end.
template <class T>
struct Amax;
template <>
struct Amax<float> {
    float m = 0.f;
    __device__ __forceinline__ void add(float v) { m = __builtin_elementwise_maximum(m, fabsf(v)); }
    __device__ __forceinline__ double get() const { return (double)m; }
};
#ifndef RAOCP_AMAX_BITS
template <>
struct Amax<double> {
    double m = 0.0;
    bool nan = false;
    __device__ __forceinline__ void add(double v) {
        m = __builtin_fmax(m, fabs(v));
        nan = nan || v != v;
    }
    __device__ __forceinline__ double get() const { return nan ? __builtin_nan("") : m; }
};
#else
// (RAOCP_AMAX_BITS, k_drc's unit) the maximum of |v| by the bit patterns: non-negative doubles
// order as unsigned integers, a NaN above +inf, so the unsigned maximum propagates NaN with no
// lane mask kept alive across the kernel's divergent role branches (whose joins each carried
// the six masks through scalar registers)
template <>
struct Amax<double> {
    double m = 0.0;
    __device__ __forceinline__ void add(double v) {
        const double a = fabs(v);
        m = (unsigned long long)__double_as_longlong(a) > (unsigned long long)__double_as_longlong(m) ? a : m;
    }
    __device__ __forceinline__ double get() const { return m; }
};
#endif

// the six residual maxima of a wave, and the per-entry terms (raocp_cp3.hip fin / account).
// A lane past its tile's nodes has zero operands (ldz / ld_rows) and zero box bounds, so
// every one of its terms is zero: nothing to mask.
template <class T>
struct Resid {
    Amax<T> m0, m1, m2, m3, m4, m5;
    T alpha, ra;
    // one dual element: eta+ = alpha (v - Pi(v)), xi2 = (d - eta+) / alpha + L(z+ - p)
    __device__ __forceinline__ void fin(T dv, T v, T pv, T b, T& ep, T& x2) {
        ep = alpha * (v - pv);
        x2 = (dv - ep) * ra + b;
        m2.add(x2);
        m5.add(ep - dv);
    }
    // account() in two parts (the same operations): every term but xi0, returning xi1; then
    // xi0 = xi1 + lc once L^T xi2 is known
    __device__ __forceinline__ T account_pre(T pp, T zz, T w) {
        const T x1 = (pp - zz) * ra - w;
        const T dl1 = zz - pp;
        const T dl0 = dl1 + w;
        m1.add(x1);
        m3.add(dl0);
        m4.add(dl1);
        return x1;
    }
    __device__ __forceinline__ void account_post(T x1, T lc) { m0.add(x1 + lc); }
    // one primal entry: pp = p, zz = z+, w = L^T(d - eta+), lc = L^T xi2
    __device__ __forceinline__ void account(T pp, T zz, T w, T lc) {
        const T x1 = (pp - zz) * ra - w;
        const T x0v = x1 + lc;
        const T dl1 = zz - pp;
        const T dl0 = dl1 + w;
        m0.add(x0v);
        m1.add(x1);
        m3.add(dl0);
        m4.add(dl1);
    }
};

// SecondOrderCone.project (cones.py:113-132) of one block as per-entry selects: the block is
// kept (|first| <= t), zeroed (|first| <= -t) or scaled, first * (nf + t) / (2 nf) and
// t -> (nf + t) / 2 (the reference's s * (first / nf) with the quotient s / nf taken once)
template <class T>
struct Soc {
    bool keep, zero;
    T q, s;
    __device__ __forceinline__ Soc(T nf, T t) {
        keep = nf <= t;
        zero = !keep && nf <= -t;
        s = (nf + t) / T(2);
        q = zero ? T(0) : s / nf;
    }
    __device__ __forceinline__ T first(T v) const { return keep ? v : v * q; }
    __device__ __forceinline__ T last(T t) const { return keep ? t : (zero ? T(0) : s); }
};
// Rectangle._constrain (rectangle.py:50-59) as selects; a NaN stays (the wave's flag, reported
// once per wave: the host raises ValueError)
template <class T>
__device__ __forceinline__ T box_sel(T v, T lo, T hi, bool& nan) {
    nan = nan || v != v;
    return v < lo ? lo : (v > hi ? hi : v);
}
__device__ __forceinline__ void flag_nan(Ctl* ctl, bool nan, int bit = 1) {
    if (__builtin_amdgcn_ballot_w64(nan) != 0 && (threadIdx.x & 63) == 0) atomicOr(&ctl->flags, bit);
}

// per-block residual maxima -> one row of `part` (plain stores, k_cp_check reduces). A wave's
// maxima by DPP steps within rows of 16 lanes (xor 1, xor 2, half-mirror, mirror), then the
// row broadcasts 15 and 31 (GFX9 wave64 DPP): lane 63 ends with them (NaN-propagating nmax
// throughout; the ds_bpermute butterfly it replaces cost k_cp6 ~0.7 us per workgroup)
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(v), __double2loint(v), CTRL, RM, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(v), __double2hiint(v), CTRL, RM, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_nmax(double v) {
    v = nmax(v, dpp_d<0xB1, 0xF>(v));   // lane ^ 1
    v = nmax(v, dpp_d<0x4E, 0xF>(v));   // lane ^ 2
    v = nmax(v, dpp_d<0x141, 0xF>(v));  // row half-mirror: the 8-lane maxima
    v = nmax(v, dpp_d<0x140, 0xF>(v));  // row mirror: the 16-lane maxima
    v = nmax(v, dpp_d<0x142, 0xA>(v));  // row_bcast15 into rows 1 and 3
    v = nmax(v, dpp_d<0x143, 0xC>(v));  // row_bcast31 into rows 2 and 3
    return v;
}
// the same into part[row * 6 ..] with the per-wave maxima staged in LDS scratch s_red (6 x 16)
template <class T>
__device__ __forceinline__ void block_maxima_at(double* part, int row, const Resid<T>& r,
                                                __attribute__((address_space(3))) double* s_red) {
    const double mm[6] = {wave_nmax(r.m0.get()), wave_nmax(r.m1.get()), wave_nmax(r.m2.get()),
                          wave_nmax(r.m3.get()), wave_nmax(r.m4.get()), wave_nmax(r.m5.get())};
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) _Pragma("unroll") for (int q = 0; q < 6; ++q) s_red[q * 16 + wv] = mm[q];
    // an LDS barrier: the workgroup's global stores stay in flight (__syncthreads would wait for them)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (threadIdx.x < 6) {
        double b = s_red[threadIdx.x * 16];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) b = nmax(b, s_red[threadIdx.x * 16 + w]);
        part[(size_t)row * 6 + threadIdx.x] = b;
    }
}
template <class T>
__device__ __forceinline__ void block_maxima(double* part, const Resid<T>& r) {
    __shared__ double s_red[6][16];
    const double mm[6] = {wave_nmax(r.m0.get()), wave_nmax(r.m1.get()), wave_nmax(r.m2.get()),
                          wave_nmax(r.m3.get()), wave_nmax(r.m4.get()), wave_nmax(r.m5.get())};
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) _Pragma("unroll") for (int q = 0; q < 6; ++q) s_red[q][wv] = mm[q];
    __syncthreads();
    if (threadIdx.x < 6) {
        double b = s_red[threadIdx.x][0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) b = nmax(b, s_red[threadIdx.x][w]);
        part[(size_t)blockIdx.x * 6 + threadIdx.x] = b;
    }
}

template <class T>
__device__ __forceinline__ T bcast(T v, int src) {
    return __shfl(v, src, 64);
}

// a row-layout vector (R rows) in LDS as R / 16 chunks of 4 per lane: chunk rt of lane at
// base[(rt 64 + lane) 4 ..] (16-B / 32-B lane-contiguous accesses, conflict-free)
template <class T, int R>
__device__ __forceinline__ void lds_put(__attribute__((address_space(3))) T* base, const T (&a)[(R + 15) / 16][4], bool add) {
    typedef typename V4a<T>::type vt;
    typedef __attribute__((address_space(3))) vt lvt;
    const int lane = threadIdx.x & 63;
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) {
        lvt* q = (lvt*)(base + (rt * 64 + lane) * 4);
        vt w;
        if (add) {
            w = *q;
            _Pragma("unroll") for (int e = 0; e < 4; ++e) w[e] += a[rt][e];
        } else {
            _Pragma("unroll") for (int e = 0; e < 4; ++e) w[e] = a[rt][e];
        }
        *q = w;
    }
}
template <class T, int R>
__device__ __forceinline__ void lds_get(const __attribute__((address_space(3))) T* base, T (&a)[(R + 15) / 16][4]) {
    typedef typename V4a<T>::type vt;
    typedef const __attribute__((address_space(3))) vt lvt;
    const int lane = threadIdx.x & 63;
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) {
        const vt w = *(lvt*)(base + (rt * 64 + lane) * 4);
        _Pragma("unroll") for (int e = 0; e < 4; ++e) a[rt][e] = w[e];
    }
}

// the same vector compacted: lane's R / 4 values at base[lane R / 4 ..] (no padded chunk
// slots: nx = 20 keeps 5 of the 8 values a row-layout chunk pair holds), 16-B accesses where
// R / 4 is even
template <class T, int R>
__device__ __forceinline__ void lds_putc(__attribute__((address_space(3))) T* base, const T (&a)[(R + 15) / 16][4]) {
    constexpr int KC = R / 4;
    __attribute__((address_space(3))) T* b = base + (threadIdx.x & 63) * KC;
    if constexpr (KC % 2 == 0 && sizeof(T) == 8) {
        typedef T v2 __attribute__((ext_vector_type(2)));
        _Pragma("unroll") for (int t = 0; t < KC; t += 2) *(__attribute__((address_space(3))) v2*)(b + t) = v2{a[t >> 2][t & 3], a[(t + 1) >> 2][(t + 1) & 3]};
    } else {
        _Pragma("unroll") for (int t = 0; t < KC; ++t) b[t] = a[t >> 2][t & 3];
    }
}
template <class T, int R>
__device__ __forceinline__ void lds_getc(const __attribute__((address_space(3))) T* base, T (&a)[(R + 15) / 16][4]) {
    constexpr int KC = R / 4;
    const __attribute__((address_space(3))) T* b = base + (threadIdx.x & 63) * KC;
    _Pragma("unroll") for (int rt = 0; rt < (R + 15) / 16; ++rt) _Pragma("unroll") for (int e = 0; e < 4; ++e) a[rt][e] = T(0);
    if constexpr (KC % 2 == 0 && sizeof(T) == 8) {
        typedef T v2 __attribute__((ext_vector_type(2)));
        _Pragma("unroll") for (int t = 0; t < KC; t += 2) {
            const v2 w = *(const __attribute__((address_space(3))) v2*)(b + t);
            a[t >> 2][t & 3] = w[0];
            a[(t + 1) >> 2][(t + 1) & 3] = w[1];
        }
    } else {
        _Pragma("unroll") for (int t = 0; t < KC; ++t) a[t >> 2][t & 3] = b[t];
    }
}

}  // namespace
}  // namespace raocp
