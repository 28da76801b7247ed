// raocp_common.h — types and device helpers shared by the translation units of
// libraocp_hip.so (raocp_capi.hip with raocp_kernels.hip, raocp_dynr.hip): the CP control
// block, the rotating iterate buffers, address-space typedefs, the agent-scope hand-off
// accessors and the one-wave stopping test. Header-only (inline device functions, no
// kernels), so every translation unit may include it.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace raocp {

typedef unsigned long long u64;

struct Ctl {
    u64 red[6];          // |xi0| |xi1| |xi2| |delta0| |delta1| |delta2| maxima (bit patterns)
    double alpha;        // CP step size (alpha_1 = alpha_2, solver.py:116-118)
    int k;               // current CP iteration
    int done;            // 1 once the stopping test fired
    int final_k;
    int flags;           // bit0: NaN reached a box projection
    int max_iters;
    int pad;
    double tol;
};

// the stopping test of the previous CP iteration run by an extra workgroup of the next
// iteration's first dynamics launch (raocp_capi.hip, defer_check): on = 0 disables it
struct ChkArg {
    Ctl* ctl;
    double* hist;
    const double* part;
    int rows;
    int on;
};

// explicit address spaces: loads through these types are ds_read / global_load, never flat
typedef __attribute__((address_space(3))) double ldsd;
typedef __attribute__((address_space(1))) double glbd;
// node records for the dynamics sweep: a builtin 4-int vector (usable in any address space)
typedef int Rec __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const Rec glbrec;
typedef __attribute__((address_space(3))) Rec ldsrec;

// the rotating CP buffers: primal Z[k % 3], dual E[k % 2] (selected by the iteration counter)
struct Bufs {
    double* z0;
    double* z1;
    double* z2;
    double* e0;
    double* e1;
};

__device__ __forceinline__ glbd* pick2(const Bufs& bf, int k) { return (glbd*)((k & 1) ? bf.e1 : bf.e0); }
__device__ __forceinline__ glbd* pick3(const Bufs& bf, int k) {
    const int w = k % 3;
    return (glbd*)(w == 0 ? bf.z0 : (w == 1 ? bf.z1 : bf.z2));
}

// agent-scope relaxed accesses (global_store / global_load ... sc1): write-through stores and
// L1-bypassing loads for values another workgroup of the same launch reads (MI355X: per-XCD
// L2s are not coherent with each other)
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __longlong_as_double(
        (long long)__hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// max for the residual reductions: a NaN operand wins (fmax would drop it). The reference
// takes its inf-norms with numpy, which propagates NaN, so a NaN residual fails the
// stopping test `max(error) <= tol` there (solver.py:137-161) and must fail it here too.
__device__ __forceinline__ double nmax(double a, double b) { return (a > b || a != a) ? a : b; }

// k_cp_check by one wave (the deferred test's extra workgroup): lanes take rows, then a
// butterfly of NaN-propagating maxima; the same record, history row and decision
__device__ __forceinline__ void cp_check_wave(const ChkArg& ck) {
    Ctl* ctl = ck.ctl;
    if (ctl->done) return;
    const int lane = threadIdx.x & 63;
    double m[6] = {0, 0, 0, 0, 0, 0};
    for (int r = lane; r < ck.rows; r += 64)
        _Pragma("unroll") for (int q = 0; q < 6; ++q) m[q] = nmax(m[q], ck.part[(size_t)r * 6 + q]);
    _Pragma("unroll") for (int off = 32; off > 0; off >>= 1)
        _Pragma("unroll") for (int q = 0; q < 6; ++q) m[q] = nmax(m[q], __shfl_xor(m[q], off));
    if (lane != 0) return;
    const int k = ctl->k;
    for (int q = 0; q < 6; ++q) ck.hist[(size_t)k * 6 + q] = m[q];
    const double err = nmax(nmax(m[0], m[1]), m[2]);
    if (k >= ctl->max_iters || err <= ctl->tol || (ctl->flags & 1)) {
        ctl->done = 1;
        ctl->final_k = k;
    } else {
        ctl->k = k + 1;
    }
}

}  // namespace raocp
