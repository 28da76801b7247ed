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

// Diagnostic builds (make DIAG=1, -DRAOCP_DIAG) compile in the in-kernel timestamps and the
// timing-only modes that skip work (RAOCP_CP2_DBG, RAOCP_DR_FAULT bits 2-5); a release build
// folds every such test to false, so no product kernel carries a path that skips arithmetic.
#ifdef RAOCP_DIAG
constexpr bool kDiag = true;
#else
constexpr bool kDiag = false;
#endif

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

// what a batch's last stopping test publishes to pinned host memory (raocp_capi.hip h_pub):
// the control block and the hand-off sweeps' error word, read by the host after its stream
// synchronisation instead of two device-to-host copies
struct CtlPub {
    Ctl ctl;
    unsigned err;
    unsigned pad[3];
};

// the stopping test of the previous CP iteration run by an extra workgroup of the next
// iteration's first dynamics launch (raocp_capi.hip, defer_check): on = 0 disables it
struct ChkArg {
    Ctl* ctl;
    double* hist;
    const double* part;
    int rows;
    int on;
    // 0, or the ctl->flags bit that the iteration being tested raised for a NaN in a box: a CP
    // kernel that may run beside the test of the iteration before it (k_drc: the next
    // iteration's CP step is in the launch whose extra workgroup runs this test) raises bit
    // 2 << (k % 2) instead of bit 0, and the test of iteration k moves it to bit 0 (the flag
    // the host reports) only for its own k
    int nanbit;
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

// Device-side problem description (all pointers are HBM).
struct Dev {
    int n, m, nx, nu, cmax;
    int X0, U0, Y0, T0, S0, P;
    int E1, E2, E3, E4, E5, E6, E7, E11, E12, E13, E14, D;
    const int* anc;
    const int* ch_start;
    const int* nch;
    const int* rank;
    const int* yrel;     // [m] offset of y_i (and eta1_i) inside its segment
    const int* e7off;    // [m] absolute offset of eta7_i or -1
    const int* e14off;   // [n-m] absolute offset of eta14_l or -1
    // L / L^T weights, column-major: M[k*rows + r] = M_rk
    const double* SQ; const double* SR; const double* SP;
    const double* SQr; const double* SRr; const double* SPr;  // the same tables row-major
    const int* iSQ; const int* iSR; const int* iSP;
    int nSQ, nSR, nSP;   // table counts
    const double* alpha_r; const double* cond;
    const double* blo_nl; const double* bhi_nl; const double* blo_l; const double* bhi_l;
    const int* iBnl; const int* iBl;
    // dynamics projection (raocp_dyn.hip header): per child kind W = [B'; A'], per class
    // RG = [R~^-1; G] and K, per (kind, parent class) pair F = [Abar | B]; padded rows
    const double* dW; const double* dRG; const double* dKM; const double* dF;
    const double* dWT;     // per (kind, class) pair: [-Rinv B' ; A' - G B'] (one-phase backward level)
    int nkind;             // number of child kinds (rows of W)
    const double* zpage;   // 16 doubles of zeros (LDS-DMA source of padding)
    const Rec* crec;       // [n] {anc, iSQ, iSR, 0} (node 0: unused) — CP child blocks
    const Rec* frec;       // [m] {yrel, nch, ch_start, e7off} — CP family blocks (raocp_cp.hip)
    const Rec* lrec;       // [n-m] {iSP, iBl, e14off, 0} — CP leaf blocks
    const Rec* cpd_tab;    // per CP block: family {cb, ce, y0, y1}, {e7a, e7b}; leaf {e14a, e14b}
    const Rec* cp2_tab;    // per MFMA CP block (raocp_cp2.hip): family 3 records, leaf 2
    int nBnl, nBl;         // box table counts
    const Rec* ell_tab;    // [L / L^T blocks][kEllRecs] node ranges (raocp_ell.hip)
    const Rec* dblk;       // [child blocks of the CP kernels] {first parent, last parent, 0, 0}
    const Rec* ninfo;      // [m] {ch_start, nch, class, stage}
    const Rec* cinfo;      // [n] {kind, pair, anc, 0} (node 0: unused)
    const int* stage_ptr;  // [N+2] first node id of each stage (BFS numbering)
    int N;                 // last stage
    unsigned long long* stamps;  // diagnostics: s_memrealtime stamps (nullptr = off)
    int dyn_rot;           // tier kernels rotate the first wave of each staged range (always 1)
    int cp_dbg;            // diagnostics only: the workgroup / task whose stamps k_cp4 / k_cp5 / k_cp6 record
};

// The task list of a k_cp3 / k_cp4 launch (host-built, raocp_capi.hip cp3_tasks): tiles of 16
// leaves [l0, l1) when the leaves run as tasks of their own (split), then tiles of 16 parents
// from the start of each parent range [lo[r], hi[r]) (raocp_cp3.hip).
constexpr int kCp3MaxR = 36;
struct Cp3Tasks {
    int l0, l1;    // split leaf tiles (l0 == l1: none)
    int split;     // the leaf rows belong to the leaf tasks (1) or to their parents' tiles (0)
    int mL;        // first parent whose children are leaves
    int ext2;      // children's eta2 (eta+, xi2) from the buffers
    int xlo, xhi;  // parents whose xi2 of eta2 is stored
    int nr;        // parent ranges
    int lo[kCp3MaxR], hi[kCp3MaxR], t0[kCp3MaxR + 1];  // t0: first task of each range
};

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
    if (ctl->flags & ck.nanbit) ctl->flags |= 1;
    if (k >= ctl->max_iters || err <= ctl->tol || (ctl->flags & 1)) {
        ctl->done = 1;
        ctl->final_k = k;
    } else {
        ctl->k = k + 1;
    }
}

}  // namespace raocp
