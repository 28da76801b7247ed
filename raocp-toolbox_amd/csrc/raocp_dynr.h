// raocp_dynr.h — host interface of the regular-tree dynamics sweep (raocp_dynr.hip, its own
// translation unit): plan structures shared by the kernels and raocp_capi.hip, and the
// launch entry points.
#pragma once

#include "raocp_common.h"

namespace raocp {

constexpr int kDrMaxTiers = 4;   // tiers of the plan (the top is tier 0)
constexpr int kDrMaxLevels = 8;  // nonleaf levels of one tier's subtrees

// one tier: subtrees rooted at stage s0 with L nonleaf levels (stages s0 .. s0 + L - 1),
// boundary at stage s0 + L (the leaves for the deepest tier, else the next tier's roots)
struct DrTier {
    int s0, L;
    int nsub;      // subtrees (C^s0)
    int bup, bdn;  // first workgroup of the tier in k_dr_up (deepest first) / k_dr_down (top first)
    int w0;        // first counter / flag word of the tier (one per subtree)
};

// kernel argument of k_dr_up / k_dr_down (passed by value)
struct DrPlan {
    int T;                   // tiers; t[0] is the top (s0 = 0, one subtree)
    DrTier t[kDrMaxTiers];
    int C;                   // branching factor (child k of node i is 1 + C i + k)
    int N;                   // leaf stage
    int nblk;                // workgroups of the sweep (k_dr_up adds one for the stopping test)
    int X0, U0;              // iterate offsets of x and u
    const double* bimg;      // backward tables, per nonleaf stage (dr_back_n doubles each)
    const double* fimg;      // forward tables, per nonleaf stage (dr_fwd_n doubles each)
    const double* zpage;     // 16 doubles of zeros (LDS-DMA source of padding)
    const double* x0;        // x0bar
    double* qbuf;            // q rows (nx each) of the tiers' roots, by node id
    double* dbuf;            // d rows (nu each) of the nonleaf nodes, by node id
    unsigned* sync;          // [0] epoch, [1] error word, [2, 2 + S) arrival counters, then S flags
    int S;                   // counter words = flag words = subtrees of all tiers
    long long timeout;       // per wait, 100 MHz ticks
    unsigned long long* stamps;  // diagnostics (nullptr = off): 64 slots per kernel, 16 per role
    int fault;               // diagnostics: 1 = the deepest tier's subtree 0 never arrives (a timeout)
};

// padded row strides (doubles): an odd number of 16-B units, so the 16-B LDS reads of lanes
// on consecutive rows spread over the banks
constexpr __host__ __device__ int dr_stride(int k) { return ((k + 1) / 2) % 2 == 0 ? (k + 1) / 2 * 2 + 2 : (k + 1) / 2 * 2; }
// split-k lanes per backward output row: one per child slot, a power of two
constexpr __host__ __device__ int dr_ks(int C) { return C <= 1 ? 1 : (C == 2 ? 2 : 4); }
// the backward level's u part: lane k of a row's split-k group takes u entries
// [k UP, (k + 1) UP), UP even; RG and u rows are zero-padded to NUP = KS UP
constexpr __host__ __device__ int dr_up(int nu, int C) { return ((nu + dr_ks(C) - 1) / dr_ks(C) + 1) / 2 * 2; }
constexpr __host__ __device__ int dr_nup(int nu, int C) { return dr_ks(C) * dr_up(nu, C); }
// per-stage table sizes (doubles): backward [R][KS][SX] WT rows, then [R][NUP] RG rows;
// forward [C][nx][SF] [Abar | B] rows, then [nu][SX] K rows
constexpr __host__ __device__ int dr_back_n(int nx, int nu, int C) {
    return (nx + nu) * dr_ks(C) * dr_stride(nx) + (nx + nu) * dr_nup(nu, C);
}
constexpr __host__ __device__ int dr_fwd_n(int nx, int nu, int C) { return C * nx * dr_stride(nx + nu) + nu * dr_stride(nx); }

// the compiled sizes (nx, nu, C)
bool dr_supported(int nx, int nu, int C);
// LDS bytes of a tier's workgroup in each kernel
size_t dr_lds_up(int nx, int nu, int C, int L, bool deepest);
size_t dr_lds_down(int nx, int nu, int C, int L);
// launches (hipGetLastError() after each is the caller's)
void dr_launch_up(const DrPlan& pl, int nx, int nu, int block, size_t lds, Bufs bf, int zsel, const Ctl* ctl,
                  ChkArg ck, hipStream_t s);
void dr_launch_down(const DrPlan& pl, int nx, int nu, int block, size_t lds, Bufs bf, int zsel, const Ctl* ctl,
                    hipStream_t s);
// kernel names for raocp_kernel_info
const char* dr_name_up(int nx, int nu);
const char* dr_name_down(int nx, int nu);

}  // namespace raocp
