// raocp_dynr.h — host interface of the regular-tree dynamics sweep (raocp_dynr.hip, its own
// translation unit): the plan shared by the kernel and raocp_capi.hip, the table geometry and
// the launch entry points.
#pragma once

#include "raocp_common.h"

namespace raocp {

constexpr int kDrMaxTiers = 4;   // tiers of the plan (the top is tier 0)
constexpr int kDrMaxGran = 8;    // hand-off granules one lane polls (a wait of <= 8 x block granules)
constexpr int kDrMaxStages = 32; // stages of the tree (leaf stage N < kDrMaxStages)
constexpr int kDrMaxL = 6;       // nonleaf levels of a tier's subtrees (compiled tier bodies)

// one tier: subtrees rooted at stage s0 with L nonleaf levels (stages s0 .. s0 + L - 1),
// boundary at stage s0 + L (the leaves for the deepest tier, else the next tier's roots)
struct DrTier {
    int s0, L;
    int nsub;  // subtrees (C^s0)
    int b0;    // first workgroup of the tier (the deepest tier first, the top last)
    int w0;    // first hand-off slot of the tier (one per subtree; the top's is unused)
};

// kernel argument of k_dr (passed by value)
struct DrPlan {
    int T;                    // tiers; t[0] is the top (s0 = 0, one subtree)
    DrTier t[kDrMaxTiers];
    int C;                    // branching factor (child k of node i is 1 + C i + k)
    int N;                    // leaf stage
    int nblk;                 // workgroups of the sweep (the stopping test adds one)
    int sbase[kDrMaxStages];  // first node of each stage
    int X0, U0;               // iterate offsets of x and u
    const double* bimg;       // backward tables, per nonleaf stage (dr_tb_n doubles each)
    const double* fimg;       // forward tables, per nonleaf stage (dr_tf_n doubles each)
    const double* zpage;      // 16 doubles of zeros (LDS-DMA source of padding)
    const double* x0;         // x0bar
    unsigned long long* gq;   // up hand-offs: per slot the root's q row, 2 nx granules {half, tag}
    unsigned long long* gx;   // down hand-offs: per slot the root's x row, 2 nx granules
    unsigned* sync;           // [0] epoch (the tag of the last projection), [1] error word
    long long timeout;        // per wait, 100 MHz ticks
    unsigned long long* stamps;  // diagnostics (nullptr = off): 32 slots per tier
    int fault;                // error-path test: bit 0 the deepest tier's subtree 0 never publishes
                              // (the wait times out, the call fails with RAOCP_ERR_STATE); timing
                              // only, diagnostic builds (kDiag) only: bit 2 no table DMAs, bit 3 no
                              // write-out, bit 4 no level arithmetic, bit 5 no row DMAs
};

// split-k lanes per backward output row: one per child slot, a power of two
constexpr __host__ __device__ int dr_ks(int C) { return C <= 1 ? 1 : (C == 2 ? 2 : 4); }
constexpr __host__ __device__ int dr_r64(int v) { return (v + 63) / 64 * 64; }
// lanes of a backward group (one per (row, slot)) and of a forward group (one per child x row
// and per u row), whole waves
constexpr __host__ __device__ int dr_gsb(int nx, int nu, int C) { return dr_r64((nx + nu) * dr_ks(C)); }
constexpr __host__ __device__ int dr_gsf(int nx, int nu, int C) { return dr_r64(C * nx + nu); }
// u entries per split-k lane, and the backward table row of a lane: nx WT entries, then its
// u entries of RG
constexpr __host__ __device__ int dr_up(int nu, int C) { return nu / dr_ks(C); }
constexpr __host__ __device__ int dr_neb(int nx, int nu, int C) { return nx + dr_up(nu, C); }
// live lanes of a backward group ((row, slot) pairs) and of a forward group (child x rows and
// u rows); the rest of the group's lanes hold zero rows and read nothing
constexpr __host__ __device__ int dr_lb(int nx, int nu, int C) { return (nx + nu) * dr_ks(C); }
constexpr __host__ __device__ int dr_lf(int nx, int nu, int C) { return C * nx + nu; }
// per-stage table sizes (doubles), element-pair-major over the live lanes: [pair p][lane][2]
constexpr __host__ __device__ int dr_tb_n(int nx, int nu, int C) { return dr_neb(nx, nu, C) * dr_lb(nx, nu, C); }
constexpr __host__ __device__ int dr_tf_n(int nx, int nu, int C) { return (nx + nu) * dr_lf(nx, nu, C); }
constexpr __host__ __device__ int dr_slot_n(int nx, int nu, int C) {
    return dr_tb_n(nx, nu, C) > dr_tf_n(nx, nu, C) ? dr_tb_n(nx, nu, C) : dr_tf_n(nx, nu, C);
}

// the compiled sizes (nx, nu, C)
bool dr_supported(int nx, int nu, int C);
// LDS bytes of a workgroup whose subtrees have L nonleaf levels
size_t dr_lds(int nx, int nu, int C, int L);
// workgroups of k_dr (512 lanes) resident per CU for a plan of at most lmax levels per tier
int dr_occupancy(int nx, int nu, int C, int lmax, size_t lds);
// launch (hipGetLastError() after it is the caller's)
void dr_launch(const DrPlan& pl, int nx, int nu, size_t lds, Bufs bf, int zsel, const Ctl* ctl, ChkArg ck,
               hipStream_t s);
// kernel name for raocp_kernel_info
const char* dr_name(int nx, int nu);

}  // namespace raocp
