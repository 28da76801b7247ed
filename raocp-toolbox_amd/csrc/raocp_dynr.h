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
                              // write-out, bit 4 no level arithmetic, bit 5 no row DMAs; k_drc: bit 6
                              // no CP step, bit 7 no CP operand gather, bit 9 the CP step alone (no
                              // sweep, no hand-offs: the epoch does not advance)
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

// ---- k_drc: the sweep with the CP iteration of each subtree's families fused behind its forward
// sweep (one launch per CP iteration, config 2: fp64, nx = 20, nu = 8, C = 2, every tier of L = 4
// levels). Kernel argument beside the plan: the CP operands' offsets and tables.
struct DrcArg {
    int m;                    // nonleaf nodes (the first leaf)
    int Y0, T0, S0;           // primal offsets of y, tau, s (x, u: DrPlan::X0 / U0)
    int E1, E2, E3, E4, E5, E6, E7, E11, E12, E13, E14;  // dual offsets (Dev)
    const double* cond;       // conditional probabilities, child j at [j]
    const double* alpha_r;    // AVaR alpha per nonleaf node
    const double* blo_nl;     // the one box table of the nonleaf nodes [x | u] (box == 1)
    const double* bhi_nl;
    const double* blo_l;      // the one box table of the leaves (box == 1)
    const double* bhi_l;
    const double* img;        // [sqrtQ | sqrtR | sqrtPf] MFMA fragments (k_cp3_image)
    Ctl* ctl;
    double* part;             // this iteration's residual maxima: one row of 6 per sweep workgroup
    int nanbit;               // the ctl->flags bit of this iteration's NaN-in-box flag (ChkArg::nanbit)
    int box;                  // 1: every node boxed by one table per kind; 2: no boxes
};
// doubles of the CP operand region of a workgroup (raocp_dynr.hip Cpa)
constexpr int kDrcCpa = 3904;
// the weight image (DrcArg::img): [sqrtQ 640 | sqrtR 128] (kDrcWa doubles), then [sqrtPf 640 |
// lo_nl 28 | hi_nl 28 | lo_l 20 | hi_l 20] (kDrcWb)
constexpr int kDrcWa = 768, kDrcWb = 736;
// nx, nu, C, fp64 compiled for the fused form (the plan must have L = 4 in every tier)
bool drc_supported(int nx, int nu, int C);
// LDS bytes of a k_drc workgroup (tiers of 4 levels)
size_t drc_lds(int nx, int nu, int C);
// workgroups of k_drc (512 lanes) resident per CU at lds bytes
int drc_occupancy(size_t lds);
// one launch: the projection of z1 = pick3(bf, 1) in place, then the CP iteration of every family
// (p = bf.z0, eta = bf.e0 -> eta+ = bf.e1, the next half step -> bf.z2); ck: the previous
// iteration's stopping test (an extra workgroup)
// dca: the DrcArg of this launch in device memory (one per iteration parity, raocp_capi.hip)
void drc_launch(const DrPlan& pl, const DrcArg* dca, int box, size_t lds, Bufs bf, ChkArg ck, hipStream_t s);
const char* drc_name();
// this translation unit compiled with the in-kernel stamps (make DIAG=1, or a VAR_UNIT=dynr
// variant build with -DRAOCP_DIAG, tools/build_var.sh)
bool dr_diag_build();

}  // namespace raocp
