// raocp_dyn4.h — host interface of k_dy4 (raocp_dyn4.hip, its own translation unit): the
// dynamics projection (cache.py:259-288) of the regular trees k_dy3 takes (one branching factor
// C, one class per stage, one (A, B) kind per child slot of a stage) in ONE launch: 16-parent
// tiles as dataflow tasks with per-tile flags instead of one launch per stage and direction.
#pragma once

#include "raocp_common.h"

namespace raocp {

constexpr int kDy4MaxStages = 16;

// host-built plan of one projection. Tasks, in the order every workgroup walks its share
// (task = blockIdx.x + r * nwg): the backward tiles of stages N-1 .. ts (deepest first), the
// top task (stages ts-1 .. 0 backward, then 0 .. ts-1 forward, in one workgroup), the forward
// tiles of stages ts .. N-1. A task waits only for tasks before it, so with every workgroup
// resident (the host checks the occupancy) the launch cannot deadlock.
struct Dy4Plan {
    int N, ts, C, nwg;          // stages, top stages [0, ts), branching factor, workgroups
    int same_kinds;             // every stage has the same child-slot kinds: the slot tables stay in LDS
    int i0[kDy4MaxStages + 1];  // first node of stage t (i0[N]: the first leaf)
    int nt[kDy4MaxStages];      // tiles of stage t
    int wide[kDy4MaxStages];    // stage t's tasks are 4 tiles, a wave per tile (else one tile, a wave per slot)
    int nk[kDy4MaxStages];      // tasks of stage t (per direction)
    int tb[kDy4MaxStages];      // first backward task of stage t (ts <= t < N)
    int tf[kDy4MaxStages];      // first forward task of stage t (ts <= t < N)
    int ttop, ntask;            // the top task, the task count
    int fb[kDy4MaxStages];      // first backward flag of stage t (its tiles' d and q rows are out)
    int ff[kDy4MaxStages];      // first forward flag of stage t (its tiles' children's x rows are out)
    int ftop;                   // the top's flag (the x rows of stage ts are out)
    const double* bimg;         // per-stage backward / forward table images (k_dy3_image layout)
    const double* fimg;
    int bstride, fstride;       // doubles per stage image
    int X0, U0;
    unsigned* flags;            // [nflags], tagged with the projection's epoch
    unsigned* sync;             // [0] epoch, [1] error word, [2] workgroups finished
    long long timeout;          // per wait, s_memrealtime ticks (100 MHz)
    int fault;                  // test hook (RAOCP_DY4_FAULT=1): the first deepest tile never releases its flag
};

// the compiled (type, nx, nu, branching) combinations
bool dy4_supported(bool f32, int nx, int nu, int C);
// dynamic LDS bytes of a workgroup (the larger stage image + the slot sums)
size_t dy4_lds(bool f32, int nx, int nu, int C);
// resident workgroups per CU at that LDS
int dy4_occupancy(bool f32, int nx, int nu, int C, size_t lds);
// one projection on z (the iterate), q / d: the sweep's q rows [n x nx] and d rows [m x nu],
// x0: x0bar; ck: the previous CP iteration's stopping test in an extra workgroup
void dy4_launch(const Dy4Plan& pl, bool f32, int nx, int nu, const Dev& p, const Ctl* ctl, ChkArg ck, double* z,
                double* q, double* d, const double* x0, size_t lds, hipStream_t s);
const char* dy4_name(bool f32, int nx, int nu);

}  // namespace raocp
