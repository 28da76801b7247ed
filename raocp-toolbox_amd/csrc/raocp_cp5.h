// raocp_cp5.h — host interface of k_cp5 (raocp_cp5.hip, its own translation unit): the fused
// CP iteration of raocp_cp3.hip as TWO streaming launches with small register files, for the
// large trees (configs 3, 4, 5): the leaf tiles, then the family tiles.
#pragma once

#include "raocp_common.h"

namespace raocp {

// the compiled (type, nx, nu, branching, box pattern) combinations; nbox_nl / nbox_l: the
// distinct box tables of the nonleaf / leaf nodes (at most one each)
bool cp5_supported(bool f32, int nx, int nu, int C, int bx, int nbox_nl, int nbox_l);
// the two kernels as rocprofv3 names them, "leaf x1 + fams x1"
const char* cp5_name(bool f32, int nx);
// k_cp5_leaf's form (RAOCP_CP5_LPF, read per context): 1 = one wave per SIMD with the next
// tile's operands in flight (register double buffering), 0 = two waves per SIMD, a tile's
// operands at its start and one L^T stream at a time; the default of the context's type
bool cp5_leaf_pf_default(bool f32);
// grids of the two launches for the eta2 tasks et (Cp3Tasks ranges of nonleaf nodes, 64 per task),
// the leaves [l0, l1) (lpf: the leaf launch's form) and the family task list tk
int cp5_leaf_grid(const Cp3Tasks& et, int l0, int l1, bool lpf);
int cp5_fam_grid(const Cp3Tasks& tk);
// rows of residual partials the two launches write (one per workgroup; the family launch's
// rows after the leaf launch's gl)
int cp5_rows(int gl, int gf);
// the two launches on stream s: the eta2 tasks et and the leaves [l0, l1) (residual partials in
// rows [0, gl) of part; gl = 0: no leaf launch, a shard's second CP launch), then the families
// of tk (the rows after them, cp5_rows); img is k_cp3's weight image ([sqrtQ | sqrtR | sqrtPf]
// fragments); lpf: the leaf launch's form. hipGetLastError() after it is the caller's.
void cp5_launch(const Dev& p, Ctl* ctl, Bufs bf, double* part, int C, int bx, const Cp3Tasks& et, int l0, int l1, int gl,
                const Cp3Tasks& tk, int gf, const double* img, bool lpf, hipStream_t s);

// k_cp6 (raocp_cp5.hip): the small trees' fused CP iteration, one family tile per workgroup of
// 2 C waves splitting the tile's roles (config 2); the task list as k_cp5_fams', the grid one
// workgroup per tile, the residual partials one row per workgroup (cp6_rows)
bool cp6_supported(bool f32, int nx, int nu, int C, int bx, int nbox_nl, int nbox_l);
const char* cp6_name();
int cp6_grid(const Cp3Tasks& tk);
// rows of residual partials a launch of `grid` workgroups writes
int cp6_rows(int grid);
void cp6_launch(const Dev& p, Ctl* ctl, Bufs bf, double* part, int bx, const Cp3Tasks& tk, int grid, const double* img,
                hipStream_t s);

}  // namespace raocp
