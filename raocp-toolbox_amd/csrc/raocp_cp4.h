// raocp_cp4.h — host interface of k_cp4 (raocp_cp4.hip, its own translation unit): the fused
// CP iteration of raocp_cp3.hip with every operand of a tile loaded at the tile's start.
#pragma once

#include "raocp_common.h"

namespace raocp {

// the compiled (type, nx, nu, branching, box pattern) combinations
bool cp4_supported(bool f32, int nx, int nu, int C, int bx);
const char* cp4_name(bool f32, int nx, int nu);
// one launch on stream s (hipGetLastError() after it is the caller's); the task list, weight
// image and grid are k_cp3's (raocp_capi.hip)
void cp4_launch(const Dev& p, Ctl* ctl, Bufs bf, double* part, int C, int bx, const Cp3Tasks& tk, const double* img,
                int grid, int wpb, hipStream_t s);

}  // namespace raocp
