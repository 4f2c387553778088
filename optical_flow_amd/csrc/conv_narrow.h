// Narrow-convolution fast path (cout <= 4, 3x3, stride 1): see conv_narrow.hip.
#pragma once
#include "common.h"

namespace oflow {

bool narrow_ok(const of_conv_desc* d);
int narrow_fwd(const of_conv_desc* d, const float* x, int ldx, const float* w_fwd,
               const float* bias, int act, float alpha, float* y, int ldy, hipStream_t s);
int narrow_dgrad(const of_conv_desc* d, const float* dy, int lddy, const float* w_bwd,
                 const float* act_src, int ld_act, int act, float alpha, float* dx, int lddx,
                 hipStream_t s);
size_t narrow_wgrad_ws(const of_conv_desc* d);
int narrow_wgrad(const of_conv_desc* d, const float* x, int ldx, const float* dy, int lddy,
                 float* dw, float* db, int accumulate, void* ws, hipStream_t s);

}  // namespace oflow
