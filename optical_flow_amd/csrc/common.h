// Shared helpers for liboflow (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/oflow.h"

namespace oflow {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
// Check the launch that was just issued; converts a HIP error into OF_EHIP.
int check_launch(const char* what);

// Conv launch timing (bench instrumentation), see of_timing_enable().
bool timing_on();
void timing_begin(hipStream_t s);
void timing_end(hipStream_t s, int kind, double flops);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t round_up(int64_t a, int64_t b) { return cdiv(a, b) * b; }

constexpr int kWave = 64;

// Compute units of the current device (256 on MI355X; fewer on a partitioned device), cached
// per device; 256 when no device is visible.  Grid planners size persistent grids and split-K
// targets from it, and workspace queries use the same value as the launches they size.
int device_cus();

// XCD-aware bijective block remap (cdna guide T1): the hardware deals workgroups to the 8
// XCDs round-robin; this maps them so that each XCD gets a contiguous range of work ids,
// i.e. neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Raw buffer loads (CDNA buffer resource, 32-bit byte offsets).  An offset at or past the
// resource's byte count returns 0 without a branch: padding and halo reads stay straight-line
// code, so the compiler keeps every load of a staging round in flight (a guarded pointer
// load instead becomes a branch + s_waitcnt per element).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)bytes,
                                           0x00020000);
}
__device__ __forceinline__ float4 bload4(rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}
__device__ __forceinline__ float bload1(rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0));
}
// Store counterpart: an out-of-range offset (kOOB) drops the write, no branch around it.
__device__ __forceinline__ void bstore4(float4 v, rsrc_t r, uint32_t voff) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                         r, voff, 0, 0);
}
// Channel quad at byte offset `off` with `n` valid channels (n >= 4: all), zero elsewhere;
// `ok` false -> zeros.  vec: 16-byte aligned rows and whole quads (the caller guarantees
// n <= 0 or n >= 4), one b128 and no selects on the loaded value -- a select right after
// the load would force an s_waitcnt there; else four b32, each masked by its offset.
__device__ __forceinline__ float4 bload_quad(rsrc_t r, bool ok, uint32_t off, int n, bool vec) {
  if (vec) return bload4(r, ok && n > 0 ? off : kOOB);
  return make_float4(bload1(r, ok && n > 0 ? off : kOOB), bload1(r, ok && n > 1 ? off + 4 : kOOB),
                     bload1(r, ok && n > 2 ? off + 8 : kOOB),
                     bload1(r, ok && n > 3 ? off + 12 : kOOB));
}

extern int g_warp_win;   // of_set_tuning key 7 (flow_ops.hip: warp backward form)
extern int g_corr_blk;   // of_set_tuning key 9 (flow_ops.hip: cost-volume kernel form)
extern int g_corr_ty8;   // of_set_tuning key 19 (flow_ops.hip: corr_bwd_kernel tile height)
extern int g_b16i_abl;   // of_set_tuning key 21 (conv_b16i.hip: timing ablations, wrong results)
extern int g_b16i_direct;   // of_set_tuning key 22 (conv_b16i.hip: forward direct epilogue)
extern int g_det_tpre;      // of_set_tuning key 35 (warp_det.hip: tiled mode A, d(flow) loads first)
extern int g_det_fx_grid;   // of_set_tuning key 37 (warp_det.hip: fallback grids, workgroups per CU)
extern int g_det_lds_probe;  // of_set_tuning key 38 (warp_det.hip: own_window occupancy probe)
extern int g_det_tile;      // of_set_tuning key 34 (warp_det.hip: mode A by destination tiles)
extern int g_det_rmax;      // of_set_tuning key 28 (warp_det.hip: window gather radius limit)
extern int g_b16i_persist;  // of_set_tuning key 24 (conv_b16i.hip: persistent conv_halo_b16)

}  // namespace oflow

#define OF_CHECK_ARG(cond, msg)                                   \
  do {                                                            \
    if (!(cond)) return ::oflow::fail(OF_EINVAL, (msg));          \
  } while (0)
