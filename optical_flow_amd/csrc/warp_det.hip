// Deterministic feature-warp backward ("a deterministic-mode flag (no atomics in
// the warp bwd)").
//
// The reference samples with four gather_nd taps (transformations.py:98-129, reached from
// warp_features, model.py:55-73); TF's gradient of a gather is a scatter-add into the feature
// map, whose adds land in whatever order the hardware retires them.  The default HIP backward
// (flow_ops.hip warp_bwd_gather) keeps that shape: per-tile sums added with float atomics, so
// two identical steps can differ in the last bit of d(features).  Here the scatter becomes a
// gather with a fixed summation order:
//
//   1. entries : every (source pixel p, corner k) -> key = destination pixel, value = (p, w_k)
//                (the clipped corners and weights of P2, computed exactly as the forward does);
//   2. sort    : a stable LSD radix sort of the 4·n·h·w entries by key (rocPRIM's device radix
//                sort): equal keys keep entry order p·4 + k;
//   3. bounds  : [begin, end) of each destination's run in the sorted array;
//   4. gather  : one thread per (destination pixel, channel quad) sums w · dout[p] over its run
//                in that order and STORES d(features) -- every element written once, so no
//                zero-fill pass and no atomics;
//   5. d(flow) : per source pixel over all channels in a fixed order (16 lanes x channel quads,
//                then a fixed DPP row reduction), plus the optional addend of of_warp_bwd_add.
//
// Bitwise reproducible run to run, in eager mode and inside a captured graph alike.  Bounded
// by HBM/L2 (the entries: 24 B per (pixel, corner) through the sort passes; the gather reads
// the dout rows of its run, mostly L2 hits for smooth flows), O(n·h·w) for any flow field --
// a field clipped onto the border only makes the runs of the border pixels long.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"

namespace oflow {

namespace {

struct DetCorners {
  int y[4], x[4];   // corner k: row y[k], column x[k]; bit 0 of k -> y1, bit 1 -> x1
  float a, b;       // a = x1c - x, b = y1c - y
};

// transformations.py:98-125 with the reference's transposed grid (model.py:65-71, P1): the
// sample of pixel (i, j) is column x = i + f0, row y = j + f1 (absolute: x = f0, y = f1).
__device__ __forceinline__ DetCorners det_corners(int i, int j, float f0, float f1, int h, int w,
                                                  bool absolute) {
  DetCorners t;
  const float x = absolute ? f0 : (float)i + f0;
  const float y = absolute ? f1 : (float)j + f1;
  const int xi = (int)fmaxf(fminf(floorf(x), 2147483520.f), -2147483520.f);
  const int yi = (int)fmaxf(fminf(floorf(y), 2147483520.f), -2147483520.f);
  const int x0 = min(max(xi, 0), w - 1), x1 = min(max(xi + 1, 0), w - 1);
  const int y0 = min(max(yi, 0), h - 1), y1 = min(max(yi + 1, 0), h - 1);
  t.a = (float)x1 - x;
  t.b = (float)y1 - y;
  t.y[0] = y0, t.y[1] = y1, t.y[2] = y0, t.y[3] = y1;
  t.x[0] = x0, t.x[1] = x0, t.x[2] = x1, t.x[3] = x1;
  return t;
}

__device__ __forceinline__ float det_row16_sum(float v) {   // over the 16 lanes of a DPP row
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x122, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x121, 0xF, 0xF, false));
  return v;
}

// 1. one thread per source pixel: its four (destination, (p, weight)) entries.
__global__ __launch_bounds__(256) void det_entries(const float* __restrict__ flow, int n, int h,
                                                   int w, int absolute,
                                                   uint32_t* __restrict__ keys,
                                                   uint64_t* __restrict__ vals) {
  const int64_t npix = (int64_t)n * h * w;
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int j = (int)(p % w);
  const int64_t t2 = p / w;
  const int i = (int)(t2 % h);
  const int64_t img = (t2 / h) * h * w;
  const float2 f = *reinterpret_cast<const float2*>(flow + 2 * p);
  const DetCorners t = det_corners(i, j, f.x, f.y, h, w, absolute != 0);
  uint4 k4;
  uint32_t* kk = reinterpret_cast<uint32_t*>(&k4);
  uint64_t v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    kk[k] = (uint32_t)(img + (int64_t)t.y[k] * w + t.x[k]);
    const float wt = ((k & 2) ? 1.f - t.a : t.a) * ((k & 1) ? 1.f - t.b : t.b);
    v[k] = (uint64_t)(uint32_t)p | ((uint64_t)__float_as_uint(wt) << 32);
  }
  *reinterpret_cast<uint4*>(keys + 4 * p) = k4;
  *reinterpret_cast<ulonglong2*>(vals + 4 * p) = make_ulonglong2(v[0], v[1]);
  *reinterpret_cast<ulonglong2*>(vals + 4 * p + 2) = make_ulonglong2(v[2], v[3]);
}

// 3. run bounds of every destination present in the sorted keys (absent ones stay [0, 0)).
__global__ __launch_bounds__(256) void det_bounds(const uint32_t* __restrict__ keys, int64_t ne,
                                                  int2* __restrict__ runs) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= ne) return;
  const uint32_t k = keys[e];
  if (e == 0 || keys[e - 1] != k) runs[k].x = (int)e;
  if (e == ne - 1 || keys[e + 1] != k) runs[k].y = (int)(e + 1);
}

// 4. d(features): one thread per (destination pixel, channel quad), the run summed in entry
// order (c % 4 == 0, 16-byte rows) ...
__global__ __launch_bounds__(256) void det_gather_vec(const float* __restrict__ dout, int64_t npix,
                                                      int c, const int2* __restrict__ runs,
                                                      const uint64_t* __restrict__ vals,
                                                      float* __restrict__ dinp) {
  const int nq = c >> 2;
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= npix * nq) return;
  const int64_t d = idx / nq;
  const int q = (int)(idx - d * nq);
  const int2 r = runs[d];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int e = r.x; e < r.y; ++e) {
    const uint64_t v = vals[e];
    const int64_t p = (int64_t)(uint32_t)v;
    const float wt = __uint_as_float((uint32_t)(v >> 32));
    const float4 g = *reinterpret_cast<const float4*>(dout + p * c + 4 * q);
    acc.x += wt * g.x;
    acc.y += wt * g.y;
    acc.z += wt * g.z;
    acc.w += wt * g.w;
  }
  *reinterpret_cast<float4*>(dinp + d * c + 4 * q) = acc;
}

// ... or per (destination pixel, channel) for any c.
__global__ __launch_bounds__(256) void det_gather_scalar(const float* __restrict__ dout,
                                                         int64_t npix, int c,
                                                         const int2* __restrict__ runs,
                                                         const uint64_t* __restrict__ vals,
                                                         float* __restrict__ dinp) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= npix * c) return;
  const int64_t d = idx / c;
  const int ch = (int)(idx - d * c);
  const int2 r = runs[d];
  float acc = 0.f;
  for (int e = r.x; e < r.y; ++e) {
    const uint64_t v = vals[e];
    acc += __uint_as_float((uint32_t)(v >> 32)) * dout[(int64_t)(uint32_t)v * c + ch];
  }
  dinp[d * c + ch] = acc;
}

// 5. d(flow) (c % 4 == 0): 16 lanes per source pixel, lane q sums channel quads q, q + 16, ...
// in order, then a fixed DPP reduction over the row -- the default kernel's per-pixel order
// for c == 64.
__global__ __launch_bounds__(256) void det_dflow_vec(const float* __restrict__ dout,
                                                     const float* __restrict__ inp, int n, int h,
                                                     int w, int c, const float* __restrict__ flow,
                                                     int absolute, float* __restrict__ dflow,
                                                     const float* __restrict__ dfa, int ldfa) {
  const int64_t npix = (int64_t)n * h * w;
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t p = gid >> 4;
  const int q = (int)(gid & 15);
  const bool ok = p < npix;
  const int64_t pp = ok ? p : npix - 1;
  const int j = (int)(pp % w);
  const int64_t t2 = pp / w;
  const int i = (int)(t2 % h);
  const int64_t img = (t2 / h) * h * w;
  const float2 f = *reinterpret_cast<const float2*>(flow + 2 * pp);
  const DetCorners t = det_corners(i, j, f.x, f.y, h, w, absolute != 0);
  const float a = t.a, bq = t.b;
  int64_t off[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) off[k] = (img + (int64_t)t.y[k] * w + t.x[k]) * c;
  auto dot = [](float4 u, float4 v) { return u.x * v.x + u.y * v.y + u.z * v.z + u.w * v.w; };
  auto sub = [](float4 u, float4 v) { return make_float4(u.x - v.x, u.y - v.y, u.z - v.z, u.w - v.w); };
  float gx = 0.f, gy = 0.f;
  for (int cq = 4 * q; cq < c; cq += 64) {
    const float4 g = *reinterpret_cast<const float4*>(dout + pp * c + cq);
    const float4 P0 = *reinterpret_cast<const float4*>(inp + off[0] + cq);
    const float4 P1 = *reinterpret_cast<const float4*>(inp + off[1] + cq);
    const float4 P2 = *reinterpret_cast<const float4*>(inp + off[2] + cq);
    const float4 P3 = *reinterpret_cast<const float4*>(inp + off[3] + cq);
    gx += -(bq * dot(g, sub(P0, P2)) + (1.f - bq) * dot(g, sub(P1, P3)));
    gy += -(a * dot(g, sub(P0, P1)) + (1.f - a) * dot(g, sub(P2, P3)));
  }
  gx = det_row16_sum(gx);
  gy = det_row16_sum(gy);
  if (q == 0 && ok) {
    if (dfa) {
      gx = dfa[p * ldfa] + gx;
      gy = dfa[p * ldfa + 1] + gy;
    }
    *reinterpret_cast<float2*>(dflow + 2 * p) = make_float2(gx, gy);
  }
}

__global__ __launch_bounds__(256) void det_dflow_scalar(const float* __restrict__ dout,
                                                        const float* __restrict__ inp, int n,
                                                        int h, int w, int c,
                                                        const float* __restrict__ flow,
                                                        int absolute, float* __restrict__ dflow,
                                                        const float* __restrict__ dfa, int ldfa) {
  const int64_t npix = (int64_t)n * h * w;
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int j = (int)(p % w);
  const int64_t t2 = p / w;
  const int i = (int)(t2 % h);
  const int64_t img = (t2 / h) * h * w;
  const DetCorners t = det_corners(i, j, flow[2 * p], flow[2 * p + 1], h, w, absolute != 0);
  const float a = t.a, bq = t.b;
  float gx = 0.f, gy = 0.f;
  for (int e = 0; e < c; ++e) {
    const float g = dout[p * c + e];
    const float p00 = inp[(img + (int64_t)t.y[0] * w + t.x[0]) * c + e];
    const float p01 = inp[(img + (int64_t)t.y[1] * w + t.x[1]) * c + e];
    const float p10 = inp[(img + (int64_t)t.y[2] * w + t.x[2]) * c + e];
    const float p11 = inp[(img + (int64_t)t.y[3] * w + t.x[3]) * c + e];
    gx -= g * (bq * (p00 - p10) + (1.f - bq) * (p01 - p11));
    gy -= g * (a * (p00 - p01) + (1.f - a) * (p10 - p11));
  }
  dflow[2 * p] = dfa ? dfa[p * ldfa] + gx : gx;
  dflow[2 * p + 1] = dfa ? dfa[p * ldfa + 1] + gy : gy;
}

// Workspace layout (256-byte aligned pieces): keys in/out (4 B per entry), values in/out
// (8 B per entry), runs (8 B per destination pixel), the sort's own scratch.
struct DetWs {
  size_t keys_in, keys_out, vals_in, vals_out, runs, sort, total, sort_bytes;
};

unsigned key_bits(int64_t npix) {
  unsigned b = 1;
  while (b < 32 && ((int64_t)1 << b) < npix) ++b;
  return b;
}

int det_layout(int64_t npix, DetWs& L) {
  const int64_t ne = 4 * npix;
  size_t sort_bytes = 0;
  const hipError_t e = rocprim::radix_sort_pairs(
      nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint64_t*)nullptr,
      (uint64_t*)nullptr, (size_t)ne, 0u, key_bits(npix), (hipStream_t)0, false);
  if (e != hipSuccess) return fail(OF_EHIP, std::string("warp bwd det: sort size query: ") +
                                                hipGetErrorString(e));
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  size_t o = 0;
  L.keys_in = o, o += al(ne * 4);
  L.keys_out = o, o += al(ne * 4);
  L.vals_in = o, o += al(ne * 8);
  L.vals_out = o, o += al(ne * 8);
  L.runs = o, o += al(npix * 8);
  L.sort = o, o += al(sort_bytes);
  L.total = o;
  L.sort_bytes = sort_bytes;
  return OF_OK;
}

}  // namespace

extern "C" {

size_t of_warp_bwd_det_workspace(int n, int h, int w, int c) {
  (void)c;
  if (n <= 0 || h <= 0 || w <= 0) return 0;
  DetWs L;
  if (det_layout((int64_t)n * h * w, L)) return 0;
  return L.total;
}

int of_warp_bwd_det(const float* dout, const float* inp, int n, int h, int w, int c,
                    const float* flow, int absolute, float* dinp, float* dflow,
                    const float* dflow_add, int ld_add, void* ws, size_t ws_bytes, void* stream) {
  OF_CHECK_ARG(dout && inp && flow && dflow, "warp bwd det: NULL pointer");
  OF_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0, "warp bwd det: dims");
  OF_CHECK_ARG(!dflow_add || ld_add >= 2, "warp bwd det: ld of the added flow gradient");
  const int64_t npix = (int64_t)n * h * w;
  OF_CHECK_ARG(4 * npix < INT32_MAX, "warp bwd det: too many pixels");
  hipStream_t s = as_stream(stream);
  const bool vec = c % 4 == 0 && ((uintptr_t)dout & 15) == 0 && ((uintptr_t)inp & 15) == 0 &&
                   (!dinp || ((uintptr_t)dinp & 15) == 0);
  if (dinp) {
    DetWs L;
    if (int st = det_layout(npix, L)) return st;
    OF_CHECK_ARG(ws && ws_bytes >= L.total, "warp bwd det: workspace too small");
    char* base = static_cast<char*>(ws);
    uint32_t* kin = reinterpret_cast<uint32_t*>(base + L.keys_in);
    uint32_t* kout = reinterpret_cast<uint32_t*>(base + L.keys_out);
    uint64_t* vin = reinterpret_cast<uint64_t*>(base + L.vals_in);
    uint64_t* vout = reinterpret_cast<uint64_t*>(base + L.vals_out);
    int2* runs = reinterpret_cast<int2*>(base + L.runs);
    const int64_t ne = 4 * npix;
    hipLaunchKernelGGL(det_entries, dim3((unsigned)cdiv(npix, 256)), dim3(256), 0, s, flow, n, h,
                       w, absolute, kin, vin);
    if (int st = check_launch("warp_bwd_det: entries")) return st;
    size_t sb = L.sort_bytes;
    const hipError_t e = rocprim::radix_sort_pairs(base + L.sort, sb, kin, kout, vin, vout,
                                                   (size_t)ne, 0u, key_bits(npix), s, false);
    if (e != hipSuccess)
      return fail(OF_EHIP, std::string("warp bwd det: sort: ") + hipGetErrorString(e));
    if (hipMemsetAsync(runs, 0, (size_t)npix * sizeof(int2), s) != hipSuccess)
      return check_launch("warp_bwd_det: runs memset");
    hipLaunchKernelGGL(det_bounds, dim3((unsigned)cdiv(ne, 256)), dim3(256), 0, s, kout, ne, runs);
    if (int st = check_launch("warp_bwd_det: bounds")) return st;
    if (vec) {
      hipLaunchKernelGGL(det_gather_vec, dim3((unsigned)cdiv(npix * (c / 4), 256)), dim3(256), 0,
                         s, dout, npix, c, runs, vout, dinp);
    } else {
      hipLaunchKernelGGL(det_gather_scalar, dim3((unsigned)cdiv(npix * c, 256)), dim3(256), 0, s,
                         dout, npix, c, runs, vout, dinp);
    }
    if (int st = check_launch("warp_bwd_det: gather")) return st;
  }
  if (vec) {
    hipLaunchKernelGGL(det_dflow_vec, dim3((unsigned)cdiv(npix * 16, 256)), dim3(256), 0, s, dout,
                       inp, n, h, w, c, flow, absolute, dflow, dflow_add, ld_add);
  } else {
    hipLaunchKernelGGL(det_dflow_scalar, dim3((unsigned)cdiv(npix, 256)), dim3(256), 0, s, dout,
                       inp, n, h, w, c, flow, absolute, dflow, dflow_add, ld_add);
  }
  return check_launch("warp_bwd_det: dflow");
}

}  // extern "C"

}  // namespace oflow
