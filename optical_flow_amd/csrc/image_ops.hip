// Image kernels either side of the training step (SURVEY.md §8 f):
//   row 1 -- of_preprocess_pairs: cv2.resize(INTER_LINEAR) of 8-bit BGR frames + /255 - mean
//            + pair packing into the (B, H, W, 6) float32 batch (data_reader.py:36-64);
//   row 4 -- of_flow_color / of_flow_intensity: drawing.py's HSV flow picture and intensity.
//
// All three are HBM/latency-bound elementwise passes (no contraction).  Bit-exactness with
// the CPU restatement (oracle/data_np.py) needs IEEE single ops in exactly the reference
// order, so floating-point contraction is disabled in this file, divisions and sqrtf are the
// correctly rounded ones (hipcc's default), and __fsqrt_rn is avoided: without
// OCML_BASIC_ROUNDED_OPERATIONS it is the native (1-ulp) square root.
#include "common.h"

#pragma clang fp contract(off)

namespace oflow {

// ---- cv2.resize(src, (W, H)) for CV_8UC3, INTER_LINEAR --------------------------------------
// OpenCV's generic resize (imgproc/resize.cpp, 4.x):
//   scale = 1 / ((double)dsize / ssize);  f = (float)((d + 0.5) * scale - 0.5);  s = floor(f);
//   f -= s;  weights (short) = saturate_cast<short>({1 - f, f} * 2048)  (INTER_RESIZE_COEF_SCALE).
// Horizontal (HResizeLinear): s < 0 -> s = 0, f = 0; for s + 1 >= ssize the column is the
//   border formula S[min(s, ssize-1)] * 2048; else S[s]*a0 + S[s+1]*a1 (int).
// Vertical (VResizeLinear, 128-bit universal-intrinsic path; f is NOT clamped): rows
//   clip(s, 0, h-1) and clip(s+1, 0, h-1), out = sat_u8((((S0>>4)*b0 >> 16) +
//   ((S1>>4)*b1 >> 16) + 2) >> 2).
// Special cases taken by cv::resize before the generic path: dsize == ssize copies, and an
// exact 2x downscale on both axes is INTER_AREA ((a + b + c + d + 2) >> 2).
struct Axis {
  int s0, s1;   // source indices (already clipped)
  int w0, w1;   // fixed-point weights
  bool border;  // horizontal border column: S[s0] * 2048
};

__device__ __forceinline__ float cv_coord(int d, int dsize, int ssize, int& s) {
  const double inv = (double)dsize / (double)ssize;
  const double scale = 1.0 / inv;
  float f = (float)(((double)d + 0.5) * scale - 0.5);
  s = (int)floorf(f);
  return f - (float)s;
}

__device__ __forceinline__ Axis cv_haxis(int dx, int dw, int sw) {
  int s;
  float f = cv_coord(dx, dw, sw, s);
  if (s < 0) { f = 0.f; s = 0; }
  Axis a;
  a.border = s + 1 >= sw;
  if (s >= sw - 1) { f = 0.f; s = sw - 1; }
  a.s0 = s;
  a.s1 = min(s + 1, sw - 1);
  a.w0 = __float2int_rn((1.f - f) * 2048.f);
  a.w1 = __float2int_rn(f * 2048.f);
  return a;
}

__device__ __forceinline__ Axis cv_vaxis(int dy, int dh, int sh) {
  int s;
  const float f = cv_coord(dy, dh, sh, s);
  Axis a;
  a.border = false;
  a.s0 = min(max(s, 0), sh - 1);
  a.s1 = min(max(s + 1, 0), sh - 1);
  a.w0 = __float2int_rn((1.f - f) * 2048.f);
  a.w1 = __float2int_rn(f * 2048.f);
  return a;
}

__device__ __forceinline__ int hrow(const uint8_t* row, const Axis& a, int c) {
  const int v0 = row[a.s0 * 3 + c];
  if (a.border) return v0 * 2048;
  return v0 * a.w0 + row[a.s1 * 3 + c] * a.w1;
}

__device__ __forceinline__ int mul_hi16(int a, int b) { return (a * b) >> 16; }

// data_reader.py:59-63 + :40-41: float32(u8) / 255 (float32), minus the float64 means, stored
// into the float32 batch (numpy's float64 -> float32 cast rounds to nearest).
__device__ __forceinline__ float normalise(int u8, int c) {
  const double mean = c == 0 ? 123.0 / 255.0 : c == 1 ? 117.0 / 255.0 : 104.0 / 255.0;
  const float v = __fdiv_rn((float)u8, 255.0f);
  return (float)((double)v - mean);
}

__device__ __forceinline__ void resize_pixel(const uint8_t* img, int sh, int sw, int y, int x,
                                             int oh, int ow, int out[3]) {
  if (sh == oh && sw == ow) {
    const uint8_t* p = img + ((size_t)y * sw + x) * 3;
    out[0] = p[0]; out[1] = p[1]; out[2] = p[2];
    return;
  }
  if (sw == 2 * ow && sh == 2 * oh) {  // INTER_AREA fast path (exact 2x on both axes)
    const uint8_t* p = img + ((size_t)(2 * y) * sw + 2 * x) * 3;
    const uint8_t* q = p + (size_t)sw * 3;
    for (int c = 0; c < 3; ++c) out[c] = (p[c] + p[3 + c] + q[c] + q[3 + c] + 2) >> 2;
    return;
  }
  const Axis ax = cv_haxis(x, ow, sw);
  const Axis ay = cv_vaxis(y, oh, sh);
  const uint8_t* r0 = img + (size_t)ay.s0 * sw * 3;
  const uint8_t* r1 = img + (size_t)ay.s1 * sw * 3;
  for (int c = 0; c < 3; ++c) {
    const int h0 = hrow(r0, ax, c), h1 = hrow(r1, ax, c);
    const int v = (mul_hi16(h0 >> 4, ay.w0) + mul_hi16(h1 >> 4, ay.w1) + 2) >> 2;
    out[c] = min(max(v, 0), 255);
  }
}

__global__ void __launch_bounds__(256) preprocess_pairs_kernel(const uint8_t* __restrict__ raw,
                                                               int npairs, int oh, int ow,
                                                               float* __restrict__ out) {
  const int64_t total = (int64_t)npairs * oh * ow;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % ow);
  const int y = (int)((i / ow) % oh);
  const int b = (int)(i / ((int64_t)ow * oh));
  const of_image_desc* descs = reinterpret_cast<const of_image_desc*>(raw);
  float v[6];
  for (int k = 0; k < 2; ++k) {
    const of_image_desc d = descs[2 * b + k];
    int px[3] = {0, 0, 0};
    if (d.h > 0 && d.w > 0) resize_pixel(raw + d.offset, d.h, d.w, y, x, oh, ow, px);
    for (int c = 0; c < 3; ++c) v[3 * k + c] = normalise(px[c], c);
  }
  float2* o = reinterpret_cast<float2*>(out + i * 6);
  o[0] = make_float2(v[0], v[1]);
  o[1] = make_float2(v[2], v[3]);
  o[2] = make_float2(v[4], v[5]);
}

int launch_preprocess_pairs(const void* dev_raw, int npairs, int out_h, int out_w, float* out,
                            hipStream_t s) {
  const int64_t total = (int64_t)npairs * out_h * out_w;
  if (total == 0) return OF_OK;
  const int64_t blocks = cdiv(total, 256);
  if (blocks > 0x7fffffff) return fail(OF_EINVAL, "preprocess_pairs: batch too large");
  hipLaunchKernelGGL(preprocess_pairs_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                     static_cast<const uint8_t*>(dev_raw), npairs, out_h, out_w, out);
  return check_launch("preprocess_pairs");
}

// ---- drawing.py:45-53, draw_optical_flow_color ------------------------------------------------
// cv2.cartToPolar (float32; angle by OpenCV's fastAtan32f polynomial, in radians), hue =
// angle * 180 / pi / 2 truncated to uint8, value = cv2.normalize(mag, 0, 255, NORM_MINMAX)
// truncated to uint8, saturation 255, then cv2.cvtColor(HSV2BGR) on 8 bits (HSV2RGB_b:
// h * 6/180, s and v / 255, sector table, * 255 rounded).
constexpr float kAtanP1 = 0.9997878412794807f * (float)(180 / M_PI);
constexpr float kAtanP3 = -0.3258083974640975f * (float)(180 / M_PI);
constexpr float kAtanP5 = 0.1555786518463281f * (float)(180 / M_PI);
constexpr float kAtanP7 = -0.04432655554792128f * (float)(180 / M_PI);

__device__ __forceinline__ float cv_fast_atan_deg(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float eps = (float)2.220446049250313e-16;  // (float)DBL_EPSILON
  float a, c, c2;
  if (ax >= ay) {
    c = __fdiv_rn(ay, ax + eps);
    c2 = c * c;
    a = (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
  } else {
    c = __fdiv_rn(ax, ay + eps);
    c2 = c * c;
    a = 90.f - (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

__device__ __forceinline__ float flow_mag(const float* f) {
  return sqrtf(f[0] * f[0] + f[1] * f[1]);
}

// One workgroup per image: min / max of the flow magnitude (cv2.normalize NORM_MINMAX).
__global__ void __launch_bounds__(256) flow_mag_minmax_kernel(const float* __restrict__ flow,
                                                              int64_t npix, float* __restrict__ mm) {
  const float* f = flow + (int64_t)blockIdx.x * npix * 2;
  float lo = INFINITY, hi = -INFINITY;
  for (int64_t p = threadIdx.x; p < npix; p += blockDim.x) {
    const float m = flow_mag(f + 2 * p);
    lo = fminf(lo, m);
    hi = fmaxf(hi, m);
  }
  __shared__ float slo[256], shi[256];
  slo[threadIdx.x] = lo;
  shi[threadIdx.x] = hi;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) {
      slo[threadIdx.x] = fminf(slo[threadIdx.x], slo[threadIdx.x + k]);
      shi[threadIdx.x] = fmaxf(shi[threadIdx.x], shi[threadIdx.x + k]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    mm[2 * blockIdx.x] = slo[0];
    mm[2 * blockIdx.x + 1] = shi[0];
  }
}

__device__ __forceinline__ int cv_round_u8(float v) {
  return min(max(__float2int_rn(v), 0), 255);
}

__global__ void __launch_bounds__(256) flow_color_kernel(const float* __restrict__ flow,
                                                         int64_t npix, int n,
                                                         const float* __restrict__ mm,
                                                         uint8_t* __restrict__ bgr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * n) return;
  const int img = (int)(i / npix);
  const float* f = flow + 2 * i;
  // cartToPolar: angle in radians = degrees * (float)(pi/180)
  const float ang = cv_fast_atan_deg(f[1], f[0]) * (float)(M_PI / 180.0);
  const int hue = (int)(__fdiv_rn(ang * 180.f, (float)M_PI) / 2.f);   // numpy float32, uint8 cast
  const double smin = mm[2 * img], smax = mm[2 * img + 1];
  const double scale = 255.0 * (smax - smin > 2.220446049250313e-16 ? 1.0 / (smax - smin) : 0.0);
  const double shift = 0.0 - smin * scale;
  const float val = flow_mag(f) * (float)scale + (float)shift;          // convertTo, float
  const int V = (int)fminf(fmaxf(val, 0.f), 255.f);
  // HSV2RGB_b: 8-bit H, S = 255, V -> float, sector table, back to 8 bits
  float h = (float)hue * (6.f / 180.f);
  const float s = 255.f * (1.f / 255.f), v = (float)V * (1.f / 255.f);
  float b, g, r;
  if (s == 0.f) {
    b = g = r = v;
  } else {
    while (h < 0.f) h += 6.f;
    while (h >= 6.f) h -= 6.f;
    int sector = (int)floorf(h);
    h -= (float)sector;
    if ((unsigned)sector >= 6u) { sector = 0; h = 0.f; }
    const float tab[4] = {v, v * (1.f - s), v * (1.f - s * h), v * (1.f - s * (1.f - h))};
    const int sd[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
    b = tab[sd[sector][0]];
    g = tab[sd[sector][1]];
    r = tab[sd[sector][2]];
  }
  uint8_t* o = bgr + 3 * i;
  o[0] = (uint8_t)cv_round_u8(b * 255.f);
  o[1] = (uint8_t)cv_round_u8(g * 255.f);
  o[2] = (uint8_t)cv_round_u8(r * 255.f);
}

// drawing.py:37-42 draw_optical_flow_intensity: sqrt(u^2 + u^2) / 20, min 1 (the reference
// squares channel 0 twice; kept).
__global__ void __launch_bounds__(256) flow_intensity_kernel(const float* __restrict__ flow,
                                                             int64_t total,
                                                             float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const float u = flow[2 * i];
  const float m = sqrtf(u * u + u * u);
  out[i] = fminf(__fdiv_rn(m, 20.0f), 1.0f);
}

}  // namespace oflow

using namespace oflow;

extern "C" {

int of_preprocess_pairs(const void* dev_raw, int npairs, int out_h, int out_w, float* out,
                        void* stream) {
  OF_CHECK_ARG(dev_raw && out && npairs >= 0 && out_h > 0 && out_w > 0,
               "preprocess_pairs: bad arguments");
  return launch_preprocess_pairs(dev_raw, npairs, out_h, out_w, out, as_stream(stream));
}

int of_flow_color(const float* flow, int n, int h, int w, uint8_t* bgr, float* ws, void* stream) {
  OF_CHECK_ARG(flow && bgr && ws && n > 0 && h > 0 && w > 0, "flow_color: bad arguments");
  hipStream_t s = as_stream(stream);
  const int64_t npix = (int64_t)h * w;
  hipLaunchKernelGGL(flow_mag_minmax_kernel, dim3(n), dim3(256), 0, s, flow, npix, ws);
  int rc = check_launch("flow_mag_minmax");
  if (rc != OF_OK) return rc;
  hipLaunchKernelGGL(flow_color_kernel, dim3((unsigned)cdiv(npix * n, 256)), dim3(256), 0, s, flow,
                     npix, n, ws, bgr);
  return check_launch("flow_color");
}

int of_flow_intensity(const float* flow, int64_t npix, float* out, void* stream) {
  OF_CHECK_ARG(flow && out && npix > 0, "flow_intensity: bad arguments");
  hipLaunchKernelGGL(flow_intensity_kernel, dim3((unsigned)cdiv(npix, 256)), dim3(256), 0,
                     as_stream(stream), flow, npix, out);
  return check_launch("flow_intensity");
}

}  // extern "C"
