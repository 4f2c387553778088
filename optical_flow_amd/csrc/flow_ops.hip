// Flow-specific HBM-bound kernels: cost volume, bilinear warp (reference convention),
// x2 flow upscale, loss image pyramid, Siamese split, photometric L1 loss.
//
// All NHWC fp32.  Each kernel cites the reference call it replaces.
#include "common.h"

namespace oflow {

// ================================================================ cost volume (K6) =====
// model.py:29-42: cv[p][i*(2d+1)+j] = sum_c f1[p][c] * f2[p + (i-d, j-d)][c], zero padded.
// One thread per output pixel of an 8 x 32 tile; channels in chunks of CC staged through LDS
// (f2 halo tile, pixel stride CC+4 floats -> conflict-free ds_read_b128).
constexpr int CT_Y = 8, CT_X = 32, CC = 16, CPS = CC + 4;

template <int D>
__global__ __launch_bounds__(256) void corr_fwd_kernel(const float* __restrict__ f1, int ld1,
                                                       const float* __restrict__ f2, int ld2,
                                                       int h, int w, int c,
                                                       float* __restrict__ out, int ldo,
                                                       int vec) {
  constexpr int ND = 2 * D + 1, NK = ND * ND;
  constexpr int HY = CT_Y + 2 * D, HX = CT_X + 2 * D;
  __shared__ float tile[HY * HX * CPS];
  const int b = blockIdx.z;
  const int y0 = blockIdx.y * CT_Y, x0 = blockIdx.x * CT_X;
  const int ty = threadIdx.x / CT_X, tx = threadIdx.x % CT_X;
  const int y = y0 + ty, x = x0 + tx;
  const bool valid = y < h && x < w;
  float acc[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) acc[k] = 0.f;
  const int64_t img = (int64_t)b * h * w;
  for (int c0 = 0; c0 < c; c0 += CC) {
    const int cc = min(CC, c - c0);
    __syncthreads();
    // stage f2 halo tile: HY*HX pixels x (CC/4) quads
    for (int q = threadIdx.x; q < HY * HX * (CC / 4); q += 256) {
      const int pix = q / (CC / 4), cq = q % (CC / 4);
      const int hy = pix / HX, hx = pix % HX;
      const int sy = y0 - D + hy, sx = x0 - D + hx;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if ((unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w && 4 * cq < cc) {
        const float* src = f2 + (img + (int64_t)sy * w + sx) * ld2 + c0 + 4 * cq;
        if (vec && 4 * cq + 4 <= cc) {
          v = *reinterpret_cast<const float4*>(src);
        } else {
          float t[4] = {0.f, 0.f, 0.f, 0.f};
          for (int e = 0; e < cc - 4 * cq; ++e) t[e] = src[e];
          v = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
      *reinterpret_cast<float4*>(&tile[pix * CPS + 4 * cq]) = v;
    }
    float a[CC];
    if (valid) {
      const float* src = f1 + (img + (int64_t)y * w + x) * ld1 + c0;
#pragma unroll
      for (int e = 0; e < CC; ++e) a[e] = e < cc ? src[e] : 0.f;
    } else {
#pragma unroll
      for (int e = 0; e < CC; ++e) a[e] = 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ND; ++i) {
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const float* t = &tile[((ty + i) * HX + tx + j) * CPS];
        float s = acc[i * ND + j];
#pragma unroll
        for (int e = 0; e < CC; e += 4) {
          const float4 v = *reinterpret_cast<const float4*>(t + e);
          s = fmaf(a[e], v.x, s);
          s = fmaf(a[e + 1], v.y, s);
          s = fmaf(a[e + 2], v.z, s);
          s = fmaf(a[e + 3], v.w, s);
        }
        acc[i * ND + j] = s;
      }
    }
  }
  if (valid) {
    float* o = out + (img + (int64_t)y * w + x) * ldo;
#pragma unroll
    for (int k = 0; k < NK; ++k) o[k] = acc[k];
  }
}

// Gradient of the cost volume w.r.t. one input (gather form, no atomics):
//   SIGN=+1 (df1): df[p][c] = sum_k dcv[p][k]       * src[p + d_k][c]     (src = f2)
//   SIGN=-1 (df2): df[q][c] = sum_k dcv[q - d_k][k] * src[q - d_k][c]     (src = f1)
template <int D, int SIGN>
__global__ __launch_bounds__(256) void corr_bwd_kernel(const float* __restrict__ dcv, int lddcv,
                                                       const float* __restrict__ src, int lds,
                                                       int h, int w, int c,
                                                       float* __restrict__ df, int lddf,
                                                       int accumulate, int vec) {
  constexpr int ND = 2 * D + 1, NK = ND * ND;
  constexpr int HY = CT_Y + 2 * D, HX = CT_X + 2 * D;
  __shared__ float tile[HY * HX * CPS];
  const int b = blockIdx.z;
  const int y0 = blockIdx.y * CT_Y, x0 = blockIdx.x * CT_X;
  const int ty = threadIdx.x / CT_X, tx = threadIdx.x % CT_X;
  const int y = y0 + ty, x = x0 + tx;
  const bool valid = y < h && x < w;
  const int64_t img = (int64_t)b * h * w;
  float coef[NK];
#pragma unroll
  for (int i = 0; i < ND; ++i) {
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int k = i * ND + j;
      float v = 0.f;
      if (valid) {
        if (SIGN > 0) {
          v = dcv[(img + (int64_t)y * w + x) * lddcv + k];
        } else {
          const int sy = y - (i - D), sx = x - (j - D);
          if ((unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w)
            v = dcv[(img + (int64_t)sy * w + sx) * lddcv + k];
        }
      }
      coef[k] = v;
    }
  }
  for (int c0 = 0; c0 < c; c0 += CC) {
    const int cc = min(CC, c - c0);
    __syncthreads();
    for (int q = threadIdx.x; q < HY * HX * (CC / 4); q += 256) {
      const int pix = q / (CC / 4), cq = q % (CC / 4);
      const int hy = pix / HX, hx = pix % HX;
      const int sy = y0 - D + hy, sx = x0 - D + hx;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if ((unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w && 4 * cq < cc) {
        const float* s = src + (img + (int64_t)sy * w + sx) * lds + c0 + 4 * cq;
        if (vec && 4 * cq + 4 <= cc) {
          v = *reinterpret_cast<const float4*>(s);
        } else {
          float t[4] = {0.f, 0.f, 0.f, 0.f};
          for (int e = 0; e < cc - 4 * cq; ++e) t[e] = s[e];
          v = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
      *reinterpret_cast<float4*>(&tile[pix * CPS + 4 * cq]) = v;
    }
    __syncthreads();
    float acc[CC];
#pragma unroll
    for (int e = 0; e < CC; ++e) acc[e] = 0.f;
#pragma unroll
    for (int i = 0; i < ND; ++i) {
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const int oy = SIGN > 0 ? i : 2 * D - i;   // tile row of src[p + SIGN*d]
        const int ox = SIGN > 0 ? j : 2 * D - j;
        const float* t = &tile[((ty + oy) * HX + tx + ox) * CPS];
        const float cf = coef[i * ND + j];
#pragma unroll
        for (int e = 0; e < CC; e += 4) {
          const float4 v = *reinterpret_cast<const float4*>(t + e);
          acc[e] = fmaf(cf, v.x, acc[e]);
          acc[e + 1] = fmaf(cf, v.y, acc[e + 1]);
          acc[e + 2] = fmaf(cf, v.z, acc[e + 2]);
          acc[e + 3] = fmaf(cf, v.w, acc[e + 3]);
        }
      }
    }
    if (valid) {
      float* o = df + (img + (int64_t)y * w + x) * lddf + c0;
      for (int e = 0; e < cc; ++e) o[e] = accumulate ? o[e] + acc[e] : acc[e];
    }
  }
}

// ===================================================================== warp (K7) =======
// transformations.py:85-129 with the grid of model.py:65-71 (P1, P2):
//   x = i + flow0 (i = ROW index), y = j + flow1 (j = COLUMN index), sampled as column x,
//   row y; x0/x1/y0/y1 clipped; weights from the clipped x1/y1 and unclipped x/y.
struct WarpTap {
  int64_t o00, o01, o10, o11;   // pixel offsets of (x0,y0),(x0,y1),(x1,y0),(x1,y1)
  float a, b;                   // a = x1c - x, b = y1c - y
  bool xsame, ysame;
};

__device__ __forceinline__ WarpTap warp_tap(int i, int j, float f0, float f1, int h, int w,
                                            int64_t img, bool absolute = false) {
  WarpTap t;
  const float x = absolute ? f0 : (float)i + f0;
  const float y = absolute ? f1 : (float)j + f1;
  const float xf = floorf(x), yf = floorf(y);
  // float->int like tf.cast (truncation of an already-floored value), then clip.
  const int xi = (int)fmaxf(fminf(xf, 2147483520.f), -2147483520.f);
  const int yi = (int)fmaxf(fminf(yf, 2147483520.f), -2147483520.f);
  const int x0 = min(max(xi, 0), w - 1), x1 = min(max(xi + 1, 0), w - 1);
  const int y0 = min(max(yi, 0), h - 1), y1 = min(max(yi + 1, 0), h - 1);
  t.a = (float)x1 - x;
  t.b = (float)y1 - y;
  t.o00 = img + (int64_t)y0 * w + x0;
  t.o01 = img + (int64_t)y1 * w + x0;
  t.o10 = img + (int64_t)y0 * w + x1;
  t.o11 = img + (int64_t)y1 * w + x1;
  t.xsame = x0 == x1;
  t.ysame = y0 == y1;
  return t;
}

// One thread per (pixel, channel quad); C % 4 == 0.
__global__ __launch_bounds__(256) void warp_fwd_vec(const float* __restrict__ inp, int n, int h,
                                                    int w, int c,
                                                    const float* __restrict__ flow,
                                                    float* __restrict__ out, int absolute) {
  const int nq = c >> 2;
  const int64_t total = (int64_t)n * h * w * nq;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = idx / nq;
    const int q = (int)(idx - p * nq);
    const int j = (int)(p % w);
    const int64_t t2 = p / w;
    const int i = (int)(t2 % h);
    const int64_t img = (t2 / h) * h * w;
    const float2 f = *reinterpret_cast<const float2*>(flow + 2 * p);
    const WarpTap t = warp_tap(i, j, f.x, f.y, h, w, img, absolute);
    const float4 v00 = *reinterpret_cast<const float4*>(inp + t.o00 * c + 4 * q);
    const float4 v01 = *reinterpret_cast<const float4*>(inp + t.o01 * c + 4 * q);
    const float4 v10 = *reinterpret_cast<const float4*>(inp + t.o10 * c + 4 * q);
    const float4 v11 = *reinterpret_cast<const float4*>(inp + t.o11 * c + 4 * q);
    const float w00 = t.a * t.b, w01 = t.a * (1.f - t.b);
    const float w10 = (1.f - t.a) * t.b, w11 = (1.f - t.a) * (1.f - t.b);
    float4 r;
    r.x = w00 * v00.x + w01 * v01.x + w10 * v10.x + w11 * v11.x;
    r.y = w00 * v00.y + w01 * v01.y + w10 * v10.y + w11 * v11.y;
    r.z = w00 * v00.z + w01 * v01.z + w10 * v10.z + w11 * v11.z;
    r.w = w00 * v00.w + w01 * v01.w + w10 * v10.w + w11 * v11.w;
    *reinterpret_cast<float4*>(out + p * c + 4 * q) = r;
  }
}

// Generic channel count: one thread per pixel.
__global__ __launch_bounds__(256) void warp_fwd_scalar(const float* __restrict__ inp, int n,
                                                       int h, int w, int c,
                                                       const float* __restrict__ flow,
                                                       float* __restrict__ out, int absolute) {
  const int64_t total = (int64_t)n * h * w;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(p % w);
    const int64_t t2 = p / w;
    const int i = (int)(t2 % h);
    const int64_t img = (t2 / h) * h * w;
    const WarpTap t = warp_tap(i, j, flow[2 * p], flow[2 * p + 1], h, w, img, absolute);
    const float w00 = t.a * t.b, w01 = t.a * (1.f - t.b);
    const float w10 = (1.f - t.a) * t.b, w11 = (1.f - t.a) * (1.f - t.b);
    for (int e = 0; e < c; ++e)
      out[p * c + e] = w00 * inp[t.o00 * c + e] + w01 * inp[t.o01 * c + e] +
                       w10 * inp[t.o10 * c + e] + w11 * inp[t.o11 * c + e];
  }
}

// Backward, one wave per pixel, lanes over channels: the four corner scatters of a wave are
// 64 consecutive floats each (256 contiguous bytes per atomic wave-instruction: the shape
// that runs at the chip-wide atomic rate), loads are coalesced rows, and d(flow) is a
// 64-lane xor-shuffle reduction.  dinp scatter with fp32 atomics (GatherNd's adjoint).
__global__ __launch_bounds__(256) void warp_bwd_wave(const float* __restrict__ dout,
                                                     const float* __restrict__ inp, int n,
                                                     int h, int w, int c,
                                                     const float* __restrict__ flow,
                                                     float* __restrict__ dinp,
                                                     float* __restrict__ dflow, int absolute) {
  const int64_t npix = (int64_t)n * h * w;
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t p = wave0; p < npix; p += nwaves) {
    const int j = (int)(p % w);
    const int64_t t2 = p / w;
    const int i = (int)(t2 % h);
    const int64_t img = (t2 / h) * h * w;
    const float2 f = *reinterpret_cast<const float2*>(flow + 2 * p);
    const WarpTap t = warp_tap(i, j, f.x, f.y, h, w, img, absolute);
    const float a = t.a, b = t.b;
    const float w00 = a * b, w01 = a * (1.f - b), w10 = (1.f - a) * b,
                w11 = (1.f - a) * (1.f - b);
    float gx = 0.f, gy = 0.f;
    for (int e = lane; e < c; e += 64) {
      const float g = dout[p * c + e];
      const float p00 = inp[t.o00 * c + e], p01 = inp[t.o01 * c + e];
      const float p10 = inp[t.o10 * c + e], p11 = inp[t.o11 * c + e];
      gx -= g * (b * (p00 - p10) + (1.f - b) * (p01 - p11));
      gy -= g * (a * (p00 - p01) + (1.f - a) * (p10 - p11));
      if (dinp) {
        atomicAdd(dinp + t.o00 * c + e, w00 * g);
        atomicAdd(dinp + t.o01 * c + e, w01 * g);
        atomicAdd(dinp + t.o10 * c + e, w10 * g);
        atomicAdd(dinp + t.o11 * c + e, w11 * g);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      gx += __shfl_xor(gx, o, 64);
      gy += __shfl_xor(gy, o, 64);
    }
    if (lane == 0) *reinterpret_cast<float2*>(dflow + 2 * p) = make_float2(gx, gy);
  }
}

__global__ __launch_bounds__(256) void warp_bwd_scalar(const float* __restrict__ dout,
                                                       const float* __restrict__ inp, int n,
                                                       int h, int w, int c,
                                                       const float* __restrict__ flow,
                                                       float* __restrict__ dinp,
                                                       float* __restrict__ dflow, int absolute) {
  const int64_t total = (int64_t)n * h * w;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(p % w);
    const int64_t t2 = p / w;
    const int i = (int)(t2 % h);
    const int64_t img = (t2 / h) * h * w;
    const WarpTap t = warp_tap(i, j, flow[2 * p], flow[2 * p + 1], h, w, img, absolute);
    const float a = t.a, b = t.b;
    float gx = 0.f, gy = 0.f;
    for (int e = 0; e < c; ++e) {
      const float g = dout[p * c + e];
      const float p00 = inp[t.o00 * c + e], p01 = inp[t.o01 * c + e];
      const float p10 = inp[t.o10 * c + e], p11 = inp[t.o11 * c + e];
      gx -= g * (b * (p00 - p10) + (1.f - b) * (p01 - p11));
      gy -= g * (a * (p00 - p01) + (1.f - a) * (p10 - p11));
      if (dinp) {
        atomicAdd(dinp + t.o00 * c + e, a * b * g);
        atomicAdd(dinp + t.o01 * c + e, a * (1.f - b) * g);
        atomicAdd(dinp + t.o10 * c + e, (1.f - a) * b * g);
        atomicAdd(dinp + t.o11 * c + e, (1.f - a) * (1.f - b) * g);
      }
    }
    dflow[2 * p] = gx;
    dflow[2 * p + 1] = gy;
  }
}

// ============================================================= upscale x2 (K8) ========
// tf.image.resize(x, 2h, 2w) * scale, half-pixel centres (model.py:76-77; P6, P7).
// Output row Y: src = 0.5*Y - 0.25 clamped at 0 -> lo = floor(src), hi = min(lo+1, h-1).
__device__ __forceinline__ void up_coord(int Y, int h, int& lo, int& hi, float& l) {
  float s = 0.5f * (float)Y - 0.25f;
  s = fmaxf(s, 0.f);
  lo = (int)s;
  hi = min(lo + 1, h - 1);
  l = s - (float)lo;
}

__global__ __launch_bounds__(256) void upscale2x_fwd_kernel(const float* __restrict__ in, int n,
                                                            int h, int w, int c, float scale,
                                                            float* __restrict__ out, int ldo) {
  const int H = 2 * h, W = 2 * w;
  const int64_t total = (int64_t)n * H * W * c;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(idx % c);
    const int64_t p = idx / c;
    const int X = (int)(p % W);
    const int64_t t2 = p / W;
    const int Y = (int)(t2 % H);
    const int64_t b = t2 / H;
    int y0, y1, x0, x1;
    float ly, lx;
    up_coord(Y, h, y0, y1, ly);
    up_coord(X, w, x0, x1, lx);
    const float* base = in + b * h * w * c + e;
    const float v00 = base[((int64_t)y0 * w + x0) * c], v01 = base[((int64_t)y0 * w + x1) * c];
    const float v10 = base[((int64_t)y1 * w + x0) * c], v11 = base[((int64_t)y1 * w + x1) * c];
    const float top = v00 + (v01 - v00) * lx;
    const float bot = v10 + (v11 - v10) * lx;
    out[p * ldo + e] = (top + (bot - top) * ly) * scale;
  }
}

// Adjoint: input row t receives from output rows Y in {2t-1, 2t, 2t+1, 2t+2} with the
// weights of up_coord (gather form, deterministic).
__device__ __forceinline__ int up_taps(int t, int h, int* Ys, float* ws) {
  int cnt = 0;
  for (int Y = max(2 * t - 1, 0); Y <= min(2 * t + 2, 2 * h - 1); ++Y) {
    int lo, hi;
    float l;
    up_coord(Y, h, lo, hi, l);
    float wgt = 0.f;
    if (lo == t) wgt += 1.f - l;
    if (hi == t) wgt += l;
    if (wgt != 0.f) {
      Ys[cnt] = Y;
      ws[cnt] = wgt;
      ++cnt;
    }
  }
  return cnt;
}

__global__ __launch_bounds__(256) void upscale2x_bwd_kernel(const float* __restrict__ dout,
                                                            int lddo, int n, int h, int w,
                                                            int c, float scale,
                                                            float* __restrict__ din, int accum) {
  const int H = 2 * h, W = 2 * w;
  const int64_t total = (int64_t)n * h * w * c;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(idx % c);
    const int64_t p = idx / c;
    const int x = (int)(p % w);
    const int64_t t2 = p / w;
    const int y = (int)(t2 % h);
    const int64_t b = t2 / h;
    int Ys[4], Xs[4];
    float wy[4], wx[4];
    const int ny = up_taps(y, h, Ys, wy);
    const int nx = up_taps(x, w, Xs, wx);
    float s = 0.f;
    for (int u = 0; u < ny; ++u) {
      float r = 0.f;
      for (int v = 0; v < nx; ++v)
        r += wx[v] * dout[((b * H + Ys[u]) * W + Xs[v]) * lddo + e];
      s += wy[u] * r;
    }
    s *= scale;
    din[idx] = accum ? din[idx] + s : s;
  }
}

// ======================================================= loss image pyramid (K11) ======
// loss.py:17-18: resize(batch, H/2^s, W/2^s); with scale f = 2^s the half-pixel source is
// f*y + (f-1)/2, i.e. rows f*y + f/2 - 1 and f*y + f/2 with weight 1/2 each (same in x).
__global__ __launch_bounds__(256) void pyramid6_kernel(const float* __restrict__ in, int n,
                                                       int H, int W, int level, float* out) {
  const int f = 1 << level;
  const int h = H / f, w = W / f;
  const int64_t total = (int64_t)n * h * w * 6;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(idx % 6);
    const int64_t p = idx / 6;
    const int x = (int)(p % w);
    const int64_t t2 = p / w;
    const int y = (int)(t2 % h);
    const int64_t b = t2 / h;
    const int y0 = f * y + f / 2 - 1, x0 = f * x + f / 2 - 1;
    const float* base = in + (b * H * W) * 6 + e;
    const float v00 = base[((int64_t)y0 * W + x0) * 6];
    const float v01 = base[((int64_t)y0 * W + x0 + 1) * 6];
    const float v10 = base[((int64_t)(y0 + 1) * W + x0) * 6];
    const float v11 = base[((int64_t)(y0 + 1) * W + x0 + 1) * 6];
    const float top = v00 + (v01 - v00) * 0.5f;
    const float bot = v10 + (v11 - v10) * 0.5f;
    out[idx] = top + (bot - top) * 0.5f;
  }
}

// Siamese split (model.py:122-123,131-132): (B,H,W,6) -> (2B,H,W,4), channel 3 zero.
__global__ __launch_bounds__(256) void split_pair_kernel(const float* __restrict__ in, int n,
                                                         int h, int w, float* __restrict__ out) {
  const int64_t npix = (int64_t)n * h * w;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix;
       p += (int64_t)gridDim.x * blockDim.x) {
    const float* s = in + p * 6;
    *reinterpret_cast<float4*>(out + p * 4) = make_float4(s[0], s[1], s[2], 0.f);
    *reinterpret_cast<float4*>(out + (npix + p) * 4) = make_float4(s[3], s[4], s[5], 0.f);
  }
}

// ================================================== photometric L1 (K12) ===============
// loss.py:26-28: |img1 - warp(img2, flow)| summed over (b,i,j,c<3); per-block partials.
constexpr int PL_THREADS = 256;
constexpr int PL_PIX_PER_BLOCK = 1024;

__device__ __forceinline__ void photo_sample(const float* img6, int64_t p, int i, int j,
                                             float f0, float f1, int h, int w, int64_t img,
                                             float* diff, WarpTap& t, float v[4][3]) {
  t = warp_tap(i, j, f0, f1, h, w, img);
  const float a = t.a, b = t.b;
  const float w00 = a * b, w01 = a * (1.f - b), w10 = (1.f - a) * b,
              w11 = (1.f - a) * (1.f - b);
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    v[0][e] = img6[t.o00 * 6 + 3 + e];
    v[1][e] = img6[t.o01 * 6 + 3 + e];
    v[2][e] = img6[t.o10 * 6 + 3 + e];
    v[3][e] = img6[t.o11 * 6 + 3 + e];
    const float warped = w00 * v[0][e] + w01 * v[1][e] + w10 * v[2][e] + w11 * v[3][e];
    diff[e] = img6[p * 6 + e] - warped;
  }
}

__global__ __launch_bounds__(PL_THREADS) void photo_l1_fwd_kernel(const float* __restrict__ img6,
                                                                  const float* __restrict__ flow,
                                                                  int n, int h, int w,
                                                                  float* __restrict__ partials) {
  const int64_t npix = (int64_t)n * h * w;
  const int64_t p0 = (int64_t)blockIdx.x * PL_PIX_PER_BLOCK;
  float s = 0.f;
  for (int k = threadIdx.x; k < PL_PIX_PER_BLOCK; k += PL_THREADS) {
    const int64_t p = p0 + k;
    if (p >= npix) break;
    const int j = (int)(p % w);
    const int64_t t2 = p / w;
    const int i = (int)(t2 % h);
    const int64_t img = (t2 / h) * h * w;
    float diff[3], v[4][3];
    WarpTap t;
    photo_sample(img6, p, i, j, flow[2 * p], flow[2 * p + 1], h, w, img, diff, t, v);
    s += fabsf(diff[0]) + fabsf(diff[1]) + fabsf(diff[2]);
  }
  // block reduction: wave shuffles then LDS
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ float red[PL_THREADS / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < PL_THREADS / 64; ++k) t += red[k];
    partials[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(256) void photo_l1_bwd_kernel(const float* __restrict__ img6,
                                                           const float* __restrict__ flow, int n,
                                                           int h, int w, float coef,
                                                           const float* __restrict__ dloss,
                                                           float* __restrict__ dflow) {
  const int64_t npix = (int64_t)n * h * w;
  if (dloss) coef *= dloss[0];
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(p % w);
    const int64_t t2 = p / w;
    const int i = (int)(t2 % h);
    const int64_t img = (t2 / h) * h * w;
    float diff[3], v[4][3];
    WarpTap t;
    photo_sample(img6, p, i, j, flow[2 * p], flow[2 * p + 1], h, w, img, diff, t, v);
    const float a = t.a, b = t.b;
    float gx = 0.f, gy = 0.f;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      // d|d|/d warped = -sign(d)  (tf Abs grad, sign(0) = 0)
      const float sg = diff[e] > 0.f ? 1.f : (diff[e] < 0.f ? -1.f : 0.f);
      const float g = -coef * sg;
      gx -= g * (b * (v[0][e] - v[2][e]) + (1.f - b) * (v[1][e] - v[3][e]));
      gy -= g * (a * (v[0][e] - v[1][e]) + (1.f - a) * (v[2][e] - v[3][e]));
    }
    dflow[2 * p] = gx;
    dflow[2 * p + 1] = gy;
  }
}

struct SumArgs {
  const float* parts[8];
  int counts[8];
  float coefs[8];
  int ngroups;
};

__global__ __launch_bounds__(256) void sum_partials_kernel(SumArgs a, float* __restrict__ out) {
  __shared__ float red[4];
  float total = 0.f;
  for (int g = 0; g < a.ngroups; ++g) {
    float s = 0.f;
    for (int k = threadIdx.x; k < a.counts[g]; k += 256) s += a.parts[g][k];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    s = red[0] + red[1] + red[2] + red[3];
    total += a.coefs[g] * s;
  }
  if (threadIdx.x == 0) out[0] = total;
}

inline int grid_for(int64_t work, int per_block = 256, int cap = 8192) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(work, per_block), cap));
}

}  // namespace oflow

using namespace oflow;

extern "C" {

int of_corr_fwd(const float* f1, int ld1, const float* f2, int ld2, int n, int h, int w, int c,
                int max_disp, float* out, int ldo, void* stream) {
  OF_CHECK_ARG(f1 && f2 && out, "corr fwd: NULL pointer");
  OF_CHECK_ARG(max_disp == 3, "corr: only max_disp=3 (the reference default) is compiled");
  OF_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0, "corr fwd: dims");
  OF_CHECK_ARG(ld1 >= c && ld2 >= c && ldo >= 49, "corr fwd: strides");
  const int vec = (ld2 % 4 == 0 && ((uintptr_t)f2 & 15) == 0) ? 1 : 0;
  dim3 grid(cdiv(w, CT_X), cdiv(h, CT_Y), n);
  hipLaunchKernelGGL(corr_fwd_kernel<3>, grid, dim3(256), 0, as_stream(stream), f1, ld1, f2, ld2,
                     h, w, c, out, ldo, vec);
  return check_launch("corr_fwd");
}

int of_corr_bwd(const float* dcv, int lddcv, const float* f1, int ld1, const float* f2, int ld2,
                int n, int h, int w, int c, int max_disp, float* df1, int lddf1, int acc1,
                float* df2, int lddf2, int acc2, void* stream) {
  OF_CHECK_ARG(dcv && f1 && f2, "corr bwd: NULL pointer");
  OF_CHECK_ARG(max_disp == 3, "corr: only max_disp=3 (the reference default) is compiled");
  OF_CHECK_ARG(ld1 >= c && ld2 >= c, "corr bwd: strides");
  const int vec1 = (ld1 % 4 == 0 && ((uintptr_t)f1 & 15) == 0) ? 1 : 0;
  const int vec2 = (ld2 % 4 == 0 && ((uintptr_t)f2 & 15) == 0) ? 1 : 0;
  dim3 grid(cdiv(w, CT_X), cdiv(h, CT_Y), n);
  hipStream_t s = as_stream(stream);
  int st;
  if (df1) {
    hipLaunchKernelGGL((corr_bwd_kernel<3, 1>), grid, dim3(256), 0, s, dcv, lddcv, f2, ld2, h, w,
                       c, df1, lddf1, acc1, vec2);
    if ((st = check_launch("corr_bwd_f1"))) return st;
  }
  if (df2) {
    hipLaunchKernelGGL((corr_bwd_kernel<3, -1>), grid, dim3(256), 0, s, dcv, lddcv, f1, ld1, h,
                       w, c, df2, lddf2, acc2, vec1);
    if ((st = check_launch("corr_bwd_f2"))) return st;
  }
  return OF_OK;
}

static int warp_fwd_impl(const float* inp, int n, int h, int w, int c, const float* flow,
                         float* out, int absolute, void* stream) {
  OF_CHECK_ARG(inp && flow && out, "warp fwd: NULL pointer");
  OF_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0, "warp fwd: dims");
  hipStream_t s = as_stream(stream);
  const int64_t npix = (int64_t)n * h * w;
  if (c % 4 == 0 && ((uintptr_t)inp & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    hipLaunchKernelGGL(warp_fwd_vec, dim3(grid_for(npix * (c / 4))), dim3(256), 0, s, inp, n, h,
                       w, c, flow, out, absolute);
  } else {
    hipLaunchKernelGGL(warp_fwd_scalar, dim3(grid_for(npix)), dim3(256), 0, s, inp, n, h, w, c,
                       flow, out, absolute);
  }
  return check_launch("warp_fwd");
}

int of_warp_fwd(const float* inp, int n, int h, int w, int c, const float* flow, float* out,
                void* stream) {
  return warp_fwd_impl(inp, n, h, w, c, flow, out, 0, stream);
}

int of_bilinear_fwd(const float* inp, int n, int h, int w, int c, const float* pts, float* out,
                    void* stream) {
  return warp_fwd_impl(inp, n, h, w, c, pts, out, 1, stream);
}

static int warp_bwd_impl(const float* dout, const float* inp, int n, int h, int w, int c,
                         const float* flow, float* dinp, float* dflow, int absolute,
                         void* stream) {
  OF_CHECK_ARG(dout && inp && flow && dflow, "warp bwd: NULL pointer");
  hipStream_t s = as_stream(stream);
  const int64_t npix = (int64_t)n * h * w;
  if (c >= 16) {
    const int g = grid_for(npix * 64, 256, 16384);
    hipLaunchKernelGGL(warp_bwd_wave, dim3(g), dim3(256), 0, s, dout, inp, n, h, w, c, flow,
                       dinp, dflow, absolute);
  } else {
    hipLaunchKernelGGL(warp_bwd_scalar, dim3(grid_for(npix)), dim3(256), 0, s, dout, inp, n, h,
                       w, c, flow, dinp, dflow, absolute);
  }
  return check_launch("warp_bwd");
}

int of_warp_bwd(const float* dout, const float* inp, int n, int h, int w, int c,
                const float* flow, float* dinp, float* dflow, void* stream) {
  return warp_bwd_impl(dout, inp, n, h, w, c, flow, dinp, dflow, 0, stream);
}

int of_bilinear_bwd(const float* dout, const float* inp, int n, int h, int w, int c,
                    const float* pts, float* dinp, float* dpts, void* stream) {
  return warp_bwd_impl(dout, inp, n, h, w, c, pts, dinp, dpts, 1, stream);
}

int of_upscale2x_fwd(const float* in, int n, int h, int w, int c, float scale, float* out,
                     int ldo, void* stream) {
  OF_CHECK_ARG(in && out && ldo >= c, "upscale fwd: args");
  const int64_t total = (int64_t)n * 4 * h * w * c;
  hipLaunchKernelGGL(upscale2x_fwd_kernel, dim3(grid_for(total)), dim3(256), 0,
                     as_stream(stream), in, n, h, w, c, scale, out, ldo);
  return check_launch("upscale2x_fwd");
}

int of_upscale2x_bwd(const float* dout, int lddo, int n, int h, int w, int c, float scale,
                     float* din, int accumulate, void* stream) {
  OF_CHECK_ARG(dout && din && lddo >= c, "upscale bwd: args");
  const int64_t total = (int64_t)n * h * w * c;
  hipLaunchKernelGGL(upscale2x_bwd_kernel, dim3(grid_for(total)), dim3(256), 0,
                     as_stream(stream), dout, lddo, n, h, w, c, scale, din, accumulate);
  return check_launch("upscale2x_bwd");
}

int of_pyramid6(const float* batch, int n, int h, int w, int levels, float* const* outs,
                void* stream) {
  OF_CHECK_ARG(batch && outs && levels >= 1 && levels <= 8, "pyramid: args");
  OF_CHECK_ARG(h % (1 << levels) == 0 && w % (1 << levels) == 0,
               "pyramid: H and W must be divisible by 2^levels (P17)");
  hipStream_t s = as_stream(stream);
  for (int l = 1; l <= levels; ++l) {
    const int64_t total = (int64_t)n * (h >> l) * (w >> l) * 6;
    hipLaunchKernelGGL(pyramid6_kernel, dim3(grid_for(total)), dim3(256), 0, s, batch, n, h, w, l,
                       outs[l - 1]);
    int st = check_launch("pyramid6");
    if (st) return st;
  }
  return OF_OK;
}

int of_split_pair(const float* batch, int n, int h, int w, float* out, void* stream) {
  OF_CHECK_ARG(batch && out && ((uintptr_t)out & 15) == 0, "split pair: args");
  hipLaunchKernelGGL(split_pair_kernel, dim3(grid_for((int64_t)n * h * w)), dim3(256), 0,
                     as_stream(stream), batch, n, h, w, out);
  return check_launch("split_pair");
}

int of_photo_l1_partials(int n, int h, int w) {
  return (int)cdiv((int64_t)n * h * w, PL_PIX_PER_BLOCK);
}

int of_photo_l1_fwd(const float* img6, const float* flow, int n, int h, int w, float* partials,
                    void* stream) {
  OF_CHECK_ARG(img6 && flow && partials, "photo l1 fwd: NULL pointer");
  const int blocks = of_photo_l1_partials(n, h, w);
  hipLaunchKernelGGL(photo_l1_fwd_kernel, dim3(blocks), dim3(PL_THREADS), 0, as_stream(stream),
                     img6, flow, n, h, w, partials);
  return check_launch("photo_l1_fwd");
}

int of_photo_l1_bwd(const float* img6, const float* flow, int n, int h, int w, float coef,
                    const float* dloss, float* dflow, void* stream) {
  OF_CHECK_ARG(img6 && flow && dflow, "photo l1 bwd: NULL pointer");
  hipLaunchKernelGGL(photo_l1_bwd_kernel, dim3(grid_for((int64_t)n * h * w)), dim3(256), 0,
                     as_stream(stream), img6, flow, n, h, w, coef, dloss, dflow);
  return check_launch("photo_l1_bwd");
}

int of_sum_partials(const float* const* parts, const int* counts, const float* coefs,
                    int ngroups, float* out, void* stream) {
  OF_CHECK_ARG(ngroups >= 1 && ngroups <= 8 && parts && counts && coefs && out,
               "sum partials: args");
  SumArgs a{};
  for (int g = 0; g < ngroups; ++g) {
    a.parts[g] = parts[g];
    a.counts[g] = counts[g];
    a.coefs[g] = coefs[g];
  }
  a.ngroups = ngroups;
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, as_stream(stream), a, out);
  return check_launch("sum_partials");
}

}  // extern "C"
