// Channel reductions, BN/ReLU backward, max-pool, Keras Adam, elementwise helpers.
#include "common.h"

namespace oflow {

// ------------------------------------------------------------------ column reductions --
// Block = 64 channels x 4 pixel rows; each block owns a contiguous pixel range and writes one
// partial row; a finalize pass sums partial rows in a fixed order (bitwise reproducible).
constexpr int CS_PIX_PER_BLOCK = 1024;

inline int colsum_blocks(int64_t npix) { return (int)cdiv(npix, CS_PIX_PER_BLOCK); }

__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ x,
                                                             int64_t npix, int c, int ld,
                                                             float* __restrict__ part) {
  const int cl = threadIdx.x & 63, pr = threadIdx.x >> 6;
  const int ch = blockIdx.y * 64 + cl;
  const int64_t p0 = (int64_t)blockIdx.x * CS_PIX_PER_BLOCK;
  const int64_t p1 = min(npix, p0 + CS_PIX_PER_BLOCK);
  float s = 0.f;
  if (ch < c)
    for (int64_t p = p0 + pr; p < p1; p += 4) s += x[p * ld + ch];
  __shared__ float red[4][64];
  red[pr][cl] = s;
  __syncthreads();
  if (pr == 0 && ch < c)
    part[(int64_t)blockIdx.x * c + ch] = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
}

__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part,
                                                           int nblk, int c,
                                                           float* __restrict__ out, int accum) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[(int64_t)b * c + ch];
  out[ch] = accum ? out[ch] + s : s;
}

// BN(inference)+residual+act backward: dt = dy*act'(y); dz = dt*g*invstd; dres = dt.
__global__ __launch_bounds__(256) void bn_relu_bwd_partial(
    int64_t npix, int c, int act, const float* __restrict__ dy, const float* __restrict__ y,
    const float* __restrict__ z, const float* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ var, float eps, float* __restrict__ dz, float* __restrict__ dres,
    float* __restrict__ part) {
  const int cl = threadIdx.x & 63, pr = threadIdx.x >> 6;
  const int ch = blockIdx.y * 64 + cl;
  const int64_t p0 = (int64_t)blockIdx.x * CS_PIX_PER_BLOCK;
  const int64_t p1 = min(npix, p0 + CS_PIX_PER_BLOCK);
  float sb = 0.f, sg = 0.f;
  if (ch < c) {
    const float invstd = rsqrtf(var[ch] + eps);
    const float sc = gamma[ch] * invstd;
    const float mu = mean[ch];
    for (int64_t p = p0 + pr; p < p1; p += 4) {
      const int64_t o = p * c + ch;
      const float dt = (act == OF_ACT_NONE || y[o] > 0.f) ? dy[o] : 0.f;
      dz[o] = dt * sc;
      if (dres) dres[o] = dt;
      sb += dt;
      sg += dt * (z[o] - mu) * invstd;
    }
  }
  __shared__ float red[2][4][64];
  red[0][pr][cl] = sb;
  red[1][pr][cl] = sg;
  __syncthreads();
  if (pr == 0 && ch < c) {
    part[((int64_t)blockIdx.x * 2 + 0) * c + ch] =
        red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
    part[((int64_t)blockIdx.x * 2 + 1) * c + ch] =
        red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
  }
}

__global__ __launch_bounds__(256) void bn_relu_bwd_final(const float* __restrict__ part,
                                                         int nblk, int c,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ var,
                                                         float eps, float* __restrict__ dgamma,
                                                         float* __restrict__ dbeta,
                                                         float* __restrict__ dbias, int accum) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  float sb = 0.f, sg = 0.f;
  for (int b = 0; b < nblk; ++b) {
    sb += part[((int64_t)b * 2 + 0) * c + ch];
    sg += part[((int64_t)b * 2 + 1) * c + ch];
  }
  const float db = sb * gamma[ch] * rsqrtf(var[ch] + eps);
  if (dbeta) dbeta[ch] = accum ? dbeta[ch] + sb : sb;
  if (dgamma) dgamma[ch] = accum ? dgamma[ch] + sg : sg;
  if (dbias) dbias[ch] = accum ? dbias[ch] + db : db;
}

// ------------------------------------------------------------------------- max pool ----
__global__ __launch_bounds__(256) void maxpool2_fwd_kernel(const float* __restrict__ x, int n,
                                                           int h, int w, int c,
                                                           float* __restrict__ y) {
  const int ho = h / 2, wo = w / 2, cq = c / 4;
  const int64_t total = (int64_t)n * ho * wo * cq;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(idx % cq);
    const int64_t p = idx / cq;
    const int ox = (int)(p % wo);
    const int64_t t2 = p / wo;
    const int oy = (int)(t2 % ho);
    const int64_t b = t2 / ho;
    const float* base = x + ((b * h + 2 * oy) * (int64_t)w + 2 * ox) * c + 4 * q;
    const float4 a = *reinterpret_cast<const float4*>(base);
    const float4 bb = *reinterpret_cast<const float4*>(base + c);
    const float4 cc = *reinterpret_cast<const float4*>(base + (int64_t)w * c);
    const float4 d = *reinterpret_cast<const float4*>(base + (int64_t)w * c + c);
    float4 r;
    r.x = fmaxf(fmaxf(a.x, bb.x), fmaxf(cc.x, d.x));
    r.y = fmaxf(fmaxf(a.y, bb.y), fmaxf(cc.y, d.y));
    r.z = fmaxf(fmaxf(a.z, bb.z), fmaxf(cc.z, d.z));
    r.w = fmaxf(fmaxf(a.w, bb.w), fmaxf(cc.w, d.w));
    *reinterpret_cast<float4*>(y + p * c + 4 * q) = r;
  }
}

// Gradient to the first maximum of each window in row-major order (torch / TF CPU argmax).
__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ dy, int n,
                                                           int h, int w, int c,
                                                           float* __restrict__ dx) {
  const int ho = h / 2, wo = w / 2;
  const int64_t total = (int64_t)n * ho * wo * c;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(idx % c);
    const int64_t p = idx / c;
    const int ox = (int)(p % wo);
    const int64_t t2 = p / wo;
    const int oy = (int)(t2 % ho);
    const int64_t b = t2 / ho;
    const int64_t o0 = ((b * h + 2 * oy) * (int64_t)w + 2 * ox) * c + e;
    const int64_t offs[4] = {o0, o0 + c, o0 + (int64_t)w * c, o0 + (int64_t)w * c + c};
    int best = 0;
    float bv = x[offs[0]];
    for (int k = 1; k < 4; ++k) {
      const float v = x[offs[k]];
      if (v > bv) {
        bv = v;
        best = k;
      }
    }
    const float g = dy[idx];
    for (int k = 0; k < 4; ++k) dx[offs[k]] = (k == best) ? g : 0.f;
  }
}

// ---------------------------------------------------------------------- Keras Adam -----
// ResourceApplyAdam (train.py:34,56): m += (g-m)(1-b1); v += (g^2-v)(1-b2);
// p -= lr_t*m/(sqrt(v)+eps), lr_t = lr*sqrt(1-b2^t)/(1-b1^t) computed on the host.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n, float lr_t, float b1, float b2,
                                                   float eps, float gs) {
  const int64_t nq = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (int64_t i = tid; i < nq; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    gg.x *= gs; gg.y *= gs; gg.z *= gs; gg.w *= gs;
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
#define OF_ADAM1(c)                                  \
  mm.c += (gg.c - mm.c) * (1.f - b1);                \
  vv.c += (gg.c * gg.c - vv.c) * (1.f - b2);         \
  pp.c -= lr_t * mm.c / (sqrtf(vv.c) + eps);
    OF_ADAM1(x) OF_ADAM1(y) OF_ADAM1(z) OF_ADAM1(w)
#undef OF_ADAM1
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  for (int64_t i = 4 * nq + tid; i < n; i += stride) {
    const float gi = g[i] * gs;
    m[i] += (gi - m[i]) * (1.f - b1);
    v[i] += (gi * gi - v[i]) * (1.f - b2);
    p[i] -= lr_t * m[i] / (sqrtf(v[i]) + eps);
  }
}

// ---------------------------------------------------------------------- elementwise ----
__global__ __launch_bounds__(256) void add_kernel(float* __restrict__ y,
                                                  const float* __restrict__ x, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] += x[i];
}

__global__ __launch_bounds__(256) void fill_kernel(float* __restrict__ y, float v, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = v;
}

__global__ __launch_bounds__(256) void copy_strided_kernel(const float* __restrict__ src,
                                                           int lds, float* __restrict__ dst,
                                                           int ldd, int64_t npix, int c) {
  const int64_t total = npix * c;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / c;
    const int e = (int)(i - p * c);
    dst[p * ldd + e] = src[p * lds + e];
  }
}

__global__ __launch_bounds__(256) void copy_strided_vec(const float* __restrict__ src, int lds,
                                                        float* __restrict__ dst, int ldd,
                                                        int64_t npix, int c) {
  const int cq = c / 4;
  const int64_t total = npix * cq;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / cq;
    const int q = (int)(i - p * cq);
    *reinterpret_cast<float4*>(dst + p * ldd + 4 * q) =
        *reinterpret_cast<const float4*>(src + p * lds + 4 * q);
  }
}

__global__ __launch_bounds__(256) void act_bwd_kernel(const float* __restrict__ dy,
                                                      const float* __restrict__ y, int act,
                                                      float alpha, float* __restrict__ dz,
                                                      int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float s = y[i] > 0.f ? 1.f : (act == OF_ACT_LEAKY ? alpha : 0.f);
    dz[i] = act == OF_ACT_NONE ? dy[i] : dy[i] * s;
  }
}

inline int grid_of(int64_t work) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(work, 256), 8192));
}

}  // namespace oflow

using namespace oflow;

extern "C" {

size_t of_colsum_workspace(int64_t npix, int c) {
  return (size_t)colsum_blocks(npix) * c * sizeof(float);
}

int of_colsum(const float* x, int64_t npix, int c, int ld, float* out, int accumulate,
              void* workspace, void* stream) {
  OF_CHECK_ARG(x && out && workspace && ld >= c && c > 0, "colsum: args");
  hipStream_t s = as_stream(stream);
  const int nblk = colsum_blocks(npix);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(nblk, cdiv(c, 64)), dim3(256), 0, s, x, npix,
                     c, ld, part);
  int st = check_launch("colsum_partial");
  if (st) return st;
  hipLaunchKernelGGL(colsum_final_kernel, dim3(cdiv(c, 256)), dim3(256), 0, s, part, nblk, c,
                     out, accumulate);
  return check_launch("colsum_final");
}

size_t of_bn_act_bwd_workspace(int64_t npix, int c) {
  return (size_t)colsum_blocks(npix) * 2 * c * sizeof(float);
}

int of_bn_act_bwd(int64_t npix, int c, int act, const float* dy, const float* y,
                  const float* z, const float* gamma, const float* mean, const float* var,
                  float eps, float* dz, float* dres, float* dgamma, float* dbeta, float* dbias,
                  int accumulate, void* workspace, void* stream) {
  OF_CHECK_ARG(dy && y && z && gamma && mean && var && dz && workspace, "bn_act_bwd: args");
  OF_CHECK_ARG(act == OF_ACT_NONE || act == OF_ACT_RELU, "bn_act_bwd: act must be none/relu");
  hipStream_t s = as_stream(stream);
  const int nblk = colsum_blocks(npix);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(bn_relu_bwd_partial, dim3(nblk, cdiv(c, 64)), dim3(256), 0, s, npix, c, act,
                     dy, y, z, gamma, mean, var, eps, dz, dres, part);
  int st = check_launch("bn_relu_bwd_partial");
  if (st) return st;
  hipLaunchKernelGGL(bn_relu_bwd_final, dim3(cdiv(c, 256)), dim3(256), 0, s, part, nblk, c,
                     gamma, var, eps, dgamma, dbeta, dbias, accumulate);
  return check_launch("bn_relu_bwd_final");
}

int of_maxpool2_fwd(const float* x, int n, int h, int w, int c, float* y, void* stream) {
  OF_CHECK_ARG(x && y && h % 2 == 0 && w % 2 == 0 && c % 4 == 0, "maxpool fwd: args");
  const int64_t total = (int64_t)n * (h / 2) * (w / 2) * (c / 4);
  hipLaunchKernelGGL(maxpool2_fwd_kernel, dim3(grid_of(total)), dim3(256), 0, as_stream(stream),
                     x, n, h, w, c, y);
  return check_launch("maxpool2_fwd");
}

int of_maxpool2_bwd(const float* x, const float* dy, int n, int h, int w, int c, float* dx,
                    void* stream) {
  OF_CHECK_ARG(x && dy && dx && h % 2 == 0 && w % 2 == 0, "maxpool bwd: args");
  const int64_t total = (int64_t)n * (h / 2) * (w / 2) * c;
  hipLaunchKernelGGL(maxpool2_bwd_kernel, dim3(grid_of(total)), dim3(256), 0, as_stream(stream),
                     x, dy, n, h, w, c, dx);
  return check_launch("maxpool2_bwd");
}

int of_adam_keras(float* p, const float* g, float* m, float* v, int64_t n, float lr_t,
                  float beta1, float beta2, float eps, float gscale, void* stream) {
  OF_CHECK_ARG(p && g && m && v && n >= 0, "adam: args");
  OF_CHECK_ARG((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0,
               "adam: arenas must be 16-byte aligned");
  if (n == 0) return OF_OK;
  hipLaunchKernelGGL(adam_kernel, dim3(std::min<int64_t>(grid_of(n / 4 + 1), 2048)), dim3(256),
                     0, as_stream(stream), p, g, m, v, n, lr_t, beta1, beta2, eps, gscale);
  return check_launch("adam");
}

int of_act_bwd(const float* dy, const float* y, int act, float alpha, float* dz, int64_t n,
               void* stream) {
  OF_CHECK_ARG(dy && y && dz, "act bwd: args");
  if (n == 0) return OF_OK;
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_of(n)), dim3(256), 0, as_stream(stream), dy, y,
                     act, alpha, dz, n);
  return check_launch("act_bwd");
}

int of_add_inplace(float* y, const float* x, int64_t n, void* stream) {
  OF_CHECK_ARG(y && x, "add: args");
  if (n == 0) return OF_OK;
  hipLaunchKernelGGL(add_kernel, dim3(grid_of(n)), dim3(256), 0, as_stream(stream), y, x, n);
  return check_launch("add");
}

int of_fill(float* y, float v, int64_t n, void* stream) {
  OF_CHECK_ARG(y, "fill: args");
  if (n == 0) return OF_OK;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_of(n)), dim3(256), 0, as_stream(stream), y, v, n);
  return check_launch("fill");
}

int of_copy_strided(const float* src, int lds, float* dst, int ldd, int64_t npix, int c,
                    void* stream) {
  OF_CHECK_ARG(src && dst && lds >= c && ldd >= c, "copy strided: args");
  if (npix == 0) return OF_OK;
  hipStream_t s = as_stream(stream);
  if (c % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0)
    hipLaunchKernelGGL(copy_strided_vec, dim3(grid_of(npix * c / 4)), dim3(256), 0, s, src, lds,
                       dst, ldd, npix, c);
  else
    hipLaunchKernelGGL(copy_strided_kernel, dim3(grid_of(npix * c)), dim3(256), 0, s, src, lds,
                       dst, ldd, npix, c);
  return check_launch("copy_strided");
}

}  // extern "C"
