// Narrow convolutions: cout <= 4, stride 1 -- the 2-channel flow layers of every flow module
// (model.py:113-114, Conv2D(2, 3, padding='same')).  With N = 2 an MFMA tile is 16x
// wasted and the GEMM path is bound by its per-tile overheads; these VALU kernels are
// instead bound by one pass over the activations:
//   forward : lanes (pixel, channel quad) gather a float4 per tap, multiply by the 4x4 weight
//             block held in LDS, reduce over the quads of the pixel with lane shuffles;
//   dgrad   : lanes (pixel, channel quad) gather dy (4 channels, broadcast within the pixel)
//             per tap and write the input gradient, times the producer activation's
//             derivative (same epilogue contract as of_conv2d_dgrad);
//   wgrad   : per (tap, pixel slice) blocks accumulate the 4x4 (ci, co) products of their
//             pixels in registers, reduce in LDS, and a second kernel sums the slices in a
//             fixed order (deterministic) into the HWIO gradient and the bias gradient.
// Weights come from the same packed buffers as the GEMM path (of_conv_pack_*).
#include "common.h"
#include "conv_narrow.h"

namespace oflow {

struct NarrowArgs {
  const float* x;
  int ldx;
  const float* dy;
  int lddy;
  const float* wt;       // fwd: packed W_f [taps*cin_p][4]; dgrad: packed W_d [taps*4][cin_p]
  const float* bias;
  float* out;
  int ldo;
  const float* act_src;  // dgrad epilogue
  int ld_act;
  int act;
  float alpha;
  int n, h, w, cin, cin_p, cout, kh, kw, pt, pl, ho, wo;
  int lg;                // log2(cin_p / 4): lanes per pixel = 1 << lg
  int nslice;            // wgrad pixel slices
  float* part;           // wgrad partials [taps][nslice][cin_p * 4 + 4]
  float* dw;
  float* db;
  int accumulate;
};

constexpr int NARROW_MAX_W = 64 * 64;   // taps * cin_p float4 rows held in LDS (64 KB)

__device__ __forceinline__ float4 fma4(float s, const float4& v, const float4& acc) {
  return make_float4(fmaf(s, v.x, acc.x), fmaf(s, v.y, acc.y), fmaf(s, v.z, acc.z),
                     fmaf(s, v.w, acc.w));
}

__device__ __forceinline__ float lane_sum(float v, int lg) {
  for (int m = 1; m < (1 << lg); m <<= 1) v += __shfl_xor(v, m);
  return v;
}

constexpr int NK3 = 9;                  // 3x3 kernels only (the flow layers)

__global__ __launch_bounds__(256, 2) void narrow_fwd_kernel(NarrowArgs a) {
  extern __shared__ float4 wl[];          // [taps * cin_p] rows of 4 output channels
  constexpr int taps = NK3;
  for (int i = threadIdx.x; i < taps * a.cin_p; i += 256)
    wl[i] = reinterpret_cast<const float4*>(a.wt)[i];
  __syncthreads();
  const int L = 1 << a.lg, q = threadIdx.x & (L - 1);
  const int64_t npix = (int64_t)a.n * a.ho * a.wo;
  const int64_t p = (int64_t)blockIdx.x * (256 >> a.lg) + (threadIdx.x >> a.lg);
  const bool valid = p < npix;
  const int64_t pc = valid ? p : 0;
  const int b = (int)(pc / ((int64_t)a.ho * a.wo));
  const int rem = (int)(pc - (int64_t)b * a.ho * a.wo);
  const int oy = rem / a.wo, ox = rem - oy * a.wo;
  const rsrc_t rx = make_rsrc(a.x + (int64_t)b * a.h * a.w * a.ldx, (int64_t)a.h * a.w * a.ldx * 4);
  float4 xv[taps];
#pragma unroll
  for (int t = 0; t < taps; ++t) {
    const int r = t / 3, s = t % 3;
    const int iy = oy + r - a.pt, ix = ox + s - a.pl;
    const bool ok = valid && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
    xv[t] = bload4(rx, ok ? 4u * ((iy * a.w + ix) * a.ldx + 4 * q) : kOOB);
  }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int t = 0; t < taps; ++t) {
    const float4* wr = &wl[t * a.cin_p + 4 * q];
    acc = fma4(xv[t].x, wr[0], acc);
    acc = fma4(xv[t].y, wr[1], acc);
    acc = fma4(xv[t].z, wr[2], acc);
    acc = fma4(xv[t].w, wr[3], acc);
  }
  const float o[4] = {lane_sum(acc.x, a.lg), lane_sum(acc.y, a.lg), lane_sum(acc.z, a.lg),
                      lane_sum(acc.w, a.lg)};
  if (valid) {                           // lane q writes output channels q, q + L, ...
#pragma unroll
    for (int co = 0; co < 4; ++co) {
      if (co < a.cout && (co & (L - 1)) == q) {
        float v = o[co];
        if (a.bias) v += a.bias[co];
        if (a.act == OF_ACT_RELU) v = v > 0.f ? v : 0.f;
        if (a.act == OF_ACT_LEAKY) v = v > 0.f ? v : a.alpha * v;
        a.out[p * a.ldo + co] = v;
      }
    }
  }
}

__global__ __launch_bounds__(256) void narrow_dgrad_kernel(NarrowArgs a) {
  extern __shared__ float4 wl[];          // [taps * 4 (co)][cin_p / 4] quads of input channels
  constexpr int taps = NK3;
  const int nq = a.cin_p / 4;
  for (int i = threadIdx.x; i < taps * 4 * nq; i += 256)
    wl[i] = reinterpret_cast<const float4*>(a.wt)[i];
  __syncthreads();
  const int L = 1 << a.lg, q = threadIdx.x & (L - 1);
  const int64_t npix = (int64_t)a.n * a.h * a.w;
  const int64_t p = (int64_t)blockIdx.x * (256 >> a.lg) + (threadIdx.x >> a.lg);
  const bool valid = p < npix;
  const int64_t pc = valid ? p : 0;
  const int b = (int)(pc / ((int64_t)a.h * a.w));
  const int rem = (int)(pc - (int64_t)b * a.h * a.w);
  const int iy = rem / a.w, ix = rem - iy * a.w;
  const rsrc_t rd =
      make_rsrc(a.dy + (int64_t)b * a.ho * a.wo * a.lddy, (int64_t)a.ho * a.wo * a.lddy * 4);
  float4 dv[taps];
#pragma unroll
  for (int t = 0; t < taps; ++t) {
    const int r = t / 3, s = t % 3;
    const int oy = iy - r + a.pt, ox = ix - s + a.pl;
    const bool ok = valid && (unsigned)oy < (unsigned)a.ho && (unsigned)ox < (unsigned)a.wo;
    dv[t] = bload4(rd, ok ? 4u * ((oy * a.wo + ox) * a.lddy) : kOOB);
  }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int t = 0; t < taps; ++t) {
    const float4* wr = &wl[(t * 4) * nq + q];
    acc = fma4(dv[t].x, wr[0], acc);
    acc = fma4(dv[t].y, wr[nq], acc);
    acc = fma4(dv[t].z, wr[2 * nq], acc);
    acc = fma4(dv[t].w, wr[3 * nq], acc);
  }
  if (!valid) return;
  if (a.act_src) {
    const float4 s = *reinterpret_cast<const float4*>(a.act_src + p * a.ld_act + 4 * q);
    const float neg = a.act == OF_ACT_LEAKY ? a.alpha : 0.f;
    acc.x *= s.x > 0.f ? 1.f : neg;
    acc.y *= s.y > 0.f ? 1.f : neg;
    acc.z *= s.z > 0.f ? 1.f : neg;
    acc.w *= s.w > 0.f ? 1.f : neg;
  }
  *reinterpret_cast<float4*>(a.out + p * a.ldo + 4 * q) = acc;
}

// grid (taps, nslice): partial[tap][slice][ci][co] (+ [4] bias sums on tap 0).
__global__ __launch_bounds__(256) void narrow_wgrad_kernel(NarrowArgs a) {
  __shared__ float red[256 * 16 + 256 * 4];
  const int tap = blockIdx.x, slice = blockIdx.y;
  const int r = tap / a.kw, s = tap - r * a.kw;
  const int L = 1 << a.lg, q = threadIdx.x & (L - 1), slot = threadIdx.x >> a.lg;
  const int P = 256 >> a.lg;
  const int64_t npix = (int64_t)a.n * a.ho * a.wo;
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  float4 bacc = make_float4(0.f, 0.f, 0.f, 0.f);
  const rsrc_t rx = make_rsrc(a.x, (int64_t)a.n * a.h * a.w * a.ldx * 4);
  const rsrc_t rd = make_rsrc(a.dy, npix * a.lddy * 4);
  const int hw = a.ho * a.wo;
  // 4 pixels per iteration, loads issued together (OOB offsets instead of branches).
  constexpr int U = 4;
  for (int p0 = slice * P + slot; p0 < (int)npix; p0 += U * a.nslice * P) {
    float4 xv[U], dv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + u * a.nslice * P;
      const bool pok = p < (int)npix;
      const int pp = pok ? p : 0;
      const int b = pp / hw;
      const int rem = pp - b * hw;
      const int oy = rem / a.wo, ox = rem - oy * a.wo;
      const int iy = oy + r - a.pt, ix = ox + s - a.pl;
      const bool ok = pok && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
      xv[u] = bload4(rx, ok ? 4u * (uint32_t)(((b * a.h + iy) * a.w + ix) * a.ldx + 4 * q) : kOOB);
      dv[u] = bload4(rd, pok ? 4u * (uint32_t)(pp * a.lddy) : kOOB);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float xs[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
      const float ds[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w};
#pragma unroll
      for (int ci = 0; ci < 4; ++ci)
#pragma unroll
        for (int co = 0; co < 4; ++co) acc[ci * 4 + co] = fmaf(xs[ci], ds[co], acc[ci * 4 + co]);
      bacc.x += dv[u].x;
      bacc.y += dv[u].y;
      bacc.z += dv[u].z;
      bacc.w += dv[u].w;
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) red[threadIdx.x * 16 + i] = acc[i];
  float* bred = red + 256 * 16;
  bred[threadIdx.x * 4 + 0] = bacc.x;
  bred[threadIdx.x * 4 + 1] = bacc.y;
  bred[threadIdx.x * 4 + 2] = bacc.z;
  bred[threadIdx.x * 4 + 3] = bacc.w;
  __syncthreads();
  const int row = a.cin_p * 4 + 4;
  float* dst = a.part + ((int64_t)tap * a.nslice + slice) * row;
  // element e < cin_p*4: (quad qq = e / 16, i = e % 16) summed over the P pixel slots
  for (int e = threadIdx.x; e < a.cin_p * 4; e += 256) {
    const int qq = e >> 4, i = e & 15;
    float sum = 0.f;
    for (int sl = 0; sl < P; ++sl) sum += red[((sl << a.lg) + qq) * 16 + i];
    dst[e] = sum;                         // = [ci = 4 qq + i/4][co = i%4]
  }
  if (threadIdx.x < 4) {
    float sum = 0.f;
    for (int sl = 0; sl < P; ++sl) sum += bred[(sl << a.lg) * 4 + threadIdx.x];   // quad 0
    dst[a.cin_p * 4 + threadIdx.x] = sum;
  }
}

__global__ __launch_bounds__(256) void narrow_wgrad_final_kernel(NarrowArgs a) {
  const int taps = a.kh * a.kw, row = a.cin_p * 4 + 4;
  const int total = taps * a.cin * a.cout + a.cout;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    float sum = 0.f;
    float* dst;
    if (e < taps * a.cin * a.cout) {
      const int t = e / (a.cin * a.cout), rem = e - t * a.cin * a.cout;
      const int ci = rem / a.cout, co = rem - ci * a.cout;
      const float* src = a.part + (int64_t)t * a.nslice * row + ci * 4 + co;
      for (int sl = 0; sl < a.nslice; ++sl) sum += src[(int64_t)sl * row];
      dst = a.dw + e;                    // HWIO: ((tap * cin + ci) * cout + co)
    } else {
      if (!a.db) continue;
      const int co = e - taps * a.cin * a.cout;
      const float* src = a.part + a.cin_p * 4 + co;   // tap 0 holds the bias sums
      for (int sl = 0; sl < a.nslice; ++sl) sum += src[(int64_t)sl * row];
      dst = a.db + co;
    }
    *dst = a.accumulate ? *dst + sum : sum;
  }
}

static int lanes_log2(int cin_p) {
  const int nq = cin_p / 4;
  return nq == 1 ? 0 : nq == 2 ? 1 : nq == 4 ? 2 : nq == 8 ? 3 : nq == 16 ? 4 : -1;
}

static NarrowArgs base(const of_conv_desc* d) {
  NarrowArgs a{};
  a.n = d->n, a.h = d->h, a.w = d->w, a.cin = d->cin, a.cin_p = d->cin_p, a.cout = d->cout;
  a.kh = d->kh, a.kw = d->kw, a.pt = d->pad_top, a.pl = d->pad_left, a.ho = d->ho, a.wo = d->wo;
  a.lg = lanes_log2(d->cin_p);
  return a;
}

static int wgrad_slices(const of_conv_desc* d) {
  const int64_t npix = (int64_t)d->n * d->ho * d->wo;
  const int taps = d->kh * d->kw;
  // ~4 blocks per CU in total (measured: more slices lose to the per-block reduction)
  return (int)std::max<int64_t>(1, std::min<int64_t>(1024 / taps, npix / 2048));
}

bool narrow_ok(const of_conv_desc* d) {
  return d->cout <= 4 && d->stride == 1 && d->kh == 3 && d->kw == 3 &&
         lanes_log2(d->cin_p) >= 0 && d->kh * d->kw * d->cin_p <= NARROW_MAX_W;
}

int narrow_fwd(const of_conv_desc* d, const float* x, int ldx, const float* w_fwd,
               const float* bias, int act, float alpha, float* y, int ldy, hipStream_t s) {
  NarrowArgs a = base(d);
  a.x = x, a.ldx = ldx, a.wt = w_fwd, a.bias = bias, a.out = y, a.ldo = ldy, a.act = act,
  a.alpha = alpha;
  OF_CHECK_ARG((int64_t)d->h * d->w * ldx < (1LL << 29), "narrow conv: image too large");
  const int64_t npix = (int64_t)d->n * d->ho * d->wo;
  const int ppb = 256 >> a.lg;
  const size_t lds = (size_t)d->kh * d->kw * d->cin_p * sizeof(float4);
  hipLaunchKernelGGL(narrow_fwd_kernel, dim3((unsigned)cdiv(npix, ppb)), dim3(256), lds, s, a);
  return check_launch("narrow_fwd");
}

int narrow_dgrad(const of_conv_desc* d, const float* dy, int lddy, const float* w_bwd,
                 const float* act_src, int ld_act, int act, float alpha, float* dx, int lddx,
                 hipStream_t s) {
  NarrowArgs a = base(d);
  a.dy = dy, a.lddy = lddy, a.wt = w_bwd, a.act_src = act_src, a.ld_act = ld_act, a.act = act,
  a.alpha = alpha, a.out = dx, a.ldo = lddx;
  OF_CHECK_ARG((int64_t)d->ho * d->wo * lddy < (1LL << 29), "narrow conv: image too large");
  OF_CHECK_ARG(lddx % 4 == 0 && (!act_src || ld_act % 4 == 0) && ((uintptr_t)dx & 15) == 0 &&
                   (!act_src || ((uintptr_t)act_src & 15) == 0),
               "narrow conv dgrad: dx / act_src rows must be float4 aligned");
  const int64_t npix = (int64_t)d->n * d->h * d->w;
  const int ppb = 256 >> a.lg;
  const size_t lds = (size_t)d->kh * d->kw * d->cin_p * sizeof(float4);
  hipLaunchKernelGGL(narrow_dgrad_kernel, dim3((unsigned)cdiv(npix, ppb)), dim3(256), lds, s, a);
  return check_launch("narrow_dgrad");
}

size_t narrow_wgrad_ws(const of_conv_desc* d) {
  return (size_t)d->kh * d->kw * wgrad_slices(d) * (d->cin_p * 4 + 4) * sizeof(float);
}

int narrow_wgrad(const of_conv_desc* d, const float* x, int ldx, const float* dy, int lddy,
                 float* dw, float* db, int accumulate, void* ws, hipStream_t s) {
  NarrowArgs a = base(d);
  a.x = x, a.ldx = ldx, a.dy = dy, a.lddy = lddy, a.dw = dw, a.db = db,
  a.accumulate = accumulate;
  a.nslice = wgrad_slices(d);
  a.part = static_cast<float*>(ws);
  OF_CHECK_ARG((int64_t)d->n * d->h * d->w * ldx < (1LL << 29) &&
                   (int64_t)d->n * d->ho * d->wo * lddy < (1LL << 29),
               "narrow conv wgrad: tensors too large");
  hipLaunchKernelGGL(narrow_wgrad_kernel, dim3(d->kh * d->kw, a.nslice), dim3(256), 0, s, a);
  int st = check_launch("narrow_wgrad");
  if (st) return st;
  const int total = d->kh * d->kw * d->cin * d->cout + d->cout;
  hipLaunchKernelGGL(narrow_wgrad_final_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     s, a);
  return check_launch("narrow_wgrad_final");
}

}  // namespace oflow
