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

// Sum the per-slice partials in a fixed order: block (tap, 64 consecutive partial columns);
// lane = column (coalesced 256-byte rows), wave w sums slices w, w+4, ...; the 4 wave sums
// are combined in LDS in wave order.  Column k < cin_p*4 is (ci = k/4, co = k%4) -> HWIO
// dW[tap][ci][co]; tap 0's columns cin_p*4 + co hold the bias sums.
__global__ __launch_bounds__(256) void narrow_wgrad_final_kernel(NarrowArgs a) {
  __shared__ float ws[4][64];
  const int tap = blockIdx.x, row = a.cin_p * 4 + 4;
  const int k = blockIdx.y * 64 + (threadIdx.x & 63), wave = threadIdx.x >> 6;
  float sum = 0.f;
  if (k < row) {
    const float* src = a.part + (int64_t)tap * a.nslice * row + k;
#pragma unroll 8
    for (int sl = wave; sl < a.nslice; sl += 4) sum += src[(int64_t)sl * row];
  }
  ws[wave][threadIdx.x & 63] = sum;
  __syncthreads();
  if (wave != 0 || k >= row) return;
  const int j = threadIdx.x & 63;
  sum = ((ws[0][j] + ws[1][j]) + ws[2][j]) + ws[3][j];
  float* dst = nullptr;
  if (k < a.cin_p * 4) {
    const int ci = k >> 2, co = k & 3;
    if (ci < a.cin && co < a.cout) dst = a.dw + ((int64_t)tap * a.cin + ci) * a.cout + co;
  } else if (tap == 0 && a.db && k - a.cin_p * 4 < a.cout) {
    dst = a.db + (k - a.cin_p * 4);
  }
  if (dst) *dst = a.accumulate ? *dst + sum : sum;
}

// ---- halo-tiled variants for cin_p == 32 (every flow head's last conv, 32 -> 2) ------------
// A workgroup owns an 8 x 32 pixel tile; the (8+2) x (32+2) x 32-channel input halo is
// staged in LDS once (each input pixel leaves L2 ~1.3x instead of 9x), each lane keeps
// its channel quad's 9 x 4 x CO weights in registers, so the inner loop is one conflict-free
// ds_read_b128 + 4*CO FMAs per tap.  Lanes: 8 per pixel (channel quads), 32 pixels per row.
constexpr int NT_W = 32, NT_H = 8, NT_HW = NT_W + 2, NT_HH = NT_H + 2, NT_Q = 8;

template <int CO>
__device__ __forceinline__ void load_wf(const float* wf, int q, float (&w)[NK3][4][CO]) {
  const float4* W4 = reinterpret_cast<const float4*>(wf);
#pragma unroll
  for (int t = 0; t < NK3; ++t)
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) {
      const float4 v = W4[t * 32 + 4 * q + ci];     // W_f row (tap, ci): 4 output channels
      w[t][ci][0] = v.x;
      w[t][ci][1] = v.y;
      if (CO > 2) { w[t][ci][CO > 2 ? 2 : 0] = v.z; w[t][ci][CO > 2 ? 3 : 0] = v.w; }
    }
}

// The halo staging issues all of a thread's loads before any LDS store: a loop of
// load -> store pairs kept one 16-byte load in flight per thread (narrow kernels at 1-2 TB/s).
constexpr int NT_HQ = NT_HH * NT_HW * NT_Q, NT_HU = (NT_HQ + 255) / 256;   // 2720 quads, 11
__device__ __forceinline__ void load_halo32(float4 (&v)[NT_HU], const NarrowArgs& a, int b,
                                            int y0, int x0) {
  const rsrc_t rx = make_rsrc(a.x + (int64_t)b * a.h * a.w * a.ldx, (int64_t)a.h * a.w * a.ldx * 4);
#pragma unroll
  for (int u = 0; u < NT_HU; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int qq = i & 7, pix = i >> 3, hy = pix / NT_HW, hx = pix - hy * NT_HW;
    const int iy = y0 + hy, ix = x0 + hx;
    const bool ok = i < NT_HQ && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
    v[u] = bload4(rx, ok ? 4u * ((iy * a.w + ix) * a.ldx + 4 * qq) : kOOB);
  }
}

__device__ __forceinline__ void store_halo32(float4* halo, const float4 (&v)[NT_HU]) {
#pragma unroll
  for (int u = 0; u < NT_HU; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (NT_HQ % 256 == 0 || i < NT_HQ) halo[i] = v[u];
  }
}

__device__ __forceinline__ void stage_halo32(float4* halo, const NarrowArgs& a, int b, int y0,
                                             int x0) {
  float4 v[NT_HU];
  load_halo32(v, a, b, y0, x0);
  store_halo32(halo, v);
}

template <int CO>
__global__ __launch_bounds__(256) void narrow_fwd_tile(NarrowArgs a) {
  __shared__ float4 halo[NT_HH * NT_HW * NT_Q];          // 43.5 KB
  const int q = threadIdx.x & 7, col = threadIdx.x >> 3;
  const int tx0 = blockIdx.x * NT_W, ty0 = blockIdx.y * NT_H, b = blockIdx.z;
  float w[NK3][4][CO];
  load_wf<CO>(a.wt, q, w);
  stage_halo32(halo, a, b, ty0 - a.pt, tx0 - a.pl);
  __syncthreads();
  float bias[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) bias[c] = (a.bias && c < a.cout) ? a.bias[c] : 0.f;
  const int ox = tx0 + col;
  for (int r = 0; r < NT_H; ++r) {
    float acc[CO];
#pragma unroll
    for (int c = 0; c < CO; ++c) acc[c] = 0.f;
#pragma unroll
    for (int t = 0; t < NK3; ++t) {
      const float4 xv = halo[((r + t / 3) * NT_HW + col + t % 3) * NT_Q + q];
#pragma unroll
      for (int c = 0; c < CO; ++c)
        acc[c] = fmaf(xv.w, w[t][3][c], fmaf(xv.z, w[t][2][c], fmaf(xv.y, w[t][1][c],
                 fmaf(xv.x, w[t][0][c], acc[c]))));
    }
#pragma unroll
    for (int c = 0; c < CO; ++c) acc[c] = lane_sum(acc[c], 3);
    const int oy = ty0 + r;
    if (q < CO && q < a.cout && oy < a.ho && ox < a.wo) {
      float v = acc[0], bv = bias[0];
#pragma unroll
      for (int c = 1; c < CO; ++c) {
        v = q == c ? acc[c] : v;
        bv = q == c ? bias[c] : bv;
      }
      v += bv;
      if (a.act == OF_ACT_RELU) v = v > 0.f ? v : 0.f;
      if (a.act == OF_ACT_LEAKY) v = v > 0.f ? v : a.alpha * v;
      a.out[(((int64_t)b * a.ho + oy) * a.wo + ox) * a.ldo + q] = v;
    }
  }
}

// dx[iy][ix][4q..4q+3] = sum_t sum_co dy[iy - r + pt][ix - s + pl][co] * W[t][4q..][co]
template <int CO>
__global__ __launch_bounds__(256) void narrow_dgrad_tile(NarrowArgs a) {
  __shared__ float dyh[NT_HH * NT_HW * CO];
  const int q = threadIdx.x & 7, col = threadIdx.x >> 3;
  const int tx0 = blockIdx.x * NT_W, ty0 = blockIdx.y * NT_H, b = blockIdx.z;
  float4 w[NK3][CO];
  const float4* W4 = reinterpret_cast<const float4*>(a.wt);   // W_d [(t*4 + co)][32]
#pragma unroll
  for (int t = 0; t < NK3; ++t)
#pragma unroll
    for (int c = 0; c < CO; ++c) w[t][c] = W4[(t * 4 + c) * 8 + q];
  const rsrc_t rd =
      make_rsrc(a.dy + (int64_t)b * a.ho * a.wo * a.lddy, (int64_t)a.ho * a.wo * a.lddy * 4);
  const int y0 = ty0 + a.pt - 2, x0 = tx0 + a.pl - 2;       // dy halo origin
  constexpr int DQ = NT_HH * NT_HW * CO, DU = (DQ + 255) / 256;
  float dv[DU];
#pragma unroll
  for (int u = 0; u < DU; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int c = i % CO, pix = i / CO, hy = pix / NT_HW, hx = pix - hy * NT_HW;
    const int oy = y0 + hy, ox = x0 + hx;
    const bool ok = i < DQ && c < a.cout && (unsigned)oy < (unsigned)a.ho && (unsigned)ox < (unsigned)a.wo;
    dv[u] = bload1(rd, ok ? 4u * ((oy * a.wo + ox) * a.lddy + c) : kOOB);
  }
#pragma unroll
  for (int u = 0; u < DU; ++u)
    if (threadIdx.x + 256 * u < DQ) dyh[threadIdx.x + 256 * u] = dv[u];
  __syncthreads();
  const int ix = tx0 + col;
  const float neg = a.act == OF_ACT_LEAKY ? a.alpha : 0.f;
  for (int r = 0; r < NT_H; ++r) {
    const int iy = ty0 + r;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int t = 0; t < NK3; ++t) {
      const float* d = &dyh[((r + 2 - t / 3) * NT_HW + col + 2 - t % 3) * CO];
#pragma unroll
      for (int c = 0; c < CO; ++c) acc = fma4(d[c], w[t][c], acc);
    }
    if (iy < a.h && ix < a.w) {
      const int64_t p = ((int64_t)b * a.h + iy) * a.w + ix;
      if (a.act_src) {
        const float4 sv = *reinterpret_cast<const float4*>(a.act_src + p * a.ld_act + 4 * q);
        acc.x *= sv.x > 0.f ? 1.f : neg;
        acc.y *= sv.y > 0.f ? 1.f : neg;
        acc.z *= sv.z > 0.f ? 1.f : neg;
        acc.w *= sv.w > 0.f ? 1.f : neg;
      }
      *reinterpret_cast<float4*>(a.out + p * a.ldo + 4 * q) = acc;
    }
  }
}

// Per-block partials of dW[t][ci][co] (+ bias sums) over a grid-stride set of 8 x 32 tiles,
// written in narrow_wgrad_kernel's partial layout (slice = block), summed by
// narrow_wgrad_final_kernel in a fixed order.
template <int CO>
__global__ __launch_bounds__(256) void narrow_wgrad_tile(NarrowArgs a, int tiles_x, int tiles_y) {
  __shared__ float4 halo[NT_HH * NT_HW * NT_Q];
  __shared__ float dyt[NT_H * NT_W * CO];
  const int q = threadIdx.x & 7, col = threadIdx.x >> 3;
  float acc[NK3][4][CO];
#pragma unroll
  for (int t = 0; t < NK3; ++t)
#pragma unroll
    for (int ci = 0; ci < 4; ++ci)
#pragma unroll
      for (int c = 0; c < CO; ++c) acc[t][ci][c] = 0.f;
  float bacc[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) bacc[c] = 0.f;
  const int ntiles = tiles_x * tiles_y * a.n;
  // the next tile's halo and dy are loaded into registers while this tile computes
  constexpr int DQ = NT_H * NT_W * CO, DU = (DQ + 255) / 256;
  float4 hv[NT_HU];
  float dv[DU];
  auto load = [&](int tile) {
    const int b = tile / (tiles_x * tiles_y), rem = tile - b * tiles_x * tiles_y;
    const int ty0 = (rem / tiles_x) * NT_H, tx0 = (rem % tiles_x) * NT_W;
    load_halo32(hv, a, b, ty0 - a.pt, tx0 - a.pl);
    const rsrc_t rd =
        make_rsrc(a.dy + (int64_t)b * a.ho * a.wo * a.lddy, (int64_t)a.ho * a.wo * a.lddy * 4);
#pragma unroll
    for (int u = 0; u < DU; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int c = i % CO, pix = i / CO, hy = pix / NT_W, hx = pix - hy * NT_W;
      const int oy = ty0 + hy, ox = tx0 + hx;
      const bool ok = i < DQ && c < a.cout && oy < a.ho && ox < a.wo;
      dv[u] = bload1(rd, ok ? 4u * ((oy * a.wo + ox) * a.lddy + c) : kOOB);
    }
  };
  if (blockIdx.x < ntiles) load(blockIdx.x);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    __syncthreads();                                   // previous tile's LDS reads done
    store_halo32(halo, hv);
#pragma unroll
    for (int u = 0; u < DU; ++u)
      if (threadIdx.x + 256 * u < DQ) dyt[threadIdx.x + 256 * u] = dv[u];
    __syncthreads();
    if (tile + (int)gridDim.x < ntiles) load(tile + gridDim.x);
#pragma unroll 1
    for (int r = 0; r < NT_H; ++r) {
      float d[CO];
#pragma unroll
      for (int c = 0; c < CO; ++c) d[c] = dyt[(r * NT_W + col) * CO + c];
#pragma unroll
      for (int c = 0; c < CO; ++c) bacc[c] += d[c];
#pragma unroll
      for (int t = 0; t < NK3; ++t) {
        const float4 xv = halo[((r + t / 3) * NT_HW + col + t % 3) * NT_Q + q];
#pragma unroll
        for (int c = 0; c < CO; ++c) {
          acc[t][0][c] = fmaf(xv.x, d[c], acc[t][0][c]);
          acc[t][1][c] = fmaf(xv.y, d[c], acc[t][1][c]);
          acc[t][2][c] = fmaf(xv.z, d[c], acc[t][2][c]);
          acc[t][3][c] = fmaf(xv.w, d[c], acc[t][3][c]);
        }
      }
    }
  }
  // reduce over the 8 pixel columns of a wave (lane bits 3..5), then over the 4 waves
  __syncthreads();
  float* red = reinterpret_cast<float*>(halo);          // [4 waves][8 q][9*4*CO + CO]
  constexpr int ROW = NK3 * 4 * CO + CO;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < NK3; ++t)
#pragma unroll
    for (int ci = 0; ci < 4; ++ci)
#pragma unroll
      for (int c = 0; c < CO; ++c) {
        float v = acc[t][ci][c];
        v += __shfl_xor(v, 8);
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        if (lane < 8) red[(wave * 8 + q) * ROW + (t * 4 + ci) * CO + c] = v;
      }
#pragma unroll
  for (int c = 0; c < CO; ++c) {
    float v = bacc[c];
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane < 8) red[(wave * 8 + q) * ROW + NK3 * 4 * CO + c] = v;
  }
  __syncthreads();
  const int row = a.cin_p * 4 + 4;                       // narrow_wgrad_final's layout
  for (int e = threadIdx.x; e < NK3 * 32 * 4 + 4; e += 256) {
    float sum = 0.f;
    int t, slot;
    if (e < NK3 * 32 * 4) {
      t = e / 128;
      const int ci = (e % 128) >> 2, co = e & 3;
      slot = co < CO ? ((ci >> 2) * ROW + (t * 4 + (ci & 3)) * CO + co) : -1;
      if (slot >= 0)
        for (int wv = 0; wv < 4; ++wv) sum += red[wv * 8 * ROW + slot];
      a.part[((int64_t)t * a.nslice + blockIdx.x) * row + (e % 128)] = sum;
    } else {
      const int co = e - NK3 * 128;
      if (co < CO)                                       // bias: counted once per pixel (q = 0)
        for (int wv = 0; wv < 4; ++wv) sum += red[(wv * 8) * ROW + NK3 * 4 * CO + co];
      a.part[(int64_t)blockIdx.x * row + a.cin_p * 4 + co] = sum;   // tap 0 holds the bias
    }
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

static bool narrow_tiled(const of_conv_desc* d) { return d->cin_p == 32 && d->cout <= 4; }
static int tiles_x(const of_conv_desc* d) { return (int)cdiv(d->wo, NT_W); }
static int tiles_y(const of_conv_desc* d) { return (int)cdiv(d->ho, NT_H); }

static int wgrad_slices(const of_conv_desc* d) {
  if (narrow_tiled(d))   // one partial per block; 3 blocks per CU, grid-stride over the tiles
    return (int)std::min<int64_t>((int64_t)tiles_x(d) * tiles_y(d) * d->n, 768);
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
  if (narrow_tiled(d) && ldx % 4 == 0) {
    const dim3 grid(tiles_x(d), tiles_y(d), d->n);
    if (d->cout <= 2) hipLaunchKernelGGL(narrow_fwd_tile<2>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(narrow_fwd_tile<4>, grid, dim3(256), 0, s, a);
    return check_launch("narrow_fwd_tile");
  }
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
  if (narrow_tiled(d)) {   // stride 1, 'same': the input grid is the output grid
    const dim3 grid((unsigned)cdiv(d->w, NT_W), (unsigned)cdiv(d->h, NT_H), d->n);
    if (d->cout <= 2) hipLaunchKernelGGL(narrow_dgrad_tile<2>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(narrow_dgrad_tile<4>, grid, dim3(256), 0, s, a);
    return check_launch("narrow_dgrad_tile");
  }
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
  if (narrow_tiled(d) && ldx % 4 == 0) {
    if (d->cout <= 2)
      hipLaunchKernelGGL(narrow_wgrad_tile<2>, dim3(a.nslice), dim3(256), 0, s, a, tiles_x(d),
                         tiles_y(d));
    else
      hipLaunchKernelGGL(narrow_wgrad_tile<4>, dim3(a.nslice), dim3(256), 0, s, a, tiles_x(d),
                         tiles_y(d));
  } else {
    hipLaunchKernelGGL(narrow_wgrad_kernel, dim3(d->kh * d->kw, a.nslice), dim3(256), 0, s, a);
  }
  int st = check_launch("narrow_wgrad");
  if (st) return st;
  hipLaunchKernelGGL(narrow_wgrad_final_kernel,
                     dim3(d->kh * d->kw, (unsigned)cdiv(d->cin_p * 4 + 4, 64)), dim3(256), 0, s, a);
  return check_launch("narrow_wgrad_final");
}

}  // namespace oflow
