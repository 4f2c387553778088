// Implicit-GEMM NHWC convolution on CDNA4 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces TF's Conv2D / Conv2DBackpropInput / Conv2DBackpropFilter behind every
// layers.Conv2D(padding='same') of the reference (model.py:12, 104-114, and the resnet
// submodule's convs).  im2col-free: every K-chunk of the A operand is gathered straight from
// the NHWC activation into an LDS tile (coalesced 16-byte loads along channels), the B
// operand is the per-step packed weight matrix (or dy for the weight gradient).
//
//   FWD   C[m=out pixel][n=cout]  = sum_{k=(tap,ci)}  x[pix(m,tap)][ci] * Wf[k][n]
//   DGRAD C[m=in  pixel][n=ci]    = sum_{k=(tap,co)} dy[pix^-1(m,tap)][co] * Wd[k][n]
//         (stride-2 layers: the transposed convolution; taps whose source is not on the
//          stride lattice contribute zero)
//   WGRAD C[m=(tap,ci)][n=cout]  = sum_{k=out pixel} x[pix(k,tap)][ci] * dy[k][n]
//         (split-K over pixels into fp32 slabs, reduced deterministically)
//
// Tiling: BM x BN x 16 per 256-thread workgroup (4 waves), each wave an (BM/WAVES_M) x
// (BN/WAVES_N) block of 32x32 MFMA tiles.  LDS holds both operands k-major ([k][m], [k][n]) so
// the MFMA operand fetch is one conflict-free ds_read_b32 per lane (lanes 0-31 row k,
// lanes 32-63 row k+1).  Global->LDS is register-staged and double-buffered: the loads of
// chunk c+1 are issued before the MFMAs of chunk c, one barrier per chunk.  Fused epilogues:
// bias, BN-inference affine, residual add, ReLU/LeakyReLU (fwd); activation derivative of
// the producer layer (dgrad).  Block ids are remapped so neighbouring tiles share an XCD L2.
#include "common.h"

namespace oflow {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };
constexpr int BK = 16;

struct GemmArgs {
  int n, h, w, ho, wo;
  int kh, kw, stride, pt, pl;
  int kc;                 // channels per tap along K (fwd: cin_p, dgrad: cout_p) / M (wgrad)
  int taps;
  int M, N, K;            // fwd/dgrad: K = padded taps*kc; wgrad: K = output pixels
  const float* A; int lda;
  const float* B; int ldb; int nb;
  float* C; int ldc;
  const float* bias;
  const float* bn_g; const float* bn_b; const float* bn_m; const float* bn_v; float bn_eps;
  const float* res; int ldr;
  float* z; int ldz;
  int act; float alpha;
  const float* act_src; int ld_act;
  int k_per_split;
  int64_t split_stride;
  int m_tiles, n_tiles;
};

__device__ __forceinline__ float act_fwd(float v, int act, float alpha) {
  if (act == OF_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == OF_ACT_LEAKY) return v > 0.f ? v : alpha * v;
  return v;
}

template <int BM, int BN, int WAVES_M, int WAVES_N, int MODE>
__global__ __launch_bounds__(256, 2) void conv_gemm_f32(GemmArgs a) {
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  static_assert(TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "tile");
  constexpr bool A_KCONTIG = (MODE != MODE_WGRAD);
  constexpr int SA = A_KCONTIG ? BM + 2 : BM + 4;   // +2: conflict-free transposed b32 writes
  constexpr int SB = BN + 4;
  constexpr int A_SLOTS = BM * BK / 4 / 256;
  constexpr int B_QUADS = BK * BN / 4;
  constexpr int B_SLOTS = (B_QUADS + 255) / 256;
  static_assert(A_SLOTS >= 1, "BM >= 64");

  __shared__ float As[2][BK * SA];
  __shared__ float Bs[2][BK * SB];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;

  // XCD-aware bijective remap: consecutive tiles -> one XCD's L2 (cdna guide T1).
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  int wgid;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tile_n = wgid % a.n_tiles;
  const int tile_m = wgid / a.n_tiles;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // ---------------- K range -------------------------------------------------------------
  int k_begin = 0, k_end = a.K;
  if (MODE == MODE_WGRAD) {
    k_begin = blockIdx.z * a.k_per_split;
    k_end = min(a.K, k_begin + a.k_per_split);
  }
  const int nchunks = (k_end - k_begin + BK - 1) / BK;

  // ---------------- A loader state ------------------------------------------------------
  // K-contig (fwd/dgrad): thread -> (row = tid/4 + 64*i, kq = tid%4), 4 channels of one tap.
  // M-contig (wgrad): thread -> (mq = tid % (BM/4), krow = tid/(BM/4) + i*256/(BM/4)).
  const int src_h = (MODE == MODE_DGRAD) ? a.ho : a.h;
  const int src_w = (MODE == MODE_DGRAD) ? a.wo : a.w;
  int a_py[A_SLOTS], a_px[A_SLOTS], a_b[A_SLOTS];
  bool a_ok[A_SLOTS];
  int ks_r = 0, ks_s = 0, ks_ci = 0, ks_tap = 0;   // fwd/dgrad: per-thread k state
  int wm_r = 0, wm_s = 0, wm_ci = 0;                // wgrad: per-thread fixed m
  bool wm_ok = false;
  int a_oy[A_SLOTS], a_ox[A_SLOTS], a_kb[A_SLOTS];  // wgrad: per-slot pixel state

  if constexpr (A_KCONTIG) {
    const int kq = tid & 3;
    const int hw = a.ho * a.wo;   // fwd: rows are output pixels
    const int hw_in = a.h * a.w;  // dgrad: rows are input pixels
#pragma unroll
    for (int i = 0; i < A_SLOTS; ++i) {
      const int m = m0 + (tid >> 2) + 64 * i;
      a_ok[i] = m < a.M;
      const int mm = a_ok[i] ? m : 0;
      if (MODE == MODE_FWD) {
        const int b = mm / hw, rem = mm - b * hw;
        const int oy = rem / a.wo, ox = rem - oy * a.wo;
        a_b[i] = b * a.h;
        a_py[i] = oy * a.stride - a.pt;
        a_px[i] = ox * a.stride - a.pl;
      } else {
        const int b = mm / hw_in, rem = mm - b * hw_in;
        const int iy = rem / a.w, ix = rem - iy * a.w;
        a_b[i] = b * a.ho;
        a_py[i] = iy + a.pt;
        a_px[i] = ix + a.pl;
      }
    }
    const int k0 = kq * 4;
    ks_tap = k0 / a.kc;
    ks_ci = k0 - ks_tap * a.kc;
    ks_r = ks_tap / a.kw;
    ks_s = ks_tap - ks_r * a.kw;
  } else {
    constexpr int MQ = BM / 4;
    const int mq = tid % MQ;
    const int m = m0 + 4 * mq;
    wm_ok = m < a.M;
    const int mm = wm_ok ? m : 0;
    const int tap = mm / a.kc;
    wm_ci = mm - tap * a.kc;
    wm_r = tap / a.kw;
    wm_s = tap - wm_r * a.kw;
    const int hw = a.ho * a.wo;
#pragma unroll
    for (int i = 0; i < A_SLOTS; ++i) {
      const int krow = tid / MQ + i * (256 / MQ);
      const int k = k_begin + krow;
      a_kb[i] = k;
      const int kk = k < a.K ? k : 0;
      const int b = kk / hw, rem = kk - b * hw;
      a_oy[i] = rem / a.wo;
      a_ox[i] = rem - a_oy[i] * a.wo;
      a_b[i] = b;
    }
  }

  float4 ra[A_SLOTS];
  float4 rb[B_SLOTS];

  auto load_a = [&]() {
    if constexpr (A_KCONTIG) {
      const bool tap_ok = ks_tap < a.taps;
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        bool ok = a_ok[i] && tap_ok;
        int sy, sx;
        if (MODE == MODE_FWD) {
          sy = a_py[i] + ks_r;
          sx = a_px[i] + ks_s;
        } else {
          const int ty = a_py[i] - ks_r, tx = a_px[i] - ks_s;
          if (a.stride == 1) {
            sy = ty;
            sx = tx;
          } else {
            ok = ok && ty >= 0 && tx >= 0 && (ty % a.stride) == 0 && (tx % a.stride) == 0;
            sy = ty / a.stride;
            sx = tx / a.stride;
          }
        }
        ok = ok && (unsigned)sy < (unsigned)src_h && (unsigned)sx < (unsigned)src_w;
        if (ok) {
          const int64_t pix = (int64_t)(a_b[i] + sy) * src_w + sx;
          v = *reinterpret_cast<const float4*>(a.A + pix * a.lda + ks_ci);
        }
        ra[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        const int sy = a_oy[i] * a.stride - a.pt + wm_r;
        const int sx = a_ox[i] * a.stride - a.pl + wm_s;
        const bool ok = wm_ok && a_kb[i] < k_end && (unsigned)sy < (unsigned)a.h &&
                        (unsigned)sx < (unsigned)a.w;
        if (ok) {
          const int64_t pix = ((int64_t)a_b[i] * a.h + sy) * a.w + sx;
          v = *reinterpret_cast<const float4*>(a.A + pix * a.lda + wm_ci);
        }
        ra[i] = v;
      }
    }
  };
  auto advance_a = [&]() {
    if constexpr (A_KCONTIG) {
      ks_ci += BK;
      while (ks_ci >= a.kc) {
        ks_ci -= a.kc;
        ++ks_tap;
        if (++ks_s >= a.kw) {
          ks_s = 0;
          ++ks_r;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        a_kb[i] += BK;
        a_ox[i] += BK;
        while (a_ox[i] >= a.wo) {
          a_ox[i] -= a.wo;
          if (++a_oy[i] >= a.ho) {
            a_oy[i] = 0;
            ++a_b[i];
          }
        }
      }
    }
  };
  auto store_a = [&](int buf) {
    if constexpr (A_KCONTIG) {
      const int kq = tid & 3;
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        float* p = &As[buf][(kq * 4) * SA + (tid >> 2) + 64 * i];
        p[0] = ra[i].x;
        p[SA] = ra[i].y;
        p[2 * SA] = ra[i].z;
        p[3 * SA] = ra[i].w;
      }
    } else {
      constexpr int MQ = BM / 4;
      const int mq = tid % MQ;
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        const int krow = tid / MQ + i * (256 / MQ);
        *reinterpret_cast<float4*>(&As[buf][krow * SA + 4 * mq]) = ra[i];
      }
    }
  };

  // ---------------- B loader --------------------------------------------------------------
  int b_k = k_begin;   // first k row of the current chunk
  auto load_b = [&]() {
    constexpr int NQ = BN / 4;
#pragma unroll
    for (int i = 0; i < B_SLOTS; ++i) {
      const int slot = tid + 256 * i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (slot < B_QUADS) {
        const int krow = slot / NQ, nq = slot - krow * NQ;
        const int n = n0 + 4 * nq;
        const int k = b_k + krow;
        bool ok = n < a.nb;
        if (MODE == MODE_WGRAD) ok = ok && k < k_end;
        if (ok) v = *reinterpret_cast<const float4*>(a.B + (int64_t)k * a.ldb + n);
      }
      rb[i] = v;
    }
  };
  auto store_b = [&](int buf) {
    constexpr int NQ = BN / 4;
#pragma unroll
    for (int i = 0; i < B_SLOTS; ++i) {
      const int slot = tid + 256 * i;
      if (slot < B_QUADS) {
        const int krow = slot / NQ, nq = slot - krow * NQ;
        *reinterpret_cast<float4*>(&Bs[buf][krow * SB + 4 * nq]) = rb[i];
      }
    }
  };

  // ---------------- main loop --------------------------------------------------------------
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm0 = (wave / WAVES_N) * WM;
  const int wn0 = (wave % WAVES_N) * WN;
  const int lrow = lane & 31, lk = lane >> 5;

  if (nchunks > 0) {
    load_a();
    load_b();
    store_a(0);
    store_b(0);
  }
  __syncthreads();

  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) {
      advance_a();
      b_k += BK;
      load_a();
      load_b();
    }
    const float* as = As[buf];
    const float* bs = Bs[buf];
#pragma unroll
    for (int st = 0; st < BK / 2; ++st) {
      const int kk = 2 * st + lk;
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = as[kk * SA + wm0 + 32 * i + lrow];
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = bs[kk * SB + wn0 + 32 * j + lrow];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_a(buf ^ 1);
      store_b(buf ^ 1);
    }
    __syncthreads();
  }

  // ---------------- epilogue ---------------------------------------------------------------
  float* C = a.C;
  if (MODE == MODE_WGRAD) C += (int64_t)blockIdx.z * a.split_stride;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + 32 * j + lrow;
    if (n >= a.N) continue;
    float bias = 0.f, scale = 1.f, shift = 0.f;
    if (MODE == MODE_FWD) {
      if (a.bias) bias = a.bias[n];
      if (a.bn_g) {
        scale = a.bn_g[n] * rsqrtf(a.bn_v[n] + a.bn_eps);
        shift = a.bn_b[n] - a.bn_m[n] * scale;
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (m >= a.M) continue;
        float v = acc[i][j][r];
        if (MODE == MODE_FWD) {
          v += bias;
          if (a.z) a.z[(int64_t)m * a.ldz + n] = v;
          if (a.bn_g) v = v * scale + shift;
          if (a.res) v += a.res[(int64_t)m * a.ldr + n];
          v = act_fwd(v, a.act, a.alpha);
        } else if (MODE == MODE_DGRAD) {
          if (a.act_src) {
            const float s = a.act_src[(int64_t)m * a.ld_act + n];
            v *= s > 0.f ? 1.f : (a.act == OF_ACT_LEAKY ? a.alpha : 0.f);
          }
        }
        C[(int64_t)m * a.ldc + n] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------- weight packing --
__global__ void pack_fwd_kernel(const float* __restrict__ w, int taps, int cin, int cout,
                                int cin_p, int kf, int nf, float* __restrict__ out) {
  const int64_t total = (int64_t)kf * nf;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(idx / nf), n = (int)(idx - (int64_t)k * nf);
    const int tap = k / cin_p, ci = k - tap * cin_p;
    float v = 0.f;
    if (tap < taps && ci < cin && n < cout) v = w[((int64_t)tap * cin + ci) * cout + n];
    out[idx] = v;
  }
}

__global__ void pack_bwd_kernel(const float* __restrict__ w, int taps, int cin, int cout,
                                int cout_p, int kd, int nd, float* __restrict__ out) {
  const int64_t total = (int64_t)kd * nd;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(idx / nd), n = (int)(idx - (int64_t)k * nd);
    const int tap = k / cout_p, co = k - tap * cout_p;
    float v = 0.f;
    if (tap < taps && co < cout && n < cin) v = w[((int64_t)tap * cin + n) * cout + co];
    out[idx] = v;
  }
}

__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, int splits,
                                    int64_t split_stride, int taps, int kc, int cin, int cout,
                                    int ldc, float* __restrict__ dw, int accum) {
  const int64_t total = (int64_t)taps * cin * cout;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(idx % cout);
    const int64_t t2 = idx / cout;
    const int ci = (int)(t2 % cin);
    const int tap = (int)(t2 / cin);
    const int64_t off = ((int64_t)tap * kc + ci) * ldc + co;
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += ws[z * split_stride + off];
    dw[idx] = accum ? dw[idx] + s : s;
  }
}

// ------------------------------------------------------------------------------ dispatch --
namespace {

struct Geo {
  int taps, cin_p, cout_p, kf, nf, kd, nd;
};

Geo geo(const of_conv_desc* d) {
  Geo g;
  g.taps = d->kh * d->kw;
  g.cin_p = d->cin_p;
  g.cout_p = (int)round_up(d->cout, 4);
  g.kf = (int)round_up((int64_t)g.taps * g.cin_p, BK);
  g.nf = g.cout_p;
  g.kd = (int)round_up((int64_t)g.taps * g.cout_p, BK);
  g.nd = g.cin_p;
  return g;
}

int validate(const of_conv_desc* d) {
  OF_CHECK_ARG(d != nullptr, "conv desc is NULL");
  OF_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->cin > 0 && d->cout > 0, "conv dims");
  OF_CHECK_ARG(d->cin_p >= d->cin && d->cin_p % 4 == 0, "cin_p must be >= cin, multiple of 4");
  OF_CHECK_ARG(d->kh > 0 && d->kw > 0 && d->stride > 0, "conv kernel/stride");
  OF_CHECK_ARG(d->ho > 0 && d->wo > 0, "conv output dims");
  return OF_OK;
}

template <int MODE>
int launch_cfg(GemmArgs& a, hipStream_t s, int splits) {
  // Tile choice by GEMM N (output channels of this pass).
  const int N = a.N;
  dim3 block(256);
  auto go = [&](auto kern, int bm, int bn) {
    a.m_tiles = (int)cdiv(a.M, bm);
    a.n_tiles = (int)cdiv(N, bn);
    dim3 grid(a.m_tiles * a.n_tiles, 1, splits);
    hipLaunchKernelGGL(kern, grid, block, 0, s, a);
    return check_launch("conv_gemm_f32");
  };
  if (N > 96) return go(conv_gemm_f32<128, 128, 2, 2, MODE>, 128, 128);
  if (N > 64) return go(conv_gemm_f32<128, 96, 4, 1, MODE>, 128, 96);
  if (N > 32) return go(conv_gemm_f32<128, 64, 2, 2, MODE>, 128, 64);
  return go(conv_gemm_f32<128, 32, 4, 1, MODE>, 128, 32);
}

GemmArgs base_args(const of_conv_desc* d) {
  GemmArgs a{};
  a.n = d->n;
  a.h = d->h;
  a.w = d->w;
  a.ho = d->ho;
  a.wo = d->wo;
  a.kh = d->kh;
  a.kw = d->kw;
  a.stride = d->stride;
  a.pt = d->pad_top;
  a.pl = d->pad_left;
  a.taps = d->kh * d->kw;
  a.alpha = 0.f;
  return a;
}

}  // namespace
}  // namespace oflow

using namespace oflow;

extern "C" {

int64_t of_conv_wfwd_elems(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return -1;
  Geo g = geo(d);
  return (int64_t)g.kf * g.nf;
}

int64_t of_conv_wbwd_elems(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return -1;
  Geo g = geo(d);
  return (int64_t)g.kd * g.nd;
}

int of_conv_pack_weights(const of_conv_desc* d, const float* w_hwio, float* w_fwd,
                         float* w_bwd, void* stream) {
  int st = validate(d);
  if (st) return st;
  OF_CHECK_ARG(w_hwio && w_fwd, "pack: NULL pointer");
  Geo g = geo(d);
  hipStream_t s = as_stream(stream);
  {
    const int64_t total = (int64_t)g.kf * g.nf;
    const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 4096);
    hipLaunchKernelGGL(pack_fwd_kernel, dim3(blocks), dim3(256), 0, s, w_hwio, g.taps, d->cin,
                       d->cout, g.cin_p, g.kf, g.nf, w_fwd);
    if ((st = check_launch("pack_fwd"))) return st;
  }
  if (w_bwd) {
    const int64_t total = (int64_t)g.kd * g.nd;
    const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 4096);
    hipLaunchKernelGGL(pack_bwd_kernel, dim3(blocks), dim3(256), 0, s, w_hwio, g.taps, d->cin,
                       d->cout, g.cout_p, g.kd, g.nd, w_bwd);
    if ((st = check_launch("pack_bwd"))) return st;
  }
  return OF_OK;
}

int of_conv2d_fwd(const of_conv_desc* d, const float* x, int ldx, const float* w_fwd,
                  const float* bias, const float* bn_gamma, const float* bn_beta,
                  const float* bn_mean, const float* bn_var, float bn_eps,
                  const float* residual, int ldr, int act, float alpha, float* z, int ldz,
                  float* y, int ldy, void* stream) {
  int st = validate(d);
  if (st) return st;
  OF_CHECK_ARG(x && w_fwd && y, "conv fwd: NULL pointer");
  OF_CHECK_ARG(ldx >= d->cin_p && ldx % 4 == 0, "conv fwd: ldx");
  OF_CHECK_ARG(ldy >= d->cout, "conv fwd: ldy");
  OF_CHECK_ARG(!bn_gamma || (bn_beta && bn_mean && bn_var), "conv fwd: incomplete BN params");
  OF_CHECK_ARG(!residual || ldr >= d->cout, "conv fwd: ldr");
  OF_CHECK_ARG(!z || ldz >= d->cout, "conv fwd: ldz");
  OF_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)w_fwd & 15) == 0,
               "conv fwd: x / w must be 16-byte aligned");
  Geo g = geo(d);
  GemmArgs a = base_args(d);
  a.kc = g.cin_p;
  a.M = d->n * d->ho * d->wo;
  a.N = d->cout;
  a.K = g.kf;
  a.A = x;
  a.lda = ldx;
  a.B = w_fwd;
  a.ldb = g.nf;
  a.nb = g.nf;
  a.C = y;
  a.ldc = ldy;
  a.bias = bias;
  a.bn_g = bn_gamma;
  a.bn_b = bn_beta;
  a.bn_m = bn_mean;
  a.bn_v = bn_var;
  a.bn_eps = bn_eps;
  a.res = residual;
  a.ldr = ldr;
  a.z = z;
  a.ldz = ldz;
  a.act = act;
  a.alpha = alpha;
  hipStream_t s = as_stream(stream);
  const double flops = 2.0 * a.M * d->cout * (double)g.taps * d->cin;
  if (timing_on()) timing_begin(s);
  st = launch_cfg<MODE_FWD>(a, s, 1);
  if (timing_on()) timing_end(s, 0, flops);
  return st;
}

int of_conv2d_dgrad(const of_conv_desc* d, const float* dy, int lddy, const float* w_bwd,
                    const float* act_src, int ld_act, int act, float alpha, float* dx,
                    int lddx, void* stream) {
  int st = validate(d);
  if (st) return st;
  Geo g = geo(d);
  OF_CHECK_ARG(dy && w_bwd && dx, "conv dgrad: NULL pointer");
  OF_CHECK_ARG(lddy >= g.cout_p && lddy % 4 == 0, "conv dgrad: lddy (>= round_up(cout,4))");
  OF_CHECK_ARG(lddx >= d->cin_p, "conv dgrad: lddx");
  OF_CHECK_ARG(!act_src || ld_act >= d->cin_p, "conv dgrad: ld_act");
  OF_CHECK_ARG(((uintptr_t)dy & 15) == 0 && ((uintptr_t)w_bwd & 15) == 0,
               "conv dgrad: dy / w must be 16-byte aligned");
  GemmArgs a = base_args(d);
  a.kc = g.cout_p;
  a.M = d->n * d->h * d->w;
  a.N = g.cin_p;
  a.K = g.kd;
  a.A = dy;
  a.lda = lddy;
  a.B = w_bwd;
  a.ldb = g.nd;
  a.nb = g.nd;
  a.C = dx;
  a.ldc = lddx;
  a.act_src = act_src;
  a.ld_act = ld_act;
  a.act = act;
  a.alpha = alpha;
  hipStream_t s = as_stream(stream);
  const double flops = 2.0 * d->n * d->ho * d->wo * (double)d->cout * g.taps * d->cin;
  if (timing_on()) timing_begin(s);
  st = launch_cfg<MODE_DGRAD>(a, s, 1);
  if (timing_on()) timing_end(s, 1, flops);
  return st;
}

namespace {
struct WgradPlan {
  int splits, k_per_split, M, ldc;
  int64_t split_stride;
};
WgradPlan wgrad_plan(const of_conv_desc* d) {
  Geo g = geo(d);
  WgradPlan p;
  p.M = g.taps * g.cin_p;
  p.ldc = g.cout_p;
  const int K = d->n * d->ho * d->wo;
  const int bn = d->cout > 96 ? 128 : d->cout > 64 ? 96 : d->cout > 32 ? 64 : 32;
  const int tiles = (int)(cdiv(p.M, 128) * cdiv(d->cout, bn));
  // Aim for ~1024 workgroups; at least 4 chunks of K per split.
  int splits = (int)std::max<int64_t>(1, cdiv(1024, tiles));
  const int max_splits = (int)std::max<int64_t>(1, cdiv(K, 4 * BK));
  splits = std::min(splits, max_splits);
  p.k_per_split = (int)round_up(cdiv(K, splits), BK);
  p.splits = (int)cdiv(K, p.k_per_split);
  p.split_stride = (int64_t)p.M * p.ldc;
  return p;
}
}  // namespace

size_t of_conv2d_wgrad_workspace(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return 0;
  WgradPlan p = wgrad_plan(d);
  const size_t slabs = (size_t)p.splits * p.split_stride * sizeof(float);
  return std::max(slabs, of_colsum_workspace((int64_t)d->n * d->ho * d->wo, d->cout));
}

int of_conv2d_wgrad(const of_conv_desc* d, const float* x, int ldx, const float* dy, int lddy,
                    float* dw, float* db, int accumulate, void* workspace, size_t ws_bytes,
                    void* stream) {
  int st = validate(d);
  if (st) return st;
  Geo g = geo(d);
  OF_CHECK_ARG(x && dy && dw && workspace, "conv wgrad: NULL pointer");
  OF_CHECK_ARG(ldx >= d->cin_p && ldx % 4 == 0, "conv wgrad: ldx");
  OF_CHECK_ARG(lddy >= g.cout_p && lddy % 4 == 0, "conv wgrad: lddy");
  WgradPlan p = wgrad_plan(d);
  OF_CHECK_ARG(ws_bytes >= of_conv2d_wgrad_workspace(d), "conv wgrad: workspace too small");
  GemmArgs a = base_args(d);
  a.kc = g.cin_p;
  a.M = p.M;
  a.N = d->cout;
  a.K = d->n * d->ho * d->wo;
  a.A = x;
  a.lda = ldx;
  a.B = dy;
  a.ldb = lddy;
  a.nb = g.cout_p;
  a.C = static_cast<float*>(workspace);
  a.ldc = p.ldc;
  a.k_per_split = p.k_per_split;
  a.split_stride = p.split_stride;
  hipStream_t s = as_stream(stream);
  const double flops = 2.0 * a.K * (double)d->cout * g.taps * d->cin;
  if (timing_on()) timing_begin(s);
  st = launch_cfg<MODE_WGRAD>(a, s, p.splits);
  if (timing_on()) timing_end(s, 2, flops);
  if (st) return st;
  {
    const int64_t total = (int64_t)g.taps * d->cin * d->cout;
    const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 4096);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, s,
                       static_cast<const float*>(workspace), p.splits, p.split_stride, g.taps,
                       g.cin_p, d->cin, d->cout, p.ldc, dw, accumulate);
    if ((st = check_launch("wgrad_reduce"))) return st;
  }
  if (db) {
    // bias gradient = column sums of dy; reuse the (now consumed) slab workspace.
    st = of_colsum(dy, a.K, d->cout, lddy, db, accumulate, workspace, stream);
  }
  return st;
}

}  // extern "C"
