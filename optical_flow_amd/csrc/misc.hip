// Channel reductions, BN/ReLU backward, max-pool, Keras Adam, elementwise helpers.
#include "common.h"

namespace oflow {

// ------------------------------------------------------------------ column reductions --
// Per-channel sums over pixels of NHWC data.  Pass 1: RED_BLOCKS-ish workgroups, each owns a
// contiguous pixel range; threads = (channel quad q) x (pixel row r), float4 loads (16 B/lane,
// a wave reads whole contiguous pixel rows), 4 pixels in flight per thread; the workgroup
// writes one partial row.  Pass 2: every channel's partial rows summed in a fixed order by a
// 64-channel x 4-row workgroup -> bitwise reproducible, no atomics.
#ifndef RED_BLOCKS
#define RED_BLOCKS 512
#endif
#ifndef MPB_BATCH
#define MPB_BATCH 1
#endif
#ifndef BNP_BATCH
#define BNP_BATCH 1
#endif
#ifndef BNP_UNROLL
#define BNP_UNROLL 4   // 4 pixel rows of 3 float4 loads in flight per thread (2: -8 % on the step's BN backward)
#endif
#ifndef MPB_UNROLL
#define MPB_UNROLL 2   // the stem's max-pool + BN backward: 2 pooled pixels (18 float4 loads) in flight
#endif
constexpr int RED_TARGET_BLOCKS = RED_BLOCKS;

struct RedGeo {
  int qw;       // channel quads per row (<= 64)
  int rows;     // pixel rows per workgroup (256 / qw)
  int nblk;     // workgroups along pixels
  int64_t ppb;  // pixels per workgroup (multiple of rows)
};

inline RedGeo red_geo(int64_t npix, int c) {
  RedGeo g;
  const int cq = (c + 3) / 4;
  g.qw = 1;
  while (g.qw < cq && g.qw < 64) g.qw <<= 1;
  g.rows = 256 / g.qw;
  const int64_t min_ppb = (int64_t)g.rows * 8;
  int64_t nb = std::min<int64_t>(RED_TARGET_BLOCKS, cdiv(npix, min_ppb));
  nb = std::max<int64_t>(nb, 1);
  g.ppb = round_up(cdiv(npix, nb), g.rows);
  g.nblk = (int)cdiv(npix, g.ppb);
  return g;
}

__device__ __forceinline__ float4 ld4(const float* p, int valid) {
  // valid = number of the 4 channels that exist (1..4)
  if (valid >= 4) return *reinterpret_cast<const float4*>(p);
  float t[4] = {0.f, 0.f, 0.f, 0.f};
  for (int e = 0; e < valid; ++e) t[e] = p[e];
  return make_float4(t[0], t[1], t[2], t[3]);
}

__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

// Sum the `rows` per-row float4 accumulators of a workgroup through LDS; row 0 threads get
// the total.
__device__ __forceinline__ float4 rows_reduce(float4 v, int q, int r, int qw, int rows,
                                             float4* red) {
  red[r * qw + q] = v;
  __syncthreads();
  for (int s = rows / 2; s > 0; s >>= 1) {
    if (r < s) {
      float4 o = red[(r + s) * qw + q];
      add4(v, o);
      red[r * qw + q] = v;
    }
    __syncthreads();
  }
  return v;
}

__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ x,
                                                             int64_t npix, int c, int ld,
                                                             int qw, int rows, int64_t ppb,
                                                             int vec, float* __restrict__ part) {
  __shared__ float4 red[256];
  const int q = threadIdx.x % qw, r = threadIdx.x / qw;
  const int ch = (blockIdx.y * qw + q) * 4;
  const int64_t p0 = (int64_t)blockIdx.x * ppb;
  const int64_t p1 = min(npix, p0 + ppb);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int valid = min(4, c - ch);
  if (valid > 0) {
    int64_t p = p0 + r;
    for (; p + 3 * rows < p1; p += 4 * rows) {
      float4 a = vec ? ld4(x + p * ld + ch, 4) : ld4(x + p * ld + ch, valid);
      float4 b = vec ? ld4(x + (p + rows) * ld + ch, 4) : ld4(x + (p + rows) * ld + ch, valid);
      float4 cc = vec ? ld4(x + (p + 2 * rows) * ld + ch, 4)
                      : ld4(x + (p + 2 * rows) * ld + ch, valid);
      float4 d = vec ? ld4(x + (p + 3 * rows) * ld + ch, 4)
                     : ld4(x + (p + 3 * rows) * ld + ch, valid);
      add4(a, b);
      add4(cc, d);
      add4(a, cc);
      add4(acc, a);
    }
    for (; p < p1; p += rows) add4(acc, vec ? ld4(x + p * ld + ch, 4) : ld4(x + p * ld + ch, valid));
  }
  acc = rows_reduce(acc, q, r, qw, rows, red);
  if (r == 0 && valid > 0) {
    float* o = part + (int64_t)blockIdx.x * c + ch;
    const float v[4] = {acc.x, acc.y, acc.z, acc.w};
    for (int e = 0; e < valid; ++e) o[e] = v[e];
  }
}

// Sum `nparts` partial rows of `stride` floats (first c channels) in fixed order.
// grid.x = cdiv(c, 16); 256 threads = 16 channels x 16 row groups (many loads in flight).
__global__ __launch_bounds__(256) void rows_final_kernel(const float* __restrict__ part,
                                                         int nparts, int64_t stride, int c,
                                                         float* __restrict__ out, int accum) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int ch = blockIdx.x * 16 + cl;
  float s0 = 0.f, s1 = 0.f;
  if (ch < c) {
    int b = g;
    for (; b + 16 < nparts; b += 32) {
      s0 += part[(int64_t)b * stride + ch];
      s1 += part[(int64_t)(b + 16) * stride + ch];
    }
    for (; b < nparts; b += 16) s0 += part[(int64_t)b * stride + ch];
  }
  red[g][cl] = s0 + s1;
  __syncthreads();
  if (g == 0 && ch < c) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    out[ch] = accum ? out[ch] + t : t;
  }
}

// BN(inference)+residual+act backward, fused with its channel reductions:
// dt = dy*act'(y); dz = dt*gamma*invstd; dres = dt; partial sums of dt and dt*(z-mean)*invstd.
// Dense [npix][c] tensors, c % 4 == 0.
// FROM_Y: z (the conv output before BN) is not stored; the normalised value is recovered from
// the layer output y wherever the gradient is non-zero: y = act(gamma zhat + beta + res), so
// zhat = (y - res - beta) / gamma where act' != 0 (ReLU: y > 0; none: everywhere).  dz may
// then be NULL (the BN scale is folded into the conv's packed dgrad weights and its weight-
// gradient reduction: of_conv_pack_weights_bn, of_conv2d_wgrad_bn), dres receives t.
template <bool FROM_Y>
__global__ __launch_bounds__(256) void bn_act_bwd_partial(
    int64_t npix, int c, int act, const float* __restrict__ dy, const float* __restrict__ y,
    const float* __restrict__ z, const float* __restrict__ res, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ mean,
    const float* __restrict__ var, float eps, float* __restrict__ dz, float* __restrict__ dres,
    int qw, int rows, int64_t ppb, float* __restrict__ part) {
  __shared__ float4 red[256];
  const int q = threadIdx.x % qw, r = threadIdx.x / qw;
  const int ch = (blockIdx.y * qw + q) * 4;
  const int64_t p0 = (int64_t)blockIdx.x * ppb;
  const int64_t p1 = min(npix, p0 + ppb);
  float4 sb = make_float4(0.f, 0.f, 0.f, 0.f), sg = sb;
  const bool live = ch < c;
  if (live) {
    const float4 gm = *reinterpret_cast<const float4*>(gamma + ch);
    const float4 mu = *reinterpret_cast<const float4*>(mean + ch);
    const float4 vr = *reinterpret_cast<const float4*>(var + ch);
    const float4 is = make_float4(rsqrtf(vr.x + eps), rsqrtf(vr.y + eps), rsqrtf(vr.z + eps),
                                  rsqrtf(vr.w + eps));
    const float4 sc = make_float4(gm.x * is.x, gm.y * is.y, gm.z * is.z, gm.w * is.w);
    float4 bt = make_float4(0.f, 0.f, 0.f, 0.f), ig = bt;
    if (FROM_Y) {
      bt = *reinterpret_cast<const float4*>(beta + ch);
      ig = make_float4(1.f / gm.x, 1.f / gm.y, 1.f / gm.z, 1.f / gm.w);
    }
    const bool relu = act == OF_ACT_RELU;
    // BNP_UNROLL pixel rows per round, every load of the round issued before any use: buffer
    // loads on resources based at this block's first pixel (a row past the block's range, or
    // a null tensor, reads 0 -> t = 0 and adds nothing; its stores are dropped).  The pointer
    // form (kept for blocks of 2 GB and more, and as BNP_BATCH=0) put each row's res load and
    // dz / dres stores behind a branch, and the compiler then waited for every load in flight
    // (vmcnt(0)) once per row.
    const int64_t nb = (p1 - p0) * c * 4;              // this block's bytes per tensor
    if (BNP_BATCH && nb < (int64_t)kOOB) {
      const int64_t ob = p0 * c;
      const rsrc_t rdy = make_rsrc(dy + ob, nb), ry = make_rsrc(y + ob, nb);
      const rsrc_t rx = FROM_Y ? make_rsrc(res ? res + ob : dy, res ? nb : 0)
                               : make_rsrc(z + ob, nb);
      const rsrc_t rdz = make_rsrc(dz ? dz + ob : dy, dz ? nb : 0);
      const rsrc_t rdr = make_rsrc(dres ? dres + ob : dy, dres ? nb : 0);
      const int np = (int)(p1 - p0);
      constexpr int U = BNP_UNROLL;
      for (int pl = r; pl < np; pl += U * rows) {
        uint32_t off[U];
        float4 g[U], yy[U], xx[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int pu = pl + u * rows;
          off[u] = pu < np ? (uint32_t)(pu * c + ch) * 4u : kOOB;
          g[u] = bload4(rdy, off[u]);
          yy[u] = bload4(ry, off[u]);
          xx[u] = bload4(rx, off[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float4 zh;
          if (FROM_Y)
            zh = make_float4((yy[u].x - xx[u].x - bt.x) * ig.x, (yy[u].y - xx[u].y - bt.y) * ig.y,
                             (yy[u].z - xx[u].z - bt.z) * ig.z, (yy[u].w - xx[u].w - bt.w) * ig.w);
          else
            zh = make_float4((xx[u].x - mu.x) * is.x, (xx[u].y - mu.y) * is.y,
                             (xx[u].z - mu.z) * is.z, (xx[u].w - mu.w) * is.w);
          float4 t;
          t.x = (!relu || yy[u].x > 0.f) ? g[u].x : 0.f;
          t.y = (!relu || yy[u].y > 0.f) ? g[u].y : 0.f;
          t.z = (!relu || yy[u].z > 0.f) ? g[u].z : 0.f;
          t.w = (!relu || yy[u].w > 0.f) ? g[u].w : 0.f;
          bstore4(make_float4(t.x * sc.x, t.y * sc.y, t.z * sc.z, t.w * sc.w), rdz, off[u]);
          bstore4(t, rdr, off[u]);
          add4(sb, t);
          sg.x += t.x * zh.x;
          sg.y += t.y * zh.y;
          sg.z += t.z * zh.z;
          sg.w += t.w * zh.w;
        }
      }
    } else {
  #pragma unroll BNP_UNROLL
      for (int64_t p = p0 + r; p < p1; p += rows) {
        const int64_t o = p * c + ch;
        const float4 g = *reinterpret_cast<const float4*>(dy + o);
        const float4 yy = *reinterpret_cast<const float4*>(y + o);
        float4 zh;                                   // normalised pre-BN value
        if (FROM_Y) {
          const float4 rr = res ? *reinterpret_cast<const float4*>(res + o)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
          zh = make_float4((yy.x - rr.x - bt.x) * ig.x, (yy.y - rr.y - bt.y) * ig.y,
                           (yy.z - rr.z - bt.z) * ig.z, (yy.w - rr.w - bt.w) * ig.w);
        } else {
          const float4 zz = *reinterpret_cast<const float4*>(z + o);
          zh = make_float4((zz.x - mu.x) * is.x, (zz.y - mu.y) * is.y, (zz.z - mu.z) * is.z,
                           (zz.w - mu.w) * is.w);
        }
        float4 t;
        t.x = (!relu || yy.x > 0.f) ? g.x : 0.f;
        t.y = (!relu || yy.y > 0.f) ? g.y : 0.f;
        t.z = (!relu || yy.z > 0.f) ? g.z : 0.f;
        t.w = (!relu || yy.w > 0.f) ? g.w : 0.f;
        if (dz)
          *reinterpret_cast<float4*>(dz + o) =
              make_float4(t.x * sc.x, t.y * sc.y, t.z * sc.z, t.w * sc.w);
        if (dres) *reinterpret_cast<float4*>(dres + o) = t;
        add4(sb, t);
        sg.x += t.x * zh.x;
        sg.y += t.y * zh.y;
        sg.z += t.z * zh.z;
        sg.w += t.w * zh.w;
      }
    }
  }
  sb = rows_reduce(sb, q, r, qw, rows, red);
  __syncthreads();
  sg = rows_reduce(sg, q, r, qw, rows, red);
  if (r == 0 && live) {
    *reinterpret_cast<float4*>(part + ((int64_t)blockIdx.x * 2 + 0) * c + ch) = sb;
    *reinterpret_cast<float4*>(part + ((int64_t)blockIdx.x * 2 + 1) * c + ch) = sg;
  }
}


// Stem backward in one pass (reset18_encoder's conv1 -> layer1_bn -> ReLU -> {out0, max-pool},
// model.py:12-17): the max-pool gradient (first maximum of each 2x2 window, strict >, as
// maxpool2_bwd_kernel) plus g, the gradient of out0 from its other consumer, then the
// BN(inference)+ReLU backward and its channel sums -- one read of y, z, g and the pooled dy,
// one write of dz, instead of max-pool backward + add + bn_act_bwd (three passes over the
// largest activation of the encoder).  Pixels are 2x2 windows: npix = n*(h/2)*(w/2).
template <bool FROM_Y>     // (z not stored: zhat = (y - beta) / gamma where y > 0, as above)
__global__ __launch_bounds__(256) void maxpool_bn_act_bwd_partial(
    int64_t npix, int h, int w, int c, const float* __restrict__ dyp,
    const float* __restrict__ g, const float* __restrict__ y, const float* __restrict__ z,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ mean, const float* __restrict__ var, float eps,
    float* __restrict__ dz, int qw, int rows, int64_t ppb, float* __restrict__ part) {
  __shared__ float4 red[256];
  const int q = threadIdx.x % qw, r = threadIdx.x / qw;
  const int ch = (blockIdx.y * qw + q) * 4;
  const int64_t p0 = (int64_t)blockIdx.x * ppb;
  const int64_t p1 = min(npix, p0 + ppb);
  float4 sb = make_float4(0.f, 0.f, 0.f, 0.f), sg = sb;
  const bool live = ch < c;
  const int ho = h / 2, wo = w / 2;
  if (live) {
    const float4 gm = *reinterpret_cast<const float4*>(gamma + ch);
    const float4 mu = *reinterpret_cast<const float4*>(mean + ch);
    const float4 vr = *reinterpret_cast<const float4*>(var + ch);
    const float4 is = make_float4(rsqrtf(vr.x + eps), rsqrtf(vr.y + eps), rsqrtf(vr.z + eps),
                                  rsqrtf(vr.w + eps));
    const float4 sc = make_float4(gm.x * is.x, gm.y * is.y, gm.z * is.z, gm.w * is.w);
    float4 bt = make_float4(0.f, 0.f, 0.f, 0.f), ig = bt;
    if (FROM_Y) {
      bt = *reinterpret_cast<const float4*>(beta + ch);
      ig = make_float4(1.f / gm.x, 1.f / gm.y, 1.f / gm.z, 1.f / gm.w);
    }
    // window cursor (b, oy, ox) of p, stepped by `rows` without a division per pixel (64-bit
    // divisions, three per pooled pixel, made this kernel ALU-bound at ~2.1 TB/s)
    int ox = (int)((p0 + r) % wo), oy = (int)((p0 + r) / wo % ho);
    int64_t b = (p0 + r) / wo / ho;
    const int dox = rows % wo, doy = rows / wo;
    // Batched form (MPB_BATCH): MPB_UNROLL pooled pixels per round, their 9 loads each issued
    // before any use, on buffer resources based at the block's first full-resolution row (a
    // pixel past the block, or a null g, reads 0 and its dz stores are dropped).  The pointer
    // form below put g's loads behind a branch and waited for all loads once per pixel.
    // The block's full-resolution span: at most (its pooled rows + 2) x 2 image rows.
    const int64_t e0 = ((p0 / wo) * 2) * (int64_t)w * c;   // (b, 2 oy0, 0, 0): p0 / wo = b ho + oy0
    const int64_t span = ((p1 - p0) / wo + 2) * 2 * (int64_t)w * c * 4;
    if (MPB_BATCH && span < (int64_t)kOOB && (p1 - p0) * c * 4 < (int64_t)kOOB) {
      const int64_t tot = npix * 4 * c * 4 - e0 * 4;   // bytes of y from e0 to the end
      const int64_t nb = min(tot, span);
      const rsrc_t ry = make_rsrc(y + e0, nb), rg = make_rsrc(g ? g + e0 : y, g ? nb : 0);
      const rsrc_t rz = make_rsrc(FROM_Y ? y : z + e0, FROM_Y ? 0 : nb);
      const rsrc_t rdz = make_rsrc(dz + e0, nb);
      const rsrc_t rd = make_rsrc(dyp + p0 * c, (p1 - p0) * c * 4);
      const int np = (int)(p1 - p0);
      constexpr int U = MPB_UNROLL;
      for (int pl = r; pl < np; pl += U * rows) {
        uint32_t o[U], od[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool in = pl + u * rows < np;
          o[u] = in ? (uint32_t)(((b * h + 2 * oy) * (int64_t)w + 2 * ox) * c + ch - e0) * 4u : kOOB;
          od[u] = in ? (uint32_t)((pl + u * rows) * c + ch) * 4u : kOOB;
          ox += dox;
          oy += doy;
          if (ox >= wo) ox -= wo, ++oy;
          while (oy >= ho) oy -= ho, ++b;
        }
        const uint32_t dxo = (uint32_t)c * 4u, dyo = (uint32_t)w * c * 4u;
        auto at = [&](uint32_t base, int k) {           // corner k of a window (kOOB stays out)
          return base == kOOB ? kOOB : base + (k & 1 ? dxo : 0u) + (k & 2 ? dyo : 0u);
        };
        float4 yv[U][4], gv[U][4], zr[U][4], d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            yv[u][k] = bload4(ry, at(o[u], k));
            gv[u][k] = bload4(rg, at(o[u], k));
            if (!FROM_Y) zr[u][k] = bload4(rz, at(o[u], k));
          }
          d[u] = bload4(rd, od[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          int bx = 0, by = 0, bz = 0, bw = 0;           // first maximum per channel
          float4 mx = yv[u][0];
#pragma unroll
          for (int k = 1; k < 4; ++k) {
            if (yv[u][k].x > mx.x) bx = k, mx.x = yv[u][k].x;
            if (yv[u][k].y > mx.y) by = k, mx.y = yv[u][k].y;
            if (yv[u][k].z > mx.z) bz = k, mx.z = yv[u][k].z;
            if (yv[u][k].w > mx.w) bw = k, mx.w = yv[u][k].w;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float4 yk = yv[u][k];
            float4 zk;
            if (FROM_Y)
              zk = make_float4((yk.x - bt.x) * ig.x, (yk.y - bt.y) * ig.y, (yk.z - bt.z) * ig.z,
                               (yk.w - bt.w) * ig.w);
            else
              zk = make_float4((zr[u][k].x - mu.x) * is.x, (zr[u][k].y - mu.y) * is.y,
                               (zr[u][k].z - mu.z) * is.z, (zr[u][k].w - mu.w) * is.w);
            float4 t;
            t.x = yk.x > 0.f ? gv[u][k].x + (k == bx ? d[u].x : 0.f) : 0.f;
            t.y = yk.y > 0.f ? gv[u][k].y + (k == by ? d[u].y : 0.f) : 0.f;
            t.z = yk.z > 0.f ? gv[u][k].z + (k == bz ? d[u].z : 0.f) : 0.f;
            t.w = yk.w > 0.f ? gv[u][k].w + (k == bw ? d[u].w : 0.f) : 0.f;
            bstore4(make_float4(t.x * sc.x, t.y * sc.y, t.z * sc.z, t.w * sc.w), rdz, at(o[u], k));
            add4(sb, t);
            sg.x += t.x * zk.x;
            sg.y += t.y * zk.y;
            sg.z += t.z * zk.z;
            sg.w += t.w * zk.w;
          }
        }
      }
    } else {
  #pragma unroll MPB_UNROLL
      for (int64_t p = p0 + r; p < p1; p += rows) {
        const int64_t o0 = ((b * h + 2 * oy) * (int64_t)w + 2 * ox) * c + ch;
        ox += dox;
        oy += doy;
        if (ox >= wo) ox -= wo, ++oy;
        while (oy >= ho) oy -= ho, ++b;
        const int64_t offs[4] = {o0, o0 + c, o0 + (int64_t)w * c, o0 + (int64_t)w * c + c};
        float4 yv[4], zv[4], gv[4];
  #pragma unroll
        for (int k = 0; k < 4; ++k) {
          yv[k] = *reinterpret_cast<const float4*>(y + offs[k]);
          gv[k] = g ? *reinterpret_cast<const float4*>(g + offs[k]) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
  #pragma unroll
        for (int k = 0; k < 4; ++k) {   // zv: the normalised pre-BN values
          if (FROM_Y) {
            zv[k] = make_float4((yv[k].x - bt.x) * ig.x, (yv[k].y - bt.y) * ig.y,
                                (yv[k].z - bt.z) * ig.z, (yv[k].w - bt.w) * ig.w);
          } else {
            const float4 zz = *reinterpret_cast<const float4*>(z + offs[k]);
            zv[k] = make_float4((zz.x - mu.x) * is.x, (zz.y - mu.y) * is.y, (zz.z - mu.z) * is.z,
                                (zz.w - mu.w) * is.w);
          }
        }
        const float4 d = *reinterpret_cast<const float4*>(dyp + p * c + ch);
        // first maximum per channel (the running maxima kept as values: indexing yv by the
        // running argmax made the arrays dynamically indexed, and the compiler put them in LDS
        // with a wait after every load -- four serial memory round trips per pooled pixel)
        int bx = 0, by = 0, bz = 0, bw = 0;
        float4 mx = yv[0];
  #pragma unroll
        for (int k = 1; k < 4; ++k) {
          if (yv[k].x > mx.x) bx = k, mx.x = yv[k].x;
          if (yv[k].y > mx.y) by = k, mx.y = yv[k].y;
          if (yv[k].z > mx.z) bz = k, mx.z = yv[k].z;
          if (yv[k].w > mx.w) bw = k, mx.w = yv[k].w;
        }
  #pragma unroll
        for (int k = 0; k < 4; ++k) {
          float4 t;
          t.x = yv[k].x > 0.f ? gv[k].x + (k == bx ? d.x : 0.f) : 0.f;
          t.y = yv[k].y > 0.f ? gv[k].y + (k == by ? d.y : 0.f) : 0.f;
          t.z = yv[k].z > 0.f ? gv[k].z + (k == bz ? d.z : 0.f) : 0.f;
          t.w = yv[k].w > 0.f ? gv[k].w + (k == bw ? d.w : 0.f) : 0.f;
          *reinterpret_cast<float4*>(dz + offs[k]) =
              make_float4(t.x * sc.x, t.y * sc.y, t.z * sc.z, t.w * sc.w);
          add4(sb, t);
          sg.x += t.x * zv[k].x;
          sg.y += t.y * zv[k].y;
          sg.z += t.z * zv[k].z;
          sg.w += t.w * zv[k].w;
        }
      }
    }
  }
  sb = rows_reduce(sb, q, r, qw, rows, red);
  __syncthreads();
  sg = rows_reduce(sg, q, r, qw, rows, red);
  if (r == 0 && live) {
    *reinterpret_cast<float4*>(part + ((int64_t)blockIdx.x * 2 + 0) * c + ch) = sb;
    *reinterpret_cast<float4*>(part + ((int64_t)blockIdx.x * 2 + 1) * c + ch) = sg;
  }
}

// Sum the partial rows of bn_act_bwd_partial / maxpool_bn_act_bwd_partial in a fixed order:
// workgroup = BNF_Q channel quads x 64 row groups (grid.x = cdiv(c / 4, BNF_Q)); each thread
// sums its rows with 8 float4 loads in flight, then a fixed tree over the 64 groups.
// (A 16-row-group form with one scalar load in flight per step took 15 us per call: latency.)
// BNF_Q = 1: one wave per channel quad.  The round-2..4 form (BNF_Q = 16, one 1024-thread
// workgroup for c = 64) ran these side-stream reductions at 8 us alone but 70-80 us beside a
// main-stream convolution, its 16 waves waiting for a CU with that much room; a 64-thread
// workgroup fits in any gap.  Same per-channel order, so the results are bitwise unchanged.
#ifndef BNF_QW
#define BNF_QW 1
#endif
constexpr int BNF_Q = BNF_QW, BNF_G = 64;
__global__ __launch_bounds__(BNF_Q * BNF_G) void bn_act_bwd_final(const float* __restrict__ part,
                                                                  int nblk, int c,
                                                                  const float* __restrict__ gamma,
                                                                  const float* __restrict__ var,
                                                                  float eps, float* __restrict__ dgamma,
                                                                  float* __restrict__ dbeta,
                                                                  float* __restrict__ dbias, int accum) {
  __shared__ float4 red[2][BNF_G][BNF_Q];
  const int ql = threadIdx.x % BNF_Q, g = threadIdx.x / BNF_Q;
  const int ch = (blockIdx.x * BNF_Q + ql) * 4;
  float4 sb = make_float4(0.f, 0.f, 0.f, 0.f), sg = sb;
  if (ch < c) {
    int b = g;
    for (; b + 3 * BNF_G < nblk; b += 4 * BNF_G) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[2 * u] = *reinterpret_cast<const float4*>(part + ((int64_t)(b + u * BNF_G) * 2 + 0) * c + ch);
        v[2 * u + 1] = *reinterpret_cast<const float4*>(part + ((int64_t)(b + u * BNF_G) * 2 + 1) * c + ch);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        add4(sb, v[2 * u]);
        add4(sg, v[2 * u + 1]);
      }
    }
    for (; b < nblk; b += BNF_G) {
      add4(sb, *reinterpret_cast<const float4*>(part + ((int64_t)b * 2 + 0) * c + ch));
      add4(sg, *reinterpret_cast<const float4*>(part + ((int64_t)b * 2 + 1) * c + ch));
    }
  }
  red[0][g][ql] = sb;
  red[1][g][ql] = sg;
  __syncthreads();
  for (int s = BNF_G / 2; s > 0; s >>= 1) {
    if (g < s) {
      add4(sb, red[0][g + s][ql]);
      add4(sg, red[1][g + s][ql]);
      red[0][g][ql] = sb;
      red[1][g][ql] = sg;
    }
    __syncthreads();
  }
  if (g == 0 && ch < c) {
    const float vb[4] = {sb.x, sb.y, sb.z, sb.w}, vg[4] = {sg.x, sg.y, sg.z, sg.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = ch + e;
      const float db = vb[e] * gamma[k] * rsqrtf(var[k] + eps);
      if (dbeta) dbeta[k] = accum ? dbeta[k] + vb[e] : vb[e];
      if (dgamma) dgamma[k] = accum ? dgamma[k] + vg[e] : vg[e];
      if (dbias) dbias[k] = accum ? dbias[k] + db : db;
    }
  }
}

// ------------------------------------------------------------------------- max pool ----
// I: the index type -- 32-bit unsigned whenever the element count fits (64-bit division is a
// software routine of ~100 instructions, and three of them per element made this kernel
// ALU-bound at ~2.6 TB/s).
template <typename I>
__global__ __launch_bounds__(256) void maxpool2_fwd_kernel(const float* __restrict__ x, int n,
                                                           int h, int w, int c,
                                                           float* __restrict__ y) {
  const I ho = h / 2, wo = w / 2, cq = c / 4;
  const I total = (I)n * ho * wo * cq;
  for (I idx = blockIdx.x * (I)blockDim.x + threadIdx.x; idx < total;
       idx += (I)gridDim.x * blockDim.x) {
    const int q = (int)(idx % cq);
    const I p = idx / cq;
    const int ox = (int)(p % wo);
    const I t2 = p / wo;
    const int oy = (int)(t2 % ho);
    const int64_t b = (int64_t)(t2 / ho);
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
    *reinterpret_cast<float4*>(y + (int64_t)p * c + 4 * q) = r;
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

// Device-resident schedule for a graph-captured step: sched[0] = lr (set by the host between
// steps), sched[1] <- lr_t of the step about to run; *iter counts applied updates.  One
// thread, launched right before adam_dev_kernel, so a replayed graph advances t by itself.
__global__ void adam_sched_kernel(float* __restrict__ sched, int32_t* __restrict__ iter,
                                  float b1, float b2) {
  const int t = *iter + 1;
  *iter = t;
  const double lr = sched[0];
  sched[1] = (float)(lr * sqrt(1.0 - pow((double)b2, (double)t)) / (1.0 - pow((double)b1, (double)t)));
}

__global__ __launch_bounds__(256) void adam_dev_kernel(float* __restrict__ p,
                                                       const float* __restrict__ g,
                                                       float* __restrict__ m,
                                                       float* __restrict__ v, int64_t n,
                                                       const float* __restrict__ sched, float b1,
                                                       float b2, float eps, float gs) {
  const float lr_t = sched[1];
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
  return (size_t)red_geo(npix, c).nblk * c * sizeof(float);
}

int of_colsum(const float* x, int64_t npix, int c, int ld, float* out, int accumulate,
              void* workspace, void* stream) {
  OF_CHECK_ARG(x && out && workspace && ld >= c && c > 0 && npix > 0, "colsum: args");
  hipStream_t s = as_stream(stream);
  const RedGeo g = red_geo(npix, c);
  const int vec = (c % 4 == 0 && ld % 4 == 0 && ((uintptr_t)x & 15) == 0) ? 1 : 0;
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(g.nblk, cdiv(cdiv(c, 4), g.qw)), dim3(256), 0,
                     s, x, npix, c, ld, g.qw, g.rows, g.ppb, vec, part);
  int st = check_launch("colsum_partial");
  if (st) return st;
  hipLaunchKernelGGL(rows_final_kernel, dim3(cdiv(c, 16)), dim3(256), 0, s, part, g.nblk,
                     (int64_t)c, c, out, accumulate);
  return check_launch("colsum_final");
}

size_t of_bn_act_bwd_workspace(int64_t npix, int c) {
  return (size_t)red_geo(npix, c).nblk * 2 * c * sizeof(float);
}

int of_bn_act_bwd(int64_t npix, int c, int act, const float* dy, const float* y,
                  const float* z, const float* gamma, const float* mean, const float* var,
                  float eps, float* dz, float* dres, float* dgamma, float* dbeta, float* dbias,
                  int accumulate, void* workspace, void* stream) {
  OF_CHECK_ARG(dy && y && z && gamma && mean && var && workspace, "bn_act_bwd: args");
  OF_CHECK_ARG(act == OF_ACT_NONE || act == OF_ACT_RELU, "bn_act_bwd: act must be none/relu");
  OF_CHECK_ARG(c % 4 == 0 && npix > 0, "bn_act_bwd: c must be a multiple of 4");
  OF_CHECK_ARG((((uintptr_t)dy | (uintptr_t)y | (uintptr_t)z | (uintptr_t)dz |
                 (uintptr_t)dres | (uintptr_t)gamma | (uintptr_t)mean | (uintptr_t)var) & 15) == 0,
               "bn_act_bwd: 16-byte alignment");
  hipStream_t s = as_stream(stream);
  const RedGeo g = red_geo(npix, c);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(bn_act_bwd_partial<false>, dim3(g.nblk, cdiv(c / 4, g.qw)), dim3(256), 0, s,
                     npix, c, act, dy, y, z, nullptr, gamma, nullptr, mean, var, eps, dz, dres,
                     g.qw, g.rows, g.ppb, part);
  int st = check_launch("bn_act_bwd_partial");
  if (st) return st;
  hipLaunchKernelGGL(bn_act_bwd_final, dim3(cdiv(c / 4, BNF_Q)), dim3(BNF_Q * BNF_G), 0, s, part,
                     g.nblk, c, gamma, var, eps, dgamma, dbeta, dbias, accumulate);
  return check_launch("bn_act_bwd_final");
}


// The final pass alone, over partial rows another kernel wrote in bn_act_bwd_partial's
// layout ([nblk][2][c]: sum t, sum t zhat) -- the input-gradient epilogue's fused partial sums
// (of_conv2d_dgrad_add_act_bnp).
int of_bn_bwd_final(const float* part, int nblk, int c, const float* gamma, const float* var,
                    float eps, float* dgamma, float* dbeta, float* dbias, int accumulate,
                    void* stream) {
  OF_CHECK_ARG(part && gamma && var && nblk > 0 && c % 4 == 0, "bn_bwd_final: args");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(bn_act_bwd_final, dim3(cdiv(c / 4, BNF_Q)), dim3(BNF_Q * BNF_G), 0, s, part,
                     nblk, c, gamma, var, eps, dgamma, dbeta, dbias, accumulate);
  return check_launch("bn_bwd_final");
}

// min |x| over each of nseg segments (the BN gammas of a network, ptrs / lens in device
// memory): one workgroup per segment, a fixed-order reduction.
__global__ __launch_bounds__(256) void min_abs_segments_kernel(const float* const* ptrs,
                                                               const int* lens,
                                                               float* __restrict__ out) {
  __shared__ float red[256];
  const float* p = ptrs[blockIdx.x];
  const int n = lens[blockIdx.x];
  float m = INFINITY;
  for (int i = threadIdx.x; i < n; i += 256) m = fminf(m, fabsf(p[i]));
  red[threadIdx.x] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = fminf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

int of_min_abs_segments(const float* const* dev_ptrs, const int* dev_lens, int nseg, float* out,
                        void* stream) {
  OF_CHECK_ARG(dev_ptrs && dev_lens && out && nseg > 0, "min_abs_segments: args");
  hipLaunchKernelGGL(min_abs_segments_kernel, dim3(nseg), dim3(256), 0, as_stream(stream),
                     dev_ptrs, dev_lens, out);
  return check_launch("min_abs_segments");
}

size_t of_maxpool_bn_act_bwd_workspace(int n, int h, int w, int c) {
  return of_bn_act_bwd_workspace((int64_t)n * (h / 2) * (w / 2), c);
}

int of_maxpool_bn_act_bwd(int n, int h, int w, int c, const float* dyp, const float* g,
                          const float* y, const float* z, const float* gamma, const float* mean,
                          const float* var, float eps, float* dz, float* dgamma, float* dbeta,
                          float* dbias, int accumulate, void* workspace, void* stream) {
  OF_CHECK_ARG(dyp && y && z && gamma && mean && var && dz && workspace,
               "maxpool_bn_act_bwd: args");
  OF_CHECK_ARG(n > 0 && h % 2 == 0 && w % 2 == 0 && h > 0 && w > 0 && c % 4 == 0,
               "maxpool_bn_act_bwd: even h, w and c % 4 == 0");
  OF_CHECK_ARG((((uintptr_t)dyp | (uintptr_t)g | (uintptr_t)y | (uintptr_t)z | (uintptr_t)dz |
                 (uintptr_t)gamma | (uintptr_t)mean | (uintptr_t)var) & 15) == 0,
               "maxpool_bn_act_bwd: 16-byte alignment");
  hipStream_t s = as_stream(stream);
  const int64_t npix = (int64_t)n * (h / 2) * (w / 2);
  const RedGeo geo = red_geo(npix, c);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(maxpool_bn_act_bwd_partial<false>, dim3(geo.nblk, cdiv(c / 4, geo.qw)),
                     dim3(256), 0, s, npix, h, w, c, dyp, g, y, z, gamma, nullptr, mean, var, eps,
                     dz, geo.qw, geo.rows, geo.ppb, part);
  int st = check_launch("maxpool_bn_act_bwd_partial");
  if (st) return st;
  hipLaunchKernelGGL(bn_act_bwd_final, dim3(cdiv(c / 4, BNF_Q)), dim3(BNF_Q * BNF_G), 0, s, part,
                     geo.nblk, c, gamma, var, eps, dgamma, dbeta, dbias, accumulate);
  return check_launch("bn_act_bwd_final");
}

int of_bn_bwd_reduce(int64_t npix, int c, int act, const float* dy, const float* y,
                     const float* res, const float* gamma, const float* beta, const float* var,
                     float eps, float* t_out, float* dgamma, float* dbeta, float* dbias,
                     int accumulate, void* workspace, void* stream) {
  OF_CHECK_ARG(dy && y && gamma && beta && var && workspace, "bn_bwd_reduce: args");
  OF_CHECK_ARG(act == OF_ACT_NONE || act == OF_ACT_RELU, "bn_bwd_reduce: act must be none/relu");
  OF_CHECK_ARG(c % 4 == 0 && npix > 0, "bn_bwd_reduce: c must be a multiple of 4");
  OF_CHECK_ARG((((uintptr_t)dy | (uintptr_t)y | (uintptr_t)res | (uintptr_t)t_out |
                 (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)var) & 15) == 0,
               "bn_bwd_reduce: 16-byte alignment");
  hipStream_t s = as_stream(stream);
  const RedGeo g = red_geo(npix, c);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(bn_act_bwd_partial<true>, dim3(g.nblk, cdiv(c / 4, g.qw)), dim3(256), 0, s,
                     npix, c, act, dy, y, nullptr, res, gamma, beta, nullptr, var, eps, nullptr,
                     t_out, g.qw, g.rows, g.ppb, part);
  int st = check_launch("bn_bwd_reduce");
  if (st) return st;
  hipLaunchKernelGGL(bn_act_bwd_final, dim3(cdiv(c / 4, BNF_Q)), dim3(BNF_Q * BNF_G), 0, s, part,
                     g.nblk, c, gamma, var, eps, dgamma, dbeta, dbias, accumulate);
  return check_launch("bn_act_bwd_final");
}

int of_maxpool_bn_relu_bwd(int n, int h, int w, int c, const float* dyp, const float* g,
                           const float* y, const float* gamma, const float* beta,
                           const float* var, float eps, float* dz, float* dgamma, float* dbeta,
                           float* dbias, int accumulate, void* workspace, void* stream) {
  OF_CHECK_ARG(dyp && y && gamma && beta && var && dz && workspace, "maxpool_bn_relu_bwd: args");
  OF_CHECK_ARG(n > 0 && h % 2 == 0 && w % 2 == 0 && h > 0 && w > 0 && c % 4 == 0,
               "maxpool_bn_relu_bwd: even h, w and c % 4 == 0");
  OF_CHECK_ARG((((uintptr_t)dyp | (uintptr_t)g | (uintptr_t)y | (uintptr_t)dz |
                 (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)var) & 15) == 0,
               "maxpool_bn_relu_bwd: 16-byte alignment");
  hipStream_t s = as_stream(stream);
  const int64_t npix = (int64_t)n * (h / 2) * (w / 2);
  const RedGeo geo = red_geo(npix, c);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(maxpool_bn_act_bwd_partial<true>, dim3(geo.nblk, cdiv(c / 4, geo.qw)),
                     dim3(256), 0, s, npix, h, w, c, dyp, g, y, nullptr, gamma, beta, nullptr,
                     var, eps, dz, geo.qw, geo.rows, geo.ppb, part);
  int st = check_launch("maxpool_bn_relu_bwd_partial");
  if (st) return st;
  hipLaunchKernelGGL(bn_act_bwd_final, dim3(cdiv(c / 4, BNF_Q)), dim3(BNF_Q * BNF_G), 0, s, part,
                     geo.nblk, c, gamma, var, eps, dgamma, dbeta, dbias, accumulate);
  return check_launch("bn_act_bwd_final");
}

int of_maxpool2_fwd(const float* x, int n, int h, int w, int c, float* y, void* stream) {
  OF_CHECK_ARG(x && y && h % 2 == 0 && w % 2 == 0 && c % 4 == 0, "maxpool fwd: args");
  const int64_t total = (int64_t)n * (h / 2) * (w / 2) * (c / 4);
  if (total < (int64_t)UINT32_MAX - (int64_t)grid_of(total) * 256)
    hipLaunchKernelGGL(maxpool2_fwd_kernel<uint32_t>, dim3(grid_of(total)), dim3(256), 0,
                       as_stream(stream), x, n, h, w, c, y);
  else
    hipLaunchKernelGGL(maxpool2_fwd_kernel<int64_t>, dim3(grid_of(total)), dim3(256), 0,
                       as_stream(stream), x, n, h, w, c, y);
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

int of_adam_keras_dev(float* p, const float* g, float* m, float* v, int64_t n, float* sched,
                      int32_t* iter, float beta1, float beta2, float eps, float gscale,
                      void* stream) {
  OF_CHECK_ARG(p && g && m && v && sched && iter && n >= 0, "adam dev: args");
  OF_CHECK_ARG((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0,
               "adam: arenas must be 16-byte aligned");
  hipLaunchKernelGGL(adam_sched_kernel, dim3(1), dim3(1), 0, as_stream(stream), sched, iter,
                     beta1, beta2);
  if (n > 0)
    hipLaunchKernelGGL(adam_dev_kernel, dim3(std::min<int64_t>(grid_of(n / 4 + 1), 2048)),
                       dim3(256), 0, as_stream(stream), p, g, m, v, n, sched, beta1, beta2, eps,
                       gscale);
  return check_launch("adam dev");
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
