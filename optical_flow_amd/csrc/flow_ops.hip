// Flow-specific HBM-bound kernels: cost volume, bilinear warp (reference convention),
// x2 flow upscale, loss image pyramid, Siamese split, photometric L1 loss.
//
// All NHWC fp32.  Each kernel cites the reference call it replaces.
#include "common.h"

namespace oflow {

// ================================================================ cost volume (K6) =====
// model.py:29-42: cv[p][i*(2d+1)+j] = sum_c f1[p][c] * f2[p + (i-d, j-d)][c], zero padded.
//
// Blocks own a 4 x 16 pixel tile and one 64-channel slab (blockIdx.z = image * slabs + slab).
// The slab's f2 halo (10 x 22 pixels x 64 channels, 256-B rows: fully coalesced, one load
// round) sits in LDS; each pixel is worked by 4 adjacent lanes, 16 channels each:
//   forward : lane partial dots over its 16 channels for all 49 offsets, quad-reduced with
//             DPP; with more than one slab the partials go to a workspace and a second
//             kernel sums them (fixed order: deterministic).
//   backward: lane owns 16 output channels; the 49 coefficients of its pixel come from a
//             small LDS table (for d/d(f2) gathered with the shift the adjoint needs).
// LDS pixel stride 68 floats: the b128 reads of a wave's lane groups hit distinct banks.
constexpr int CT_Y = 4, CT_X = 16, CT_PIX = CT_Y * CT_X;
constexpr int CSLAB = 64, CSPS = CSLAB + 4;
typedef float f32x2 __attribute__((ext_vector_type(2)));

// 4 fp32 -> 4 bf16 (RNE), element 0 in the low half of .x (as conv_dev.h pack_bf16x4)
__device__ __forceinline__ uint2 pack4_bf16(const float4& v) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 r;
  r[0] = (__bf16)v.x, r[1] = (__bf16)v.y, r[2] = (__bf16)v.z, r[3] = (__bf16)v.w;
  return __builtin_bit_cast(uint2, r);
}

__device__ __forceinline__ float quad_sum(float v) {   // sum over the 4 lanes of a quad
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF,
                                                          0xF, false));   // quad_perm(1,0,3,2)
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF,
                                                          0xF, false));   // quad_perm(2,3,0,1)
  return v;
}

struct CorrFwdArgs {
  const float* f1;
  int ld1;
  const float* f2;
  int ld2;
  int h, w, c;
  float* cv;          // cost volume channel 0 of pixel 0, row stride ldcv
  int ldcv;
  int vec;            // float4 global access allowed (strides and bases 16-byte aligned)
  int slabs;          // ceil(c / 64)
  int tiles_x, tiles_y;
  float* part;        // slabs > 1: partial sums [slab][n*h*w][49]
  // Flow-module concat (model.py:97-102), optional: cat row = [f1 | cv | flow | zero pad].
  float* cat;         // row stride ldcv; cv == cat + c
  const float* flow;  // (.., 2) or NULL
  // or the concat row as a bf16 image (corr_fwd_blk, one slab group): [f1 | cv | flow | 0]
  // with ld16 channels per pixel (cat, cv NULL)
  uint16_t* cat16;
  int ld16;
};

template <int D, bool VEC>
__global__ __launch_bounds__(256, 2) void corr_fwd_kernel(CorrFwdArgs a) {
  constexpr int ND = 2 * D + 1, NK = ND * ND;
  constexpr int HY = CT_Y + 2 * D, HX = CT_X + 2 * D, NH = HY * HX;
  constexpr int NQ = NH * (CSLAB / 4), NU = (NQ + 255) / 256;
  __shared__ float4 lds4[NH * CSPS / 4];
  float* tile = reinterpret_cast<float*>(lds4);
  const int h = a.h, w = a.w;
  // 1-D grid, XCD-aware: neighbouring tiles (shared halo rows) run on one XCD's L2.
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tl = wg % (a.tiles_x * a.tiles_y), z = wg / (a.tiles_x * a.tiles_y);
  const int b = z / a.slabs, slab = z - b * a.slabs;
  const int c_lo = slab * CSLAB, cs = min(CSLAB, a.c - c_lo);
  const int y0 = (tl / a.tiles_x) * CT_Y, x0 = (tl % a.tiles_x) * CT_X;
  const int tid = threadIdx.x;
  const int pix = tid >> 2, qtr = tid & 3;
  const int ty = pix / CT_X, tx = pix % CT_X;
  const int y = y0 + ty, x = x0 + tx;
  const bool valid = y < h && x < w;
  const int64_t img = (int64_t)b * h * w;
  const int pl = y * w + x;
  const rsrc_t r1 = make_rsrc(a.f1 + img * a.ld1, (int64_t)h * w * a.ld1 * 4);
  const rsrc_t r2 = make_rsrc(a.f2 + img * a.ld2, (int64_t)h * w * a.ld2 * 4);
  // One load round: the f2 halo slab and this lane's 16 f1 channels.
  float4 hv[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int q = tid + 256 * u;
    const int hp = q >> 4, cq = q & 15;
    const int sy = y0 - D + hp / HX, sx = x0 - D + hp % HX;
    const bool ok = q < NQ && (unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w;
    hv[u] = bload_quad(r2, ok, 4 * ((sy * w + sx) * a.ld2 + c_lo + 4 * cq), cs - 4 * cq, VEC);
  }
  f32x2 f[8];
  float4 fq[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ch = qtr * 16 + 4 * e;
    fq[e] = bload_quad(r1, valid, 4 * (pl * a.ld1 + c_lo + ch), cs - ch, VEC);
    f[2 * e] = f32x2{fq[e].x, fq[e].y};
    f[2 * e + 1] = f32x2{fq[e].z, fq[e].w};
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int q = tid + 256 * u;
    if (q < NQ) *reinterpret_cast<float4*>(&tile[(q >> 4) * CSPS + 4 * (q & 15)]) = hv[u];
  }
  if (a.cat && valid) {              // f1 slice of the concat row
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ch = qtr * 16 + 4 * e;
      float* dst = a.cat + (img + pl) * a.ldcv + c_lo + ch;
      if (VEC && cs - ch >= 4) {
        *reinterpret_cast<float4*>(dst) = fq[e];
      } else {
        const float t[4] = {fq[e].x, fq[e].y, fq[e].z, fq[e].w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (k < cs - ch) dst[k] = t[k];
      }
    }
  }
  __syncthreads();
  // Packed accumulators: (even, odd) channel partial sums per offset, v_pk_fma_f32 only.
  f32x2 acc[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) acc[k] = f32x2{0.f, 0.f};
  // One channel quad per pass (not unrolled): bounds the LDS reads the scheduler can hoist.
#pragma unroll 1
  for (int e = 0; e < 4; ++e) {
    const f32x2 f0 = e == 0 ? f[0] : e == 1 ? f[2] : e == 2 ? f[4] : f[6];
    const f32x2 f1v = e == 0 ? f[1] : e == 1 ? f[3] : e == 2 ? f[5] : f[7];
    const float* tb = &tile[(ty * HX + tx) * CSPS + qtr * 16 + 4 * e];
#pragma unroll
    for (int i = 0; i < ND; ++i) {
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const f32x2* t = reinterpret_cast<const f32x2*>(tb + (i * HX + j) * CSPS);
        acc[i * ND + j] = __builtin_elementwise_fma(f0, t[0], acc[i * ND + j]);
        acc[i * ND + j] = __builtin_elementwise_fma(f1v, t[1], acc[i * ND + j]);
      }
    }
  }
  // Quad sums -> LDS [pixel][49] (odd stride: conflict-free) -> stores as contiguous runs.
  __syncthreads();                             // halo tile no longer read
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const float v = quad_sum(acc[k].x + acc[k].y);
    if ((k & 3) == qtr) tile[pix * NK + k] = v;
  }
  __syncthreads();
  {
    float* out;
    int64_t ld;
    if (a.slabs == 1) {
      out = a.cv;
      ld = a.ldcv;
    } else {
      const int64_t npix = (int64_t)(gridDim.x / (a.tiles_x * a.tiles_y * a.slabs)) * h * w;
      out = a.part + slab * npix * NK;
      ld = NK;
    }
    for (int q = tid; q < CT_PIX * NK; q += 256) {
      const int p = q / NK, k = q - p * NK;
      const int sy = y0 + p / CT_X, sx = x0 + p % CT_X;
      if (sy < h && sx < w) out[(img + sy * w + sx) * ld + k] = tile[q];
    }
  }
  if (a.cat && slab == 0 && qtr == 0 && valid) {   // flow and zero channel padding
    float* row = a.cat + (img + pl) * a.ldcv;
    int ch = a.c + NK;
    if (a.flow) {
      row[ch] = a.flow[2 * (img + pl)];
      row[ch + 1] = a.flow[2 * (img + pl) + 1];
      ch += 2;
    }
    for (; ch < a.ldcv; ++ch) row[ch] = 0.f;
  }
}

// cv[p][k] = sum over slabs of part[slab][p][k] (slab order fixed).
__global__ __launch_bounds__(256) void corr_slab_sum_kernel(const float* __restrict__ part,
                                                            int slabs, int64_t n, int nk,
                                                            float* __restrict__ cv, int ldcv) {
  const int64_t total = n * nk;
  for (int64_t q = blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    float s = part[q];
    for (int t = 1; t < slabs; ++t) s += part[t * total + q];
    const int64_t p = q / nk;
    cv[p * ldcv + (q - p * nk)] = s;
  }
}

// ---- register-blocked forward (of_set_tuning key 9 = 1, the default) ---------------------
// The form above keeps 2 workgroups of 4 waves per CU, each loading a 60 KB halo and then
// computing, with nothing in flight while it computes: at 192x256x64 it ran 179 us, 4x the
// HBM time of its operands.  Here:
//   * tile 8 x 16 pixels; thread = (4 adjacent pixels of a row, offset row i): 28
//     accumulators (7 column offsets x 4 pixels) over ALL channels, so no cross-lane sums;
//     per channel quad 4 f1 + 10 f2 ds_read_b128 feed 56 v_pk_fma_f32 (the form above: 1:1);
//   * 32-channel slabs; the workgroup is persistent over (tile, slab group) items and the next
//     slab's f1 tile + f2 halo are loaded into registers while the current slab computes;
//   * small levels (few tiles, many channels) split the slabs into groups whose partial sums
//     corr_slab_sum_kernel adds in group order (deterministic).
// LDS: halo rows of 25 pixels (pitch = 1 mod 4) and f1 rows of 17, both 36 floats a pixel:
// the ds_read_b128 lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} hold tile rows with
// distinct (row mod 4), which with 4-pixel column steps puts their 16 pixels on 16 distinct
// 16-byte bank slots.  70 KB: two workgroups per CU.
// Measured (kernel trace, batch 8, concat form): 192x256x64 168 -> 122 us, 96x128x64 46 -> 38,
// 48x64x128 46 -> 22 + 12 (slab sum).  Both forms are bound by the HBM stream (f1, f2 with
// the 14 x 22 / 8 x 16 halo re-reads, the 116-channel concat rows written: ~4.3 TB/s).
constexpr int CB_Y = 8, CB_X = 16, CB_PIX = CB_Y * CB_X, CB_QX = CB_X / 4, CB_NQ = CB_Y * CB_QX;
constexpr int CB_SC = 32, CB_PS = CB_SC + 4;                 // slab channels, LDS pixel stride
constexpr int CB_HY = CB_Y + 6, CB_HX = CB_X + 6, CB_HXP = 25, CB_F1P = CB_X + 1;
constexpr int CB_NT = CB_NQ * 7;                             // 224 threads
constexpr int CB_HQ = CB_HY * CB_HX * (CB_SC / 4), CB_HU = (CB_HQ + CB_NT - 1) / CB_NT;
constexpr int CB_FQ = CB_PIX * (CB_SC / 4), CB_FU = (CB_FQ + CB_NT - 1) / CB_NT;
constexpr int CB_LDS_HALO = CB_HY * CB_HXP * CB_PS, CB_LDS_F1 = CB_Y * CB_F1P * CB_PS;
static_assert(CB_PIX * 49 <= CB_LDS_HALO, "epilogue staging reuses the halo region");

struct CorrBlkArgs {
  CorrFwdArgs a;
  int slabs;          // ceil(c / 32)
  int spg, groups;    // slabs per group, groups per tile
  int tiles_x, tiles_y, items;
};

template <bool VEC>
__global__ __launch_bounds__(CB_NT, 2) void corr_fwd_blk(CorrBlkArgs p) {
  __shared__ float4 lds4[(CB_LDS_HALO + CB_LDS_F1) / 4];
  float* hal = reinterpret_cast<float*>(lds4);
  float* f1s = hal + CB_LDS_HALO;
  const CorrFwdArgs& a = p.a;
  const int h = a.h, w = a.w, tid = threadIdx.x;
  const int tiles = p.tiles_x * p.tiles_y;
  const int64_t npix_all = (int64_t)(p.items / (tiles * p.groups)) * h * w;
  constexpr bool vec = VEC;
  // compute role
  const int oi = tid >> 5, qd = tid & 31;
  const int cty = qd / CB_QX, ctx = (qd % CB_QX) * 4;
  const int f1b = (cty * CB_F1P + ctx) * CB_PS, f2b = ((cty + oi) * CB_HXP + ctx) * CB_PS;

  float4 hv[CB_HU], fv[CB_FU];
  auto decode = [&](int it, int s, int& b, int& y0, int& x0, int& g, int& c_lo) {
    g = it % p.groups;
    const int r = it / p.groups, tl = r % tiles;
    b = r / tiles;
    y0 = (tl / p.tiles_x) * CB_Y, x0 = (tl % p.tiles_x) * CB_X;
    c_lo = (g * p.spg + s) * CB_SC;
  };
  auto load = [&](int it, int s) {
    int b, y0, x0, g, c_lo;
    decode(it, s, b, y0, x0, g, c_lo);
    const int cs = min(CB_SC, a.c - c_lo);
    const int64_t img = (int64_t)b * h * w;
    const rsrc_t r1 = make_rsrc(a.f1 + img * a.ld1, (int64_t)h * w * a.ld1 * 4);
    const rsrc_t r2 = make_rsrc(a.f2 + img * a.ld2, (int64_t)h * w * a.ld2 * 4);
#pragma unroll
    for (int u = 0; u < CB_HU; ++u) {
      const int q = tid + CB_NT * u;
      const int hp = q >> 3, cq = q & 7;
      const int sy = y0 - 3 + hp / CB_HX, sx = x0 - 3 + hp % CB_HX;
      const bool ok = q < CB_HQ && (unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w;
      hv[u] = bload_quad(r2, ok, 4 * ((sy * w + sx) * a.ld2 + c_lo + 4 * cq), cs - 4 * cq, vec);
    }
#pragma unroll
    for (int u = 0; u < CB_FU; ++u) {
      const int q = tid + CB_NT * u;
      const int pp = q >> 3, cq = q & 7;
      const int sy = y0 + pp / CB_X, sx = x0 + pp % CB_X;
      const bool ok = q < CB_FQ && sy < h && sx < w;
      fv[u] = bload_quad(r1, ok, 4 * ((sy * w + sx) * a.ld1 + c_lo + 4 * cq), cs - 4 * cq, vec);
    }
  };

  // Persistent walk, XCD-aware: the workgroups of one XCD (blockIdx % 8) walk one contiguous
  // eighth of the items, so tiles that share halo rows are in flight on the same L2.
  const int nx = (gridDim.x >= 64 && (gridDim.x & 7) == 0) ? 8 : 1;
  const int part = blockIdx.x % nx, per = gridDim.x / nx, chunk = (p.items + nx - 1) / nx;
  auto valid = [&](int l) { return l < chunk && part * chunk + l < p.items; };
  int lt = blockIdx.x / nx, s = 0;
  if (!valid(lt)) return;                          // uniform over the workgroup
  int it = part * chunk + lt;
  load(it, s);
  f32x2 acc[28];
  for (;;) {
    int b, y0, x0, g, c_lo;
    decode(it, s, b, y0, x0, g, c_lo);
    const int64_t img = (int64_t)b * h * w;
    // install the loaded slab
#pragma unroll
    for (int u = 0; u < CB_HU; ++u) {
      const int q = tid + CB_NT * u;
      const int hp = q >> 3, cq = q & 7;
      if (q < CB_HQ)
        *reinterpret_cast<float4*>(&hal[((hp / CB_HX) * CB_HXP + hp % CB_HX) * CB_PS + 4 * cq]) = hv[u];
    }
#pragma unroll
    for (int u = 0; u < CB_FU; ++u) {
      const int q = tid + CB_NT * u;
      const int pp = q >> 3, cq = q & 7;
      if (q < CB_FQ) {
        *reinterpret_cast<float4*>(&f1s[((pp / CB_X) * CB_F1P + pp % CB_X) * CB_PS + 4 * cq]) = fv[u];
        if (a.cat16) {                               // f1 slice of the bf16 concat image
          const int sy = y0 + pp / CB_X, sx = x0 + pp % CB_X, ch = c_lo + 4 * cq;
          if (sy < h && sx < w && ch < a.c)          // (c % 4 == 0)
            *reinterpret_cast<uint2*>(a.cat16 + (img + sy * w + sx) * a.ld16 + ch) = pack4_bf16(fv[u]);
        }
        if (a.cat) {                                 // f1 slice of the concat row
          const int sy = y0 + pp / CB_X, sx = x0 + pp % CB_X, ch = c_lo + 4 * cq;
          const int n = a.c - ch;
          if (sy < h && sx < w && n > 0) {
            float* dst = a.cat + (img + sy * w + sx) * a.ldcv + ch;
            if (vec) {
              *reinterpret_cast<float4*>(dst) = fv[u];
            } else {
              const float t[4] = {fv[u].x, fv[u].y, fv[u].z, fv[u].w};
#pragma unroll
              for (int k = 0; k < 4; ++k)
                if (k < n) dst[k] = t[k];
            }
          }
        }
      }
    }
    __syncthreads();
    // next step, prefetched while this slab computes
    const int nsl = min(p.slabs - g * p.spg, p.spg);
    int nlt = lt, ns = s + 1;
    if (ns == nsl) nlt = lt + per, ns = 0;
    const bool more = valid(nlt);
    const int nit = part * chunk + nlt;
    if (more) load(nit, ns);
    if (s == 0) {
#pragma unroll
      for (int k = 0; k < 28; ++k) acc[k] = f32x2{0.f, 0.f};
    }
#pragma unroll 2
    for (int c4 = 0; c4 < CB_SC / 4; ++c4) {
      float4 fa[4], wv[10];
#pragma unroll
      for (int m = 0; m < 4; ++m) fa[m] = *reinterpret_cast<const float4*>(&f1s[f1b + m * CB_PS + 4 * c4]);
#pragma unroll
      for (int j = 0; j < 10; ++j) wv[j] = *reinterpret_cast<const float4*>(&hal[f2b + j * CB_PS + 4 * c4]);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int j = 0; j < 7; ++j) {
          acc[m * 7 + j] = __builtin_elementwise_fma(f32x2{fa[m].x, fa[m].y},
                                                     f32x2{wv[m + j].x, wv[m + j].y}, acc[m * 7 + j]);
          acc[m * 7 + j] = __builtin_elementwise_fma(f32x2{fa[m].z, fa[m].w},
                                                     f32x2{wv[m + j].z, wv[m + j].w}, acc[m * 7 + j]);
        }
      }
    }
    __syncthreads();                               // halo / f1 tile no longer read
    if (ns == 0) {                                 // last slab of the item: epilogue
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < 7; ++j)
          hal[(cty * CB_X + ctx + m) * 49 + oi * 7 + j] = acc[m * 7 + j].x + acc[m * 7 + j].y;
      __syncthreads();
      if (a.cat16) {                               // bf16 image: cv, flow, zero padding
        __bf16* o16 = reinterpret_cast<__bf16*>(a.cat16);
        for (int q = tid; q < CB_PIX * 49; q += CB_NT) {
          const int pp = q / 49, k = q - pp * 49;
          const int sy = y0 + pp / CB_X, sx = x0 + pp % CB_X;
          if (sy < h && sx < w) o16[(img + sy * w + sx) * a.ld16 + a.c + k] = (__bf16)hal[q];
        }
        for (int pp = tid; pp < CB_PIX; pp += CB_NT) {
          const int sy = y0 + pp / CB_X, sx = x0 + pp % CB_X;
          if (sy >= h || sx >= w) continue;
          const int64_t pl = img + sy * w + sx;
          __bf16* row = o16 + pl * a.ld16;
          int ch = a.c + 49;
          if (a.flow) {
            row[ch] = (__bf16)a.flow[2 * pl];
            row[ch + 1] = (__bf16)a.flow[2 * pl + 1];
            ch += 2;
          }
          for (; ch < a.ld16; ++ch) row[ch] = (__bf16)0.f;
        }
        __syncthreads();
        if (!more) break;
        lt = nlt, it = nit, s = ns;
        continue;
      }
      float* out;
      int64_t ld;
      if (p.groups == 1) {
        out = a.cv, ld = a.ldcv;
      } else {
        out = a.part + g * npix_all * 49, ld = 49;
      }
      for (int q = tid; q < CB_PIX * 49; q += CB_NT) {
        const int pp = q / 49, k = q - pp * 49;
        const int sy = y0 + pp / CB_X, sx = x0 + pp % CB_X;
        if (sy < h && sx < w) out[(img + sy * w + sx) * ld + k] = hal[q];
      }
      if (a.cat && g == 0) {                       // flow and zero channel padding
        for (int pp = tid; pp < CB_PIX; pp += CB_NT) {
          const int sy = y0 + pp / CB_X, sx = x0 + pp % CB_X;
          if (sy >= h || sx >= w) continue;
          const int64_t pl = img + sy * w + sx;
          float* row = a.cat + pl * a.ldcv;
          int ch = a.c + 49;
          if (a.flow) {
            row[ch] = a.flow[2 * pl];
            row[ch + 1] = a.flow[2 * pl + 1];
            ch += 2;
          }
          for (; ch < a.ldcv; ++ch) row[ch] = 0.f;
        }
      }
      __syncthreads();                             // staging read before the next install
    }
    if (!more) break;
    lt = nlt, it = nit, s = ns;
  }
}

// Gradient of the cost volume w.r.t. one input (gather form, no atomics):
//   SIGN=+1 (df1): df[p][c] = init[p][c] + sum_k g[p][k]       * src[p + d_k][c]   (src = f2)
//   SIGN=-1 (df2): df[q][c] = init[q][c] + sum_k g[q - d_k][k] * src[q - d_k][c]   (src = f1)
struct CorrBwdArgs {
  const float* g;     // d(cost volume), row stride ldg
  int ldg;
  const float* src;
  int lds;
  int h, w, c;
  float* df;
  int lddf;
  const float* init;  // NULL, or added to the result (row stride ldinit; may alias df)
  int ldinit;
  int vec;            // src / df / init float4 access allowed
  int slabs;
  int tiles_x, tiles_y;
};

// TY = 4: 4 x 16-pixel tiles, 256 threads, two workgroups per CU (72.5 KB of LDS); TY = 8
// (of_set_tuning key 19): 8 x 16 tiles with 512 threads, one workgroup per CU (108 KB): the
// same 8 waves per CU, the src halo read 2.4x per pixel instead of 3.4x.
template <int D, int SIGN, bool VEC, int TY = CT_Y>
__global__ __launch_bounds__(64 * TY, TY == CT_Y ? 2 : 1) void corr_bwd_kernel(CorrBwdArgs a) {
  constexpr int TX = CT_X, TPIX = TY * TX, NT = 4 * TPIX;
  constexpr int ND = 2 * D + 1, NK = ND * ND;
  constexpr int HY = TY + 2 * D, HX = TX + 2 * D, NH = HY * HX;
  constexpr int NQ = NH * (CSLAB / 4), NU = (NQ + NT - 1) / NT;
  // Coefficient loads: d/d(f1) reads each tile pixel's 49 contiguous g values; d/d(f2) reads,
  // per offset row i, the 7 contiguous g values of the source pixels that map into the tile.
  constexpr int GROW = HX * ND;                      // per source row, per offset row i
  constexpr int NGQ = SIGN > 0 ? TPIX * NK : ND * TY * GROW;
  constexpr int NG = (NGQ + NT - 1) / NT;
  __shared__ float4 lds4[NH * CSPS / 4];
  __shared__ float G[NK * TPIX];
  float* tile = reinterpret_cast<float*>(lds4);
  const int h = a.h, w = a.w;
  // 1-D grid, XCD-aware: neighbouring tiles (shared halo rows) run on one XCD's L2.
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tl = wg % (a.tiles_x * a.tiles_y), z = wg / (a.tiles_x * a.tiles_y);
  const int b = z / a.slabs, slab = z - b * a.slabs;
  const int c_lo = slab * CSLAB, cs = min(CSLAB, a.c - c_lo);
  const int y0 = (tl / a.tiles_x) * TY, x0 = (tl % a.tiles_x) * TX;
  const int tid = threadIdx.x;
  const int pix = tid >> 2, qtr = tid & 3;
  const int ty = pix / TX, tx = pix % TX;
  const int y = y0 + ty, x = x0 + tx;
  const bool valid = y < h && x < w;
  const int64_t img = (int64_t)b * h * w;
  const int pl = y * w + x;
  const rsrc_t rg = make_rsrc(a.g + img * a.ldg, (int64_t)h * w * a.ldg * 4);
  const rsrc_t rs = make_rsrc(a.src + img * a.lds, (int64_t)h * w * a.lds * 4);
  const rsrc_t ri = make_rsrc(a.init ? a.init + img * a.ldinit : nullptr,
                              a.init ? (int64_t)h * w * a.ldinit * 4 : 0);
  // One load round: coefficients, the src halo slab, the init values.
  float gv[NG];
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    const int q = tid + NT * u;
    uint32_t off = kOOB;
    if (SIGN > 0) {
      const int p = q / NK, k = q - p * NK;
      const int sy = y0 + p / TX, sx = x0 + p % TX;
      if (q < NGQ && sy < h && sx < w) off = 4 * ((sy * w + sx) * a.ldg + k);
    } else {
      const int i = q / (TY * GROW), r0 = q - i * (TY * GROW);
      const int r = r0 / GROW, rem = r0 - r * GROW;
      const int hx = rem / ND, j = rem - hx * ND;
      const int sy = y0 + r + D - i, sx = x0 - D + hx;   // source of target row r
      if (q < NGQ && (unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w)
        off = 4 * ((sy * w + sx) * a.ldg + i * ND + j);
    }
    gv[u] = bload1(rg, off);
  }
  float4 hv[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int q = tid + NT * u;
    const int hp = q >> 4, cq = q & 15;
    const int sy = y0 - D + hp / HX, sx = x0 - D + hp % HX;
    const bool ok = q < NQ && (unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w;
    hv[u] = bload_quad(rs, ok, 4 * ((sy * w + sx) * a.lds + c_lo + 4 * cq), cs - 4 * cq, VEC);
  }
  float acc[16];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ch = qtr * 16 + 4 * e;
    const float4 v = bload_quad(ri, valid, 4 * (pl * a.ldinit + c_lo + ch), cs - ch, VEC);
    acc[4 * e] = v.x;
    acc[4 * e + 1] = v.y;
    acc[4 * e + 2] = v.z;
    acc[4 * e + 3] = v.w;
  }
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    const int q = tid + NT * u;
    if (SIGN > 0) {
      const int p = q / NK, k = q - p * NK;
      if (q < NGQ) G[k * TPIX + p] = gv[u];
    } else {
      const int i = q / (TY * GROW), r0 = q - i * (TY * GROW);
      const int r = r0 / GROW, rem = r0 - r * GROW;
      const int hx = rem / ND, j = rem - hx * ND;
      const int tx2 = hx + j - 2 * D;                  // target column
      if (q < NGQ && (unsigned)tx2 < (unsigned)TX) G[(i * ND + j) * TPIX + r * TX + tx2] = gv[u];
    }
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int q = tid + NT * u;
    if (q < NQ) *reinterpret_cast<float4*>(&tile[(q >> 4) * CSPS + 4 * (q & 15)]) = hv[u];
  }
  __syncthreads();
  // One channel quad per pass (not unrolled): bounds the LDS reads the scheduler can hoist.
#pragma unroll 1
  for (int e = 0; e < 4; ++e) {
    float4 s4[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    const float* tb = &tile[(ty * HX + tx) * CSPS + qtr * 16 + 4 * e];
#pragma unroll
    for (int i = 0; i < ND; ++i) {
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const int oy = SIGN > 0 ? i : 2 * D - i;   // tile row of src[p + SIGN*d]
        const int ox = SIGN > 0 ? j : 2 * D - j;
        const float4 v = *reinterpret_cast<const float4*>(tb + (oy * HX + ox) * CSPS);
        const float cf = G[(i * ND + j) * TPIX + pix];
        float4& sa = s4[(i * ND + j) & 1];   // two chains: halves the FMA dependency depth
        sa.x = fmaf(cf, v.x, sa.x);
        sa.y = fmaf(cf, v.y, sa.y);
        sa.z = fmaf(cf, v.z, sa.z);
        sa.w = fmaf(cf, v.w, sa.w);
      }
    }
    // acc[4e..4e+3] += s4 (register index must stay static: select by e)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q == e) {
        acc[4 * q] += s4[0].x + s4[1].x;
        acc[4 * q + 1] += s4[0].y + s4[1].y;
        acc[4 * q + 2] += s4[0].z + s4[1].z;
        acc[4 * q + 3] += s4[0].w + s4[1].w;
      }
    }
  }
  if (valid) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ch = qtr * 16 + 4 * e;
      float* o = a.df + (img + pl) * a.lddf + c_lo + ch;
      if (VEC && cs - ch >= 4) {
        *reinterpret_cast<float4*>(o) = make_float4(acc[4 * e], acc[4 * e + 1], acc[4 * e + 2],
                                                    acc[4 * e + 3]);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (k < cs - ch) o[k] = acc[4 * e + k];
      }
    }
  }
}

// ---- register-blocked backward (of_set_tuning key 9 bit 1, the default) -------------------
// Same tile, slab and halo image as corr_fwd_blk; thread = (4 adjacent pixels, one channel
// quad of the slab), 256 threads.  The tile's 49 x 128 coefficients sit in LDS [k][pixel]
// (loaded once per tile, lanes over pixels: conflict-free b32 writes, and the b128 reads of
// 4 pixels' coefficients hit 16 distinct slots); per offset row, 10 src quads + 7 coefficient
// quads feed 112 FMAs (the form above: 4 per 5 loads).  Slabs are independent outputs, so
// items are (tile, slab group) without partial sums; the next slab's src halo, the init
// values and (for a new tile) the coefficients are loaded into registers while the current
// slab computes.  75 KB of LDS: two workgroups per CU.
// Measured slower than corr_bwd_kernel (192x256x64, both inputs: 266 vs 255 us; the
// coefficient rows and the src halo stream at the same ~4.3 TB/s), so it is not the default.
constexpr int CBB_NT = CB_NQ * (CB_SC / 4);                  // 256 threads
constexpr int CBB_HU = (CB_HQ + CBB_NT - 1) / CBB_NT;
constexpr int CBB_GQ = 49 * CB_PIX, CBB_GU = (CBB_GQ + CBB_NT - 1) / CBB_NT;

template <int SIGN, bool VEC>
__global__ __launch_bounds__(CBB_NT, 2) void corr_bwd_blk(CorrBwdArgs a, int slabs, int spg,
                                                          int groups, int items) {
  __shared__ float4 lds4[(CB_LDS_HALO + 49 * CB_PIX) / 4];
  float* hal = reinterpret_cast<float*>(lds4);
  float* G = hal + CB_LDS_HALO;
  const int h = a.h, w = a.w, tid = threadIdx.x;
  const int tiles = a.tiles_x * a.tiles_y;
  constexpr bool vec = VEC;
  const int qd = tid & 31, c4 = tid >> 5;
  const int cty = qd / CB_QX, ctx = (qd % CB_QX) * 4;

  float4 hv[CBB_HU], iv[4];
  float gv[CBB_GU];
  auto decode = [&](int it, int s, int& b, int& y0, int& x0, int& c_lo) {
    const int g = it % groups, r = it / groups, tl = r % tiles;
    b = r / tiles;
    y0 = (tl / a.tiles_x) * CB_Y, x0 = (tl % a.tiles_x) * CB_X;
    c_lo = (g * spg + s) * CB_SC;
  };
  auto load = [&](int it, int s) {
    int b, y0, x0, c_lo;
    decode(it, s, b, y0, x0, c_lo);
    const int cs = min(CB_SC, a.c - c_lo);
    const int64_t img = (int64_t)b * h * w;
    const rsrc_t rs = make_rsrc(a.src + img * a.lds, (int64_t)h * w * a.lds * 4);
#pragma unroll
    for (int u = 0; u < CBB_HU; ++u) {
      const int q = tid + CBB_NT * u;
      const int hp = q >> 3, cq = q & 7;
      const int sy = y0 - 3 + hp / CB_HX, sx = x0 - 3 + hp % CB_HX;
      const bool ok = q < CB_HQ && (unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w;
      hv[u] = bload_quad(rs, ok, 4 * ((sy * w + sx) * a.lds + c_lo + 4 * cq), cs - 4 * cq, vec);
    }
    const rsrc_t ri = make_rsrc(a.init ? a.init + img * a.ldinit : nullptr,
                                a.init ? (int64_t)h * w * a.ldinit * 4 : 0);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int sy = y0 + cty, sx = x0 + ctx + m;
      iv[m] = bload_quad(ri, sy < h && sx < w, 4 * ((sy * w + sx) * a.ldinit + c_lo + 4 * c4),
                         cs - 4 * c4, vec);
    }
    if (s == 0) {                                  // coefficients of a new tile
      const rsrc_t rg = make_rsrc(a.g + img * a.ldg, (int64_t)h * w * a.ldg * 4);
#pragma unroll
      for (int u = 0; u < CBB_GU; ++u) {
        const int q = tid + CBB_NT * u;
        const int k = q / CB_PIX, pp = q % CB_PIX;
        int sy = y0 + pp / CB_X, sx = x0 + pp % CB_X;
        const bool in = sy < h && sx < w;
        if (SIGN < 0) sy -= k / 7 - 3, sx -= k % 7 - 3;   // g[p - d_k][k]
        const bool ok = q < CBB_GQ && in && (unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w;
        gv[u] = bload1(rg, ok ? 4 * ((sy * w + sx) * a.ldg + k) : kOOB);
      }
    }
  };

  // Persistent walk, XCD-aware: the workgroups of one XCD (blockIdx % 8) walk one contiguous
  // eighth of the items, so tiles that share halo rows are in flight on the same L2.
  const int nx = (gridDim.x >= 64 && (gridDim.x & 7) == 0) ? 8 : 1;
  const int part = blockIdx.x % nx, per = gridDim.x / nx, chunk = (items + nx - 1) / nx;
  auto valid = [&](int l) { return l < chunk && part * chunk + l < items; };
  int lt = blockIdx.x / nx, s = 0;
  if (!valid(lt)) return;                          // uniform over the workgroup
  int it = part * chunk + lt;
  load(it, s);
  for (;;) {
    int b, y0, x0, c_lo;
    decode(it, s, b, y0, x0, c_lo);
    const int cs = min(CB_SC, a.c - c_lo);
    const int64_t img = (int64_t)b * h * w;
#pragma unroll
    for (int u = 0; u < CBB_HU; ++u) {
      const int q = tid + CBB_NT * u;
      const int hp = q >> 3, cq = q & 7;
      if (q < CB_HQ)
        *reinterpret_cast<float4*>(&hal[((hp / CB_HX) * CB_HXP + hp % CB_HX) * CB_PS + 4 * cq]) = hv[u];
    }
    if (s == 0) {
#pragma unroll
      for (int u = 0; u < CBB_GU; ++u) {
        const int q = tid + CBB_NT * u;
        if (q < CBB_GQ) G[q] = gv[u];
      }
    }
    f32x2 acc[8];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      acc[2 * m] = f32x2{iv[m].x, iv[m].y};
      acc[2 * m + 1] = f32x2{iv[m].z, iv[m].w};
    }
    __syncthreads();
    const int gid = it % groups;
    const int nsl = min(slabs - gid * spg, spg);
    int nlt = lt, ns = s + 1;
    if (ns == nsl) nlt = lt + per, ns = 0;
    const bool more = valid(nlt);
    const int nit = part * chunk + nlt;
    if (more) load(nit, ns);
#pragma unroll 1
    for (int i = 0; i < 7; ++i) {
      const int oy = SIGN > 0 ? i : 6 - i;
      const float* wb = &hal[((cty + oy) * CB_HXP + ctx) * CB_PS + 4 * c4];
      float4 wv[10];
#pragma unroll
      for (int j = 0; j < 10; ++j) wv[j] = *reinterpret_cast<const float4*>(wb + j * CB_PS);
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const float4 gq = *reinterpret_cast<const float4*>(&G[(i * 7 + j) * CB_PIX + cty * CB_X + ctx]);
        const int ox = SIGN > 0 ? j : 6 - j;
        const float gm[4] = {gq.x, gq.y, gq.z, gq.w};
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const float4 v = wv[m + ox];
          acc[2 * m] = __builtin_elementwise_fma(f32x2{gm[m], gm[m]}, f32x2{v.x, v.y}, acc[2 * m]);
          acc[2 * m + 1] = __builtin_elementwise_fma(f32x2{gm[m], gm[m]}, f32x2{v.z, v.w}, acc[2 * m + 1]);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int sy = y0 + cty, sx = x0 + ctx + m, ch = 4 * c4;
      if (sy < h && sx < w && ch < cs) {
        float* o = a.df + (img + sy * w + sx) * a.lddf + c_lo + ch;
        if (vec) {
          *reinterpret_cast<float4*>(o) = make_float4(acc[2 * m].x, acc[2 * m].y, acc[2 * m + 1].x,
                                                      acc[2 * m + 1].y);
        } else {
          const float t[4] = {acc[2 * m].x, acc[2 * m].y, acc[2 * m + 1].x, acc[2 * m + 1].y};
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (k < cs - ch) o[k] = t[k];
        }
      }
    }
    __syncthreads();                               // halo / coefficients no longer read
    if (!more) break;
    lt = nlt, it = nit, s = ns;
  }
}

// ---- fused backward (of_set_tuning key 9 bit 2, the default when both gradients are wanted) --
// d/d(f1) and d/d(f2) of one 8 x 16 tile and one 32-channel slab in one workgroup, from one
// staging of the tile's 14 x 22 coefficient halo:
//   df1[p] = sum_k g[p][k] f2[p + d_k]          (waves 0-3: f2 halo, G1[p][k] = g[p][k])
//   df2[q] = sum_k g[q - d_k][k] f1[q - d_k]    (waves 4-7: f1 halo, H[q][k] = g[q - d_k][k])
// The coefficient halo (all 49 values of each of its 308 pixels as 13 16-byte quads, the
// last one reading 3 channels past the cost volume) is read once
// per tile and scattered into both tables; the f1 / f2 halo slabs once per (tile, slab).  A
// thread owns 4 adjacent pixels x one channel quad: per offset row, 10 src + 8 coefficient
// ds_read_b128 feed 112 FMAs.  Coefficient tables are [pixel][offset row][8] with a 60-float
// pixel pitch, halo pixels have a 40-float pitch: the b128 reads of every 16-lane group hit
// distinct slots.  160,000 B of LDS, one 512-thread workgroup per CU, persistent: workgroup
// w walks items [w * items / grid, (w + 1) * items / grid) (items = (tile, slab), slabs of a
// tile adjacent; XCD-remapped, so neighbouring tiles share an L2), and loads the next item's
// halos (and, for a new tile, coefficients) into registers while the current one computes.
// Timing ablations of corr_bwd_fused (tools/ab_build.sh -DCORR_ABL=mask; wrong results, never
// in the shipped build): 1 no coefficient scatter, 2 no row compute, 4 no added-gradient loads.
#ifndef CORR_ABL
#define CORR_ABL 0
#endif
constexpr int FB_Y = 8, FB_X = 16, FB_PIX = FB_Y * FB_X;
constexpr int FB_HY = FB_Y + 6, FB_HX = FB_X + 6, FB_HPIX = FB_HY * FB_HX;   // 14 x 22
constexpr int FB_SC = 32, FB_PS = 40, FB_GP = 60, FB_NT = 512;
constexpr int FB_HQ = FB_HPIX * (FB_SC / 4), FB_HU = (FB_HQ + FB_NT - 1) / FB_NT;   // 2464, 5
constexpr int FB_GQ = FB_HPIX * 13, FB_GU = (FB_GQ + FB_NT - 1) / FB_NT;   // 4004 quads, 8
constexpr int FB_LDS = 2 * FB_HPIX * FB_PS + 2 * FB_PIX * FB_GP + 64;   // floats (+ dummy words)

struct CorrFusedArgs {
  const float* g; int ldg;
  const float* f1; int ld1;
  const float* f2; int ld2;
  float* df1; int lddf1;
  const float* init1; int ldinit1;    // NULL, or added to df1 (may alias df1)
  float* df2; int lddf2;
  const float* init2; int ldinit2;
  int h, w, c, slabs, tiles_x, tiles_y, items;
};

#ifndef CFR_UNROLL
#define CFR_UNROLL 7   // rows unrolled: 2 VGPRs spilled outside the row loop; 233 -> 226 us at level 3
#endif
// One role's 7 offset rows: ROLE 0 = df1 (src f2 at p + d), 1 = df2 (src f1 at q - d).
template <int ROLE>
__device__ __forceinline__ void corr_fused_rows(const float* hal, const float* gt, int row,
                                                int col0, int cq, f32x2 (&acc)[8]) {
#pragma unroll CFR_UNROLL
  for (int i = 0; i < 7; ++i) {
    const int hr = ROLE == 0 ? row + i : row + 6 - i;
    const float* sb = &hal[(hr * FB_HX + col0) * FB_PS + 4 * cq];
    float4 sv[10];
#pragma unroll
    for (int u = 0; u < 10; ++u) sv[u] = *reinterpret_cast<const float4*>(sb + u * FB_PS);
    // pixel by pixel: its 7 coefficients of row i (two b128 reads), 14 packed FMAs
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float* cb = &gt[(row * FB_X + col0 + m) * FB_GP + 8 * i];
      const float4 lo = *reinterpret_cast<const float4*>(cb);
      float4 hi = *reinterpret_cast<const float4*>(cb + 4);
      asm volatile("" : "+v"(hi.w));   // keep the 4th word: a b128 read, not a slower b96
      const float cf[7] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z};
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const float4 v = sv[(ROLE == 0 ? j : 6 - j) + m];
        const f32x2 c2 = {cf[j], cf[j]};
        acc[2 * m] = __builtin_elementwise_fma(c2, f32x2{v.x, v.y}, acc[2 * m]);
        acc[2 * m + 1] = __builtin_elementwise_fma(c2, f32x2{v.z, v.w}, acc[2 * m + 1]);
      }
    }
  }
}

__global__ __launch_bounds__(FB_NT, 1) void corr_bwd_fused(CorrFusedArgs a) {
  __shared__ float4 lds4[FB_LDS / 4];
  float* hal1 = reinterpret_cast<float*>(lds4);   // f1 halo slab (df2's source)
  float* hal2 = hal1 + FB_HPIX * FB_PS;           // f2 halo slab (df1's source)
  float* G1 = hal2 + FB_HPIX * FB_PS;             // [p][i][8]: g[p][7i + j]
  float* H = G1 + FB_PIX * FB_GP;                 // [q][i][8]: g[q - d_k][k], k = 7i + j
  const int tid = threadIdx.x, h = a.h, w = a.w;
  const int tiles = a.tiles_x * a.tiles_y;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int it0 = (int)((int64_t)wg * a.items / gridDim.x);
  const int it1 = (int)((int64_t)(wg + 1) * a.items / gridDim.x);
  if (it0 >= it1) return;                         // uniform over the workgroup
  auto decode = [&](int it, int& b, int& y0, int& x0, int& c_lo) {
    const int t = it / a.slabs;
    c_lo = (it - t * a.slabs) * FB_SC;
    b = t / tiles;
    const int tl = t - b * tiles;
    y0 = (tl / a.tiles_x) * FB_Y, x0 = (tl % a.tiles_x) * FB_X;
  };
  float4 hv1[FB_HU], hv2[FB_HU];
  float4 gv[FB_GU];            // coefficient quads k = 4 kq .. 4 kq + 3 (k < 49 kept)
  auto load_halo = [&](int it) {
    int b, y0, x0, c_lo;
    decode(it, b, y0, x0, c_lo);
    const int64_t img = (int64_t)b * h * w;
    const rsrc_t r1 = make_rsrc(a.f1 + img * a.ld1, (int64_t)h * w * a.ld1 * 4);
    const rsrc_t r2 = make_rsrc(a.f2 + img * a.ld2, (int64_t)h * w * a.ld2 * 4);
#pragma unroll
    for (int u = 0; u < FB_HU; ++u) {
      const int q = tid + FB_NT * u;
      const int hp = q >> 3, cq = q & 7;
      const int sy = y0 - 3 + hp / FB_HX, sx = x0 - 3 + hp % FB_HX;
      const bool ok = q < FB_HQ && (unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w;
      const int pix = sy * w + sx, ch = c_lo + 4 * cq;
      hv1[u] = bload4(r1, ok ? 4 * (pix * a.ld1 + ch) : kOOB);
      hv2[u] = bload4(r2, ok ? 4 * (pix * a.ld2 + ch) : kOOB);
    }
  };
  auto load_coef = [&](int it) {
    int b, y0, x0, c_lo;
    decode(it, b, y0, x0, c_lo);
    const int64_t img = (int64_t)b * h * w;
    const rsrc_t rg = make_rsrc(a.g + img * a.ldg, (int64_t)h * w * a.ldg * 4);
#pragma unroll
    for (int u = 0; u < FB_GU; ++u) {
      const int q = tid + FB_NT * u;
      const int hp = q / 13, kq = q - hp * 13;
      const int sy = y0 - 3 + hp / FB_HX, sx = x0 - 3 + hp % FB_HX;
      const bool ok = q < FB_GQ && (unsigned)sy < (unsigned)h && (unsigned)sx < (unsigned)w;
      gv[u] = bload4(rg, ok ? 4 * ((sy * w + sx) * a.ldg + 4 * kq) : kOOB);
    }
  };
  const int role = __builtin_amdgcn_readfirstlane(tid >> 8);   // wave-uniform: scalar rsrcs
  const int r = tid & 255, cq = r & 7, pg = r >> 3;
  const int row = pg >> 2, col0 = (pg & 3) * 4;
  int it = it0, cur_tile = -1;
  load_halo(it);
  load_coef(it);
  for (;;) {
    const int tile = it / a.slabs;
#pragma unroll
    for (int u = 0; u < FB_HU; ++u) {
      const int q = tid + FB_NT * u;
      if (q < FB_HQ) {
        const int o = (q >> 3) * FB_PS + 4 * (q & 7);
        *reinterpret_cast<float4*>(&hal1[o]) = hv1[u];
        *reinterpret_cast<float4*>(&hal2[o]) = hv2[u];
      }
    }
    if (!(CORR_ABL & 1) && tile != cur_tile) {    // uniform: scatter the new coefficients
      // straight-line: a value with no slot in a table goes to this lane's dummy word (a
      // guarded store per value compiled to a branch, an exec save and a wait each)
      float* const dummy = H + FB_PIX * FB_GP + (tid & 63);
#pragma unroll
      for (int u = 0; u < FB_GU; ++u) {
        const int q = tid + FB_NT * u;
        const int hp = q / 13, kq = q - hp * 13;
        const int hy = hp / FB_HX, hx = hp - hy * FB_HX;
        const bool live = q < FB_GQ;
        const bool own = live && (unsigned)(hy - 3) < (unsigned)FB_Y && (unsigned)(hx - 3) < (unsigned)FB_X;
        const float gq[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 4 * kq + e;
          const int i = k / 7, j = k - 7 * i;
          const bool kk = k < 49;
          float* g1 = own && kk ? &G1[((hy - 3) * FB_X + hx - 3) * FB_GP + 8 * i + j] : dummy;
          *g1 = gq[e];
          const int ty = hy + i - 6, tx = hx + j - 6;   // target q = p + d_k
          const bool hit = live && kk && (unsigned)ty < (unsigned)FB_Y && (unsigned)tx < (unsigned)FB_X;
          float* hq = hit ? &H[(ty * FB_X + tx) * FB_GP + 8 * i + j] : dummy;
          *hq = gq[e];
        }
      }
      cur_tile = tile;
    }
    __syncthreads();
    const int nit = it + 1;
    const bool more = nit < it1;
    if (more) {
      load_halo(nit);
      if (nit / a.slabs != tile) load_coef(nit);
    }
    int b, y0, x0, c_lo;
    decode(it, b, y0, x0, c_lo);
    const int64_t img = (int64_t)b * h * w;
    const int y = y0 + row, ch = c_lo + 4 * cq;
    f32x2 acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = f32x2{0.f, 0.f};
    if (CORR_ABL & 2) {
    } else if (role == 0) {
      corr_fused_rows<0>(hal2, G1, row, col0, cq, acc);
    } else {
      corr_fused_rows<1>(hal1, H, row, col0, cq, acc);
    }
    // the added gradients (issued before the rows they would land during the compute, but
    // their 16 registers push the kernel past 256 VGPRs: 23 spills)
    const float* init = role == 0 ? a.init1 : a.init2;
    const int ldi = role == 0 ? a.ldinit1 : a.ldinit2;
    float4 iv[4];
    {
      const rsrc_t ri = make_rsrc(init ? init + img * ldi : nullptr, init ? (int64_t)h * w * ldi * 4 : 0);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int x = x0 + col0 + m;
        iv[m] = bload4(ri, !(CORR_ABL & 4) && y < h && x < w ? 4 * ((y * w + x) * ldi + ch) : kOOB);
      }
    }
    float* df = role == 0 ? a.df1 : a.df2;
    const int ldd = role == 0 ? a.lddf1 : a.lddf2;
    // unguarded buffer stores (edge pixels dropped by offset): with a guarded store the
    // wait for iv sat on one path only, and the compiler then waited for every load in
    // flight -- the next item's prefetch -- at the top of the next item's row loop
    const rsrc_t rd = make_rsrc(df + img * ldd, (int64_t)h * w * ldd * 4);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int x = x0 + col0 + m;
      bstore4(make_float4(iv[m].x + acc[2 * m].x, iv[m].y + acc[2 * m].y,
                          iv[m].z + acc[2 * m + 1].x, iv[m].w + acc[2 * m + 1].y),
              rd, y < h && x < w ? 4 * ((y * w + x) * ldd + ch) : kOOB);
    }
    if (!more) break;
    __syncthreads();                              // halo / coefficients no longer read
    it = nit;
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
// I: index type, 32-bit unsigned when the element count fits (64-bit divisions per element
// made the kernel ALU-bound)
template <typename I>
__global__ __launch_bounds__(256) void warp_fwd_vec(const float* __restrict__ inp, int n, int h,
                                                    int w, int c,
                                                    const float* __restrict__ flow,
                                                    float* __restrict__ out, int absolute) {
  const I nq = c >> 2;
  const I total = (I)n * h * w * nq;
  for (I idx = blockIdx.x * (I)blockDim.x + threadIdx.x; idx < total;
       idx += (I)gridDim.x * blockDim.x) {
    const int64_t p = (int64_t)(idx / nq);
    const int q = (int)(idx % nq);
    const int j = (int)((I)p % (I)w);
    const I t2 = (I)p / (I)w;
    const int i = (int)(t2 % (I)h);
    const int64_t img = (int64_t)(t2 / (I)h) * h * w;
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
                                                     float* __restrict__ dflow, int absolute,
                                                     const float* __restrict__ dfa, int ldfa) {
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
    if (lane == 0) {
      if (dfa) {
        gx = dfa[p * ldfa] + gx;
        gy = dfa[p * ldfa + 1] + gy;
      }
      *reinterpret_cast<float2*>(dflow + 2 * p) = make_float2(gx, gy);
    }
  }
}

// Backward with per-workgroup pre-aggregation of the border scatter (grid + flow,
// c % 64 == 0).  The reference's sampler clips (P2), so samples that leave the image pile onto
// its border pixels, and the transposed grid (P1) sends every column j >= h to row h-1: with
// flows pointing off the image (the coarse levels reach tens of pixels in training) per-pixel
// atomics serialise on a few addresses, 4-17x slower (tools/flow_bench.py --flow-offset).
// A workgroup owns an 8 x 8 output tile, one wave per pixel with lanes over 64 channels (as
// warp_bwd_wave).  Corners inside the image go straight to global atomics (their adders are
// naturally spread); corners ON the border go through a 64-slot direct-mapped LDS cache of
// destination pixels: a corner whose slot is free or already holds its destination is added
// there (ds_add_f32), a collision falls back to a global atomic, and the cache is flushed with
// one 256-B atomic wave-instruction per destination: a clipped run of the tile's pixels leaves
// the workgroup as one add per destination instead of one per pixel and corner.
constexpr int WH_T = 8, WH_SLOTS = 64, WH_WAVES = 16;

__global__ __launch_bounds__(64 * WH_WAVES) void warp_bwd_agg(const float* __restrict__ dout,
                                                    const float* __restrict__ inp, int n, int h,
                                                    int w, int c,
                                                    const float* __restrict__ flow,
                                                    float* __restrict__ dinp,
                                                    float* __restrict__ dflow,
                                                    const float* __restrict__ dfa, int ldfa) {
  __shared__ float data[WH_SLOTS * 64];
  __shared__ int tag[WH_SLOTS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_i = (h + WH_T - 1) / WH_T, tiles_j = (w + WH_T - 1) / WH_T;
  const int passes = c / 64;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int cc = (bid % passes) * 64;                  // this workgroup's 64 channels
  const int tile = bid / passes;
  const int b = tile / (tiles_i * tiles_j);
  const int rem = tile - b * tiles_i * tiles_j;
  const int i0 = (rem / tiles_j) * WH_T, j0 = (rem % tiles_j) * WH_T;
  const int64_t img = (int64_t)b * h * w;

  {
    const int e = cc + lane;
    if (dinp) {
      for (int k = tid; k < WH_SLOTS * 64; k += 64 * WH_WAVES) data[k] = 0.f;
      if (tid < WH_SLOTS) tag[tid] = -1;
    }
    __syncthreads();
    for (int pr = wave; pr < WH_T * WH_T; pr += WH_WAVES) {
      const int i = i0 + pr / WH_T, j = j0 + pr % WH_T;
      if (i >= h || j >= w) continue;                 // wave-uniform
      const int64_t p = img + (int64_t)i * w + j;
      const float2 f = *reinterpret_cast<const float2*>(flow + 2 * p);
      const float x = (float)i + f.x, y = (float)j + f.y;
      const int xi = (int)fmaxf(fminf(floorf(x), 2147483520.f), -2147483520.f);
      const int yi = (int)fmaxf(fminf(floorf(y), 2147483520.f), -2147483520.f);
      const int x0 = min(max(xi, 0), w - 1), x1 = min(max(xi + 1, 0), w - 1);
      const int y0 = min(max(yi, 0), h - 1), y1 = min(max(yi + 1, 0), h - 1);
      const float a = (float)x1 - x, bq = (float)y1 - y;
      const float g = dout[p * c + e];
      const int ys[4] = {y0, y1, y0, y1}, xs[4] = {x0, x0, x1, x1};
      float pv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) pv[k] = inp[(img + (int64_t)ys[k] * w + xs[k]) * c + e];
      float gx = -g * (bq * (pv[0] - pv[2]) + (1.f - bq) * (pv[1] - pv[3]));
      float gy = -g * (a * (pv[0] - pv[1]) + (1.f - a) * (pv[2] - pv[3]));
      if (dinp) {
        const float wt[4] = {a * bq, a * (1.f - bq), (1.f - a) * bq, (1.f - a) * (1.f - bq)};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int yy = ys[k], xx = xs[k];
          const int d = yy * w + xx;
          bool cached = false;
          int sl = 0;
          if (yy == 0 || yy == h - 1 || xx == 0 || xx == w - 1) {   // wave-uniform
            sl = (xx * 7 + yy * 13) & (WH_SLOTS - 1);
            int t = 0;
            if (lane == 0) t = atomicCAS(&tag[sl], -1, d);
            t = __builtin_amdgcn_readfirstlane(t);
            cached = t == -1 || t == d;
          }
          if (cached)
            atomicAdd(&data[sl * 64 + lane], wt[k] * g);
          else
            atomicAdd(dinp + (img + d) * c + e, wt[k] * g);
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        gx += __shfl_xor(gx, o, 64);
        gy += __shfl_xor(gy, o, 64);
      }
      if (lane == 0) {
        if (passes == 1) {
          if (dfa) {
            gx = dfa[p * ldfa] + gx;
            gy = dfa[p * ldfa + 1] + gy;
          }
          *reinterpret_cast<float2*>(dflow + 2 * p) = make_float2(gx, gy);
        } else {                                       // dflow preset by the launcher
          atomicAdd(dflow + 2 * p, gx);
          atomicAdd(dflow + 2 * p + 1, gy);
        }
      }
    }
    if (dinp) {
      __syncthreads();
      for (int sl = wave; sl < WH_SLOTS; sl += WH_WAVES) {
        const int d = tag[sl];
        if (d >= 0) atomicAdd(dinp + (img + d) * c + e, data[sl * 64 + lane]);
      }
      __syncthreads();
    }
  }
}

// Backward with the scatter of a tile turned into a gather (grid + flow, c % 64 == 0).
// Smooth flows send the 4 corners of an 8 x 8 output tile onto a small destination window
// (about 9 x 9 pixels for sub-pixel flows; a clipped tile onto a strip of the border).  The
// workgroup (one 64-channel pass) takes the window's bounding box, counting-sorts its 256
// (pixel, corner) entries by destination (integer LDS atomics for the ranks, a wave scan for
// the bucket starts), and each wave then sums the weighted dout rows of one destination's
// entries in registers (lanes = 64 channels, dout rows staged in LDS) and adds the result to
// global memory once: one 256-B atomic wave-instruction per touched destination, about 1.3 per
// pixel instead of 4.  (Adding the corners into an LDS window with ds_add_f32 instead measured
// slower than the 4 global adds: 524 vs 323 us at 192x256x64, float LDS atomics on repeated
// addresses serialise.)  The flow gradient: lanes work 4 pixels x 16 channel quads (16-byte
// corner loads, a DPP row reduction over the 16 lanes of a pixel).  A tile whose window
// exceeds WG_CAP slots adds each corner's row straight to global memory.
// Timing ablations of warp_bwd_gather (tools/ab_build.sh -DWARP_ABL=mask; wrong results):
// 1 no d(features) atomics (the sums still formed), 2 no d(flow) part.
#ifndef WARP_ABL
#define WARP_ABL 0
#endif
#ifndef WARP_WPE
#define WARP_WPE
#endif
#ifndef WARP_PV_GROUP
#define WARP_PV_GROUP 2
#endif
#ifndef WARP_LATE_PV
#define WARP_LATE_PV 2
#endif
// the flow gradient's corner rows: pv[it][k] = inp row of corner k of pixel group it (lanes
// = 16 channel quads x 4 pixels)
#define warp_corner_rows(I0_, I1_)                                                              \
  _Pragma("unroll") for (int i_ = (I0_); i_ < (I1_); ++i_) {                                   \
    const float2 f = okg[i_] ? fg[i_] : make_float2(0.f, 0.f);                                 \
    int y0, y1, x0, x1;                                                                        \
    float a_, b_;                                                                              \
    corners(pixg[i_] / w, pixg[i_] % w, f, y0, y1, x0, x1, a_, b_);                            \
    const int ys[4] = {y0, y1, y0, y1}, xs[4] = {x0, x0, x1, x1};                              \
    _Pragma("unroll") for (int k = 0; k < 4; ++k) pv[i_][k] =                                  \
        *reinterpret_cast<const float4*>(inp + (img + (int64_t)ys[k] * w + xs[k]) * c + cc + 4 * q); \
  }
#ifndef WARP_CAP
#define WARP_CAP 512   // destination slots: 23.7 KB of LDS = 6 workgroups per CU (1024: 5)
#endif
constexpr int WG_T = 8, WG_CAP = WARP_CAP, WG_NT = 256;
int g_warp_win = 1;   // of_set_tuning key 7: warp_bwd_gather (1) or warp_bwd_agg (0)
int g_corr_blk = 5;   // of_set_tuning key 9: bit 0 corr_fwd_blk (else corr_fwd_kernel), bit 1 corr_bwd_blk,
                      // bit 2 corr_bwd_fused when both gradients are wanted
int g_corr_ty8 = 0;   // of_set_tuning key 19: corr_bwd_kernel on 8 x 16 tiles, 512 threads (1)

__device__ __forceinline__ float row16_sum(float v) {   // sum over the 16 lanes of a DPP row
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x122, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x121, 0xF, 0xF, false));
  return v;                                              // row_ror 8, 4, 2, 1
}

__global__ __launch_bounds__(WG_NT) WARP_WPE void warp_bwd_gather(const float* __restrict__ dout,
                                                         const float* __restrict__ inp, int n,
                                                         int h, int w, int c,
                                                         const float* __restrict__ flow,
                                                         float* __restrict__ dinp,
                                                         float* __restrict__ dflow,
                                                         const float* __restrict__ dfa, int ldfa) {
  constexpr int NP = WG_T * WG_T;                       // 64 pixels, 256 (pixel, corner) entries
  __shared__ float dtile[NP * 64];                     // dout rows of this pass
  __shared__ int2 ent[NP * 4];                         // entries sorted by destination
  __shared__ int cnt[WG_CAP], st[WG_CAP];              // per destination slot: count, start
  __shared__ int nzs[NP * 4];                          // touched slots
  __shared__ int bb[5];                                // min/max row, min/max col, #touched
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_i = (h + WG_T - 1) / WG_T, tiles_j = (w + WG_T - 1) / WG_T;
  const int passes = c / 64;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int cc = (bid % passes) * 64;
  const int tile = bid / passes;
  const int b = tile / (tiles_i * tiles_j);
  const int rem = tile - b * tiles_i * tiles_j;
  const int i0 = (rem / tiles_j) * WG_T, j0 = (rem % tiles_j) * WG_T;
  const int64_t img = (int64_t)b * h * w;

  // corners of pixel (i, j): rows {y0, y1} x columns {x0, x1} (the reference's transposed grid)
  auto corners = [&](int i, int j, float2 f, int& y0, int& y1, int& x0, int& x1, float& a,
                     float& bq) {
    const float x = (float)i + f.x, y = (float)j + f.y;
    const int xi = (int)fmaxf(fminf(floorf(x), 2147483520.f), -2147483520.f);
    const int yi = (int)fmaxf(fminf(floorf(y), 2147483520.f), -2147483520.f);
    x0 = min(max(xi, 0), w - 1), x1 = min(max(xi + 1, 0), w - 1);
    y0 = min(max(yi, 0), h - 1), y1 = min(max(yi + 1, 0), h - 1);
    a = (float)x1 - x, bq = (float)y1 - y;
  };
  auto tile_pix = [&](int p, bool& ok) {
    const int i = i0 + p / WG_T, j = j0 + p % WG_T;
    ok = i < h && j < w;
    return img + (int64_t)min(i, h - 1) * w + min(j, w - 1);
  };

  // ---- loads in three batches, each waited for once (tile pixels are clamped into the
  // image, so every address is valid and no load sits behind a branch; a guarded load per
  // element compiled to a wait per element, and each flow wait also drained the corner loads
  // issued before it): (1) the flows, the tile's dout rows and the added flow gradients,
  // (2) the corner rows, which need the flows, (3) nothing: dout and dfa arrive meanwhile.
  constexpr int IT = NP / (4 * WG_NT / 64), DU = NP * 16 / WG_NT;
  const int q = lane & 15, pg = lane >> 4;
  const int pe = tid >> 2, ke = tid & 3;               // this thread's (pixel, corner) entry
  bool okg[IT], oke;
  int pixg[IT];                                        // pixel index within the image
  float2 fg[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    pixg[it] = (int)(tile_pix((it * (WG_NT / 64) + wave) * 4 + pg, okg[it]) - img);
    fg[it] = *reinterpret_cast<const float2*>(flow + 2 * (img + pixg[it]));
  }
  const int64_t pxe = tile_pix(pe, oke);
  const float2 fe = *reinterpret_cast<const float2*>(flow + 2 * pxe);
  float4 dv[DU];
#pragma unroll
  for (int u = 0; u < DU; ++u) {
    bool ok;
    const int v = tid + u * WG_NT;
    dv[u] = *reinterpret_cast<const float4*>(dout + tile_pix(v >> 4, ok) * c + cc + 4 * (v & 15));
  }
  float fax[IT], fay[IT];                              // dfa (passes == 1 only; else unused)
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    fax[it] = dfa ? dfa[(img + pixg[it]) * ldfa] : 0.f;
    fay[it] = dfa ? dfa[(img + pixg[it]) * ldfa + 1] : 0.f;
  }
#if !WARP_LATE_PV
  float4 pv[IT][4];
  warp_corner_rows(0, IT);
#endif
  int ye = 0, xe = 0;
  float wte = 0.f;
  {
    int y0, y1, x0, x1;
    float a, bq;
    corners((int)(pxe - img) / w, (int)((pxe - img) % w), oke ? fe : make_float2(0.f, 0.f), y0,
            y1, x0, x1, a, bq);
    ye = (ke & 1) ? y1 : y0;
    xe = (ke & 2) ? x1 : x0;
    wte = ((ke & 2) ? 1.f - a : a) * ((ke & 1) ? 1.f - bq : bq);
  }
  // ---- dout rows of the tile -> LDS (out-of-image pixels: zero rows)
#pragma unroll
  for (int u = 0; u < DU; ++u) {
    const int v = tid + u * WG_NT;
    bool ok;
    (void)tile_pix(v >> 4, ok);
    *reinterpret_cast<float4*>(&dtile[(v >> 4) * 64 + 4 * (v & 15)]) =
        ok ? dv[u] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (dinp) {
    if (tid == 0) bb[0] = INT32_MAX, bb[1] = -1, bb[2] = INT32_MAX, bb[3] = -1;
    __syncthreads();
    int v0 = oke ? ye : INT32_MAX, v1 = oke ? ye : -1, v2 = oke ? xe : INT32_MAX, v3 = oke ? xe : -1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      v0 = min(v0, __shfl_xor(v0, o, 64));
      v1 = max(v1, __shfl_xor(v1, o, 64));
      v2 = min(v2, __shfl_xor(v2, o, 64));
      v3 = max(v3, __shfl_xor(v3, o, 64));
    }
    if (lane == 0) {
      atomicMin(&bb[0], v0);
      atomicMax(&bb[1], v1);
      atomicMin(&bb[2], v2);
      atomicMax(&bb[3], v3);
    }
  }
  __syncthreads();                                     // dtile and the bounding box
#if WARP_LATE_PV == 1
  // the corner rows for the flow gradient are loaded here, after the dout rows went to LDS:
  // they arrive during the destination sort and the gather, and the 64 registers they take
  // are not live together with the dout rows (156 -> fewer VGPRs, more workgroups per CU)
  float4 pv[IT][4];
  warp_corner_rows(0, IT);
#endif
  if (dinp) {
    const int wy0 = bb[0], wx0 = bb[2], wwx = bb[3] - wx0 + 1;
    const int wsz = (bb[1] - wy0 + 1) * wwx;
    if (bb[1] >= 0 && wsz <= WG_CAP) {
      for (int k = tid; k < wsz; k += WG_NT) cnt[k] = 0;
      __syncthreads();
      const int slot = (ye - wy0) * wwx + (xe - wx0);
      const int rank = oke ? atomicAdd(&cnt[slot], 1) : 0;
      __syncthreads();
      if (wave == 0) {                                 // bucket starts + touched-slot list
        const int per = (wsz + 63) / 64, k0 = min(wsz, lane * per), k1 = min(wsz, k0 + per);
        int sum = 0, nz = 0;
        for (int k = k0; k < k1; ++k) sum += cnt[k], nz += cnt[k] > 0;
        int isum = sum, inz = nz;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int ts = __shfl_up(isum, o, 64), tn = __shfl_up(inz, o, 64);
          if (lane >= o) isum += ts, inz += tn;
        }
        int run = isum - sum, nzp = inz - nz;
        for (int k = k0; k < k1; ++k) {
          const int ck = cnt[k];
          st[k] = run;
          run += ck;
          if (ck > 0) nzs[nzp++] = k;
        }
        if (lane == 63) bb[4] = inz;
      }
      __syncthreads();
      if (oke) ent[st[slot] + rank] = make_int2(pe, __float_as_int(wte));
      __syncthreads();
      const int nnz = bb[4];
      for (int u = wave; u < nnz; u += WG_NT / 64) {
        const int k = nzs[u], s0 = st[k], ne = cnt[k];
        float acc = 0.f;
        for (int e2 = 0; e2 < ne; ++e2) {
          const int2 en = ent[s0 + e2];
          acc += __int_as_float(en.y) * dtile[en.x * 64 + lane];
        }
        const int yy = wy0 + k / wwx, xx = wx0 + k % wwx;
        if (WARP_ABL & 1) {
          if (acc == 12345.f) dinp[0] = acc;             // keep the sum live
        } else {
          atomicAdd(dinp + (img + (int64_t)yy * w + xx) * c + cc + lane, acc);
        }
      }
    } else {                                           // spread flows: one add per corner
      ent[tid] = make_int2(oke ? (ye * w + xe) : -1, __float_as_int(wte));
      __syncthreads();
      for (int u = wave; u < NP * 4; u += WG_NT / 64) {
        const int2 en = ent[u];
        if (en.x < 0) continue;                        // wave-uniform
        atomicAdd(dinp + (img + en.x) * c + cc + lane,
                  __int_as_float(en.y) * dtile[(u >> 2) * 64 + lane]);
      }
    }
  }
  // ---- flow gradient
#if WARP_LATE_PV == 2
  float4 pv[IT][4];
#endif
#pragma unroll
  for (int it = 0; it < (WARP_ABL & 2 ? 0 : IT); ++it) {
#if WARP_LATE_PV == 2
    if (it % WARP_PV_GROUP == 0) {                     // corner rows in groups: fewer VGPRs
      asm volatile("" ::: "memory");
      warp_corner_rows(it, it + WARP_PV_GROUP);
    }
#endif
    const int pr = (it * (WG_NT / 64) + wave) * 4 + pg;
    float a, bq;                                       // recomputed: 8 registers fewer
    {
      int y0, y1, x0, x1;
      corners(pixg[it] / w, pixg[it] % w, okg[it] ? fg[it] : make_float2(0.f, 0.f), y0, y1, x0,
              x1, a, bq);
    }
    const float4 g = *reinterpret_cast<const float4*>(&dtile[pr * 64 + 4 * q]);
    const float4* P = pv[it];
    auto dot = [](float4 u, float4 v) { return u.x * v.x + u.y * v.y + u.z * v.z + u.w * v.w; };
    auto sub = [](float4 u, float4 v) { return make_float4(u.x - v.x, u.y - v.y, u.z - v.z, u.w - v.w); };
    float gx = -(bq * dot(g, sub(P[0], P[2])) + (1.f - bq) * dot(g, sub(P[1], P[3])));
    float gy = -(a * dot(g, sub(P[0], P[1])) + (1.f - a) * dot(g, sub(P[2], P[3])));
    gx = row16_sum(gx);
    gy = row16_sum(gy);
    if (q == 0 && okg[it]) {
      if (passes == 1) {
        *reinterpret_cast<float2*>(dflow + 2 * (img + pixg[it])) = make_float2(fax[it] + gx, fay[it] + gy);
      } else {                                         // dflow preset by the launcher
        atomicAdd(dflow + 2 * (img + pixg[it]), gx);
        atomicAdd(dflow + 2 * (img + pixg[it]) + 1, gy);
      }
    }
  }
}

__global__ __launch_bounds__(256) void warp_bwd_scalar(const float* __restrict__ dout,
                                                       const float* __restrict__ inp, int n,
                                                       int h, int w, int c,
                                                       const float* __restrict__ flow,
                                                       float* __restrict__ dinp,
                                                       float* __restrict__ dflow, int absolute,
                                                       const float* __restrict__ dfa, int ldfa) {
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
    dflow[2 * p] = dfa ? dfa[p * ldfa] + gx : gx;
    dflow[2 * p + 1] = dfa ? dfa[p * ldfa + 1] + gy : gy;
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
                                                            float* __restrict__ din, int accum,
                                                            int lddi) {
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
    const int64_t o = p * lddi + e;
    din[o] = accum ? din[o] + s : s;
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

// All levels in one launch (the per-level launches were ~5 us each, latency-bound): element
// idx of the concatenation of the levels' outputs; level l + 1 starts at begin[l].
struct PyrArgs {
  float* out[8];
  int64_t begin[9];
  int levels;
};
__global__ __launch_bounds__(256) void pyramid6_multi(const float* __restrict__ in, int n, int H,
                                                      int W, PyrArgs pa) {
  const int64_t total = pa.begin[pa.levels];
  for (int64_t gi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; gi < total;
       gi += (int64_t)gridDim.x * blockDim.x) {
    int l = 0;
    while (l + 1 < pa.levels && gi >= pa.begin[l + 1]) ++l;
    const int64_t idx = gi - pa.begin[l];
    const int f = 2 << l;
    const int h = H / f, w = W / f;
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
    pa.out[l][idx] = top + (bot - top) * 0.5f;
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

// The photometric loss of every scale in one launch: level l's blocks are [bbeg[l], bbeg[l+1])
// (forward: one partial per block, the partial arrays concatenated in level order) or its
// pixels [pbeg[l], pbeg[l+1]) (backward: d(flow) of level l at row stride ld[l]).
struct PhotoMulti {
  const float* img6[8];
  const float* flow[8];
  float* dflow[8];
  int ld[8];
  float coef[8];
  int h[8], w[8];
  int64_t beg[9];
  int levels;
};
__global__ __launch_bounds__(PL_THREADS) void photo_l1_fwd_multi(int n, PhotoMulti m,
                                                                 float* __restrict__ partials) {
  int l = 0;
  while (l + 1 < m.levels && (int64_t)blockIdx.x >= m.beg[l + 1]) ++l;
  const int h = m.h[l], w = m.w[l];
  const float* img6 = m.img6[l];
  const float* flow = m.flow[l];
  const int64_t npix = (int64_t)n * h * w;
  const int64_t p0 = ((int64_t)blockIdx.x - m.beg[l]) * PL_PIX_PER_BLOCK;
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

__global__ __launch_bounds__(256) void photo_l1_bwd_multi(int n, PhotoMulti m,
                                                          const float* __restrict__ dloss) {
  const int64_t total = m.beg[m.levels];
  const float dl = dloss ? dloss[0] : 1.f;
  for (int64_t gp = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; gp < total;
       gp += (int64_t)gridDim.x * blockDim.x) {
    int l = 0;
    while (l + 1 < m.levels && gp >= m.beg[l + 1]) ++l;
    const int h = m.h[l], w = m.w[l];
    const float* img6 = m.img6[l];
    const float* flow = m.flow[l];
    const int64_t p = gp - m.beg[l];
    const int j = (int)(p % w);
    const int64_t t2 = p / w;
    const int i = (int)(t2 % h);
    const int64_t img = (t2 / h) * h * w;
    float diff[3], v[4][3];
    WarpTap t;
    photo_sample(img6, p, i, j, flow[2 * p], flow[2 * p + 1], h, w, img, diff, t, v);
    const float a = t.a, b = t.b, coef = m.coef[l] * dl;
    float gx = 0.f, gy = 0.f;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const float sg = diff[e] > 0.f ? 1.f : (diff[e] < 0.f ? -1.f : 0.f);
      const float g = -coef * sg;
      gx -= g * (b * (v[0][e] - v[2][e]) + (1.f - b) * (v[1][e] - v[3][e]));
      gy -= g * (a * (v[0][e] - v[1][e]) + (1.f - a) * (v[2][e] - v[3][e]));
    }
    m.dflow[l][m.ld[l] * p] = gx;
    m.dflow[l][m.ld[l] * p + 1] = gy;
  }
}

__global__ __launch_bounds__(256) void photo_l1_bwd_kernel(const float* __restrict__ img6,
                                                           const float* __restrict__ flow, int n,
                                                           int h, int w, float coef,
                                                           const float* __restrict__ dloss,
                                                           float* __restrict__ dflow, int lddf) {
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
    dflow[lddf * p] = gx;
    dflow[lddf * p + 1] = gy;
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

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Slab groups of the register-blocked forward: the fewest that give >= 2 * CUs (512 on
// MI355X) (tile, group) items, one per workgroup slot of the persistent grid (96x128x64: one group of 768 tiles
// ran 38 us + no slab sum against 38 + 12 us with two groups).
static void corr_blk_plan(int n, int h, int w, int c, CorrBlkArgs& p) {
  p.slabs = (int)cdiv(c, CB_SC);
  p.tiles_x = (int)cdiv(w, CB_X), p.tiles_y = (int)cdiv(h, CB_Y);
  const int64_t tiles = (int64_t)n * p.tiles_x * p.tiles_y;
  const int want = (int)std::min<int64_t>(p.slabs, std::max<int64_t>(1, cdiv(2 * device_cus(), tiles)));
  p.spg = (int)cdiv(p.slabs, want);
  p.groups = (int)cdiv(p.slabs, p.spg);
  p.items = (int)(tiles * p.groups);
}

// Persistent grid: two workgroups per CU, a multiple of 8 (one partition per XCD) from 64 up.
static int corr_blk_grid(int items) {
  const int g = std::min(items, 2 * device_cus());
  return g >= 64 ? g & ~7 : g;
}

static size_t corr_fwd_ws(int n, int h, int w, int c) {
  const int slabs = (int)cdiv(c, CSLAB);
  CorrBlkArgs p{};
  corr_blk_plan(n, h, w, c, p);
  const int parts = std::max(slabs > 1 ? slabs : 0, p.groups > 1 ? p.groups : 0);
  return (size_t)parts * n * h * w * 49 * sizeof(float);
}

static int corr_fwd_launch(CorrFwdArgs a, int n, void* ws, size_t ws_bytes, void* stream) {
  OF_CHECK_ARG((int64_t)a.h * a.w * std::max(std::max(a.ld1, a.ld2), a.ldcv) < (1LL << 29),
               "corr: one image must hold < 2^29 elements (32-bit buffer offsets)");
  const size_t need = corr_fwd_ws(n, a.h, a.w, a.c);
  OF_CHECK_ARG(ws_bytes >= need && (need == 0 || ws), "corr fwd: workspace too small");
  a.part = static_cast<float*>(ws);
  hipStream_t s = as_stream(stream);
  if (g_corr_blk & 1) {
    CorrBlkArgs p{};
    p.a = a;
    corr_blk_plan(n, a.h, a.w, a.c, p);
    OF_CHECK_ARG((int64_t)n * p.tiles_x * p.tiles_y * p.groups < INT32_MAX, "corr fwd: too many tiles");
    const int grid = corr_blk_grid(p.items);
    if (a.vec)
      hipLaunchKernelGGL(corr_fwd_blk<true>, dim3(grid), dim3(CB_NT), 0, s, p);
    else
      hipLaunchKernelGGL(corr_fwd_blk<false>, dim3(grid), dim3(CB_NT), 0, s, p);
    int st = check_launch("corr_fwd_blk");
    if (st || p.groups == 1) return st;
    const int64_t npix = (int64_t)n * a.h * a.w;
    hipLaunchKernelGGL(corr_slab_sum_kernel, dim3(grid_for(npix * 49)), dim3(256), 0, s, a.part,
                       p.groups, npix, 49, a.cv, a.ldcv);
    return check_launch("corr_slab_sum");
  }
  a.slabs = (int)cdiv(a.c, CSLAB);
  a.tiles_x = (int)cdiv(a.w, CT_X), a.tiles_y = (int)cdiv(a.h, CT_Y);
  const dim3 grid((unsigned)((int64_t)a.tiles_x * a.tiles_y * n * a.slabs));
  if (a.vec)
    hipLaunchKernelGGL((corr_fwd_kernel<3, true>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((corr_fwd_kernel<3, false>), grid, dim3(256), 0, s, a);
  int st = check_launch("corr_fwd");
  if (st || a.slabs == 1) return st;
  const int64_t npix = (int64_t)n * a.h * a.w;
  hipLaunchKernelGGL(corr_slab_sum_kernel, dim3(grid_for(npix * 49)), dim3(256), 0, s, a.part,
                     a.slabs, npix, 49, a.cv, a.ldcv);
  return check_launch("corr_slab_sum");
}

static int corr_bwd_launch(int sign, CorrBwdArgs a, int n, hipStream_t s) {
  OF_CHECK_ARG((int64_t)a.h * a.w * std::max(std::max(a.ldg, a.lds), std::max(a.lddf, a.ldinit)) <
                   (1LL << 29),
               "corr: one image must hold < 2^29 elements (32-bit buffer offsets)");
  if (g_corr_blk & 2) {
    CorrBlkArgs p{};
    corr_blk_plan(n, a.h, a.w, a.c, p);
    OF_CHECK_ARG((int64_t)n * p.tiles_x * p.tiles_y * p.groups < INT32_MAX, "corr bwd: too many tiles");
    a.tiles_x = p.tiles_x, a.tiles_y = p.tiles_y;
    const int grid = corr_blk_grid(p.items);
    auto k = sign > 0 ? (a.vec ? corr_bwd_blk<1, true> : corr_bwd_blk<1, false>)
                      : (a.vec ? corr_bwd_blk<-1, true> : corr_bwd_blk<-1, false>);
    hipLaunchKernelGGL(k, dim3(grid), dim3(CBB_NT), 0, s, a, p.slabs, p.spg, p.groups, p.items);
    return check_launch(sign > 0 ? "corr_bwd_blk_f1" : "corr_bwd_blk_f2");
  }
  a.slabs = (int)cdiv(a.c, CSLAB);
  const int ty = g_corr_ty8 ? 2 * CT_Y : CT_Y;
  a.tiles_x = (int)cdiv(a.w, CT_X), a.tiles_y = (int)cdiv(a.h, ty);
  const dim3 grid((unsigned)((int64_t)a.tiles_x * a.tiles_y * n * a.slabs));
  if (g_corr_ty8) {
    const dim3 blk(4 * 2 * CT_Y * CT_X);
    if (sign > 0 && a.vec)
      hipLaunchKernelGGL((corr_bwd_kernel<3, 1, true, 2 * CT_Y>), grid, blk, 0, s, a);
    else if (sign > 0)
      hipLaunchKernelGGL((corr_bwd_kernel<3, 1, false, 2 * CT_Y>), grid, blk, 0, s, a);
    else if (a.vec)
      hipLaunchKernelGGL((corr_bwd_kernel<3, -1, true, 2 * CT_Y>), grid, blk, 0, s, a);
    else
      hipLaunchKernelGGL((corr_bwd_kernel<3, -1, false, 2 * CT_Y>), grid, blk, 0, s, a);
  } else if (sign > 0 && a.vec)
    hipLaunchKernelGGL((corr_bwd_kernel<3, 1, true>), grid, dim3(256), 0, s, a);
  else if (sign > 0)
    hipLaunchKernelGGL((corr_bwd_kernel<3, 1, false>), grid, dim3(256), 0, s, a);
  else if (a.vec)
    hipLaunchKernelGGL((corr_bwd_kernel<3, -1, true>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((corr_bwd_kernel<3, -1, false>), grid, dim3(256), 0, s, a);
  return check_launch(sign > 0 ? "corr_bwd_f1" : "corr_bwd_f2");
}

// Both gradients in one pass (corr_bwd_fused); false: the caller runs the per-gradient kernels.
static bool corr_fused_ok(const float* g, int ldg, int c, const float* f1, int ld1,
                          const float* f2, int ld2, const float* df1, int lddf1,
                          const float* init1, int ldinit1, const float* df2, int lddf2) {
  // (the coefficient quads read g[48 .. 51] of each pixel: ldg >= 52)
  return (g_corr_blk & 4) && df1 && df2 && c % FB_SC == 0 && ldg % 4 == 0 && ldg >= 52 &&
         al16(g) && ld1 % 4 == 0 && ld2 % 4 == 0 &&
         lddf1 % 4 == 0 && lddf2 % 4 == 0 && (!init1 || (ldinit1 % 4 == 0 && al16(init1))) &&
         al16(f1) && al16(f2) && al16(df1) && al16(df2);
}

static int corr_fused_launch(CorrFusedArgs a, int n, hipStream_t s) {
  OF_CHECK_ARG((int64_t)a.h * a.w *
                       std::max(std::max(std::max(a.ldg, a.ld1), std::max(a.ld2, a.lddf1)),
                                std::max(std::max(a.lddf2, a.ldinit1), a.ldinit2)) <
                   (1LL << 29),
               "corr: one image must hold < 2^29 elements (32-bit buffer offsets)");
  a.slabs = a.c / FB_SC;
  a.tiles_x = (int)cdiv(a.w, FB_X), a.tiles_y = (int)cdiv(a.h, FB_Y);
  const int64_t items = (int64_t)n * a.tiles_x * a.tiles_y * a.slabs;
  OF_CHECK_ARG(items < INT32_MAX / 2, "corr bwd: too many tiles");
  a.items = (int)items;
  const int grid = (int)std::min<int64_t>(items, device_cus());
  hipLaunchKernelGGL(corr_bwd_fused, dim3(grid), dim3(FB_NT), 0, s, a);
  return check_launch("corr_bwd_fused");
}

size_t of_corr_fwd_workspace(int n, int h, int w, int c, int max_disp) {
  (void)max_disp;
  return n > 0 && h > 0 && w > 0 && c > 0 ? corr_fwd_ws(n, h, w, c) : 0;
}

int of_corr_fwd(const float* f1, int ld1, const float* f2, int ld2, int n, int h, int w, int c,
                int max_disp, float* out, int ldo, void* workspace, size_t ws_bytes,
                void* stream) {
  OF_CHECK_ARG(f1 && f2 && out, "corr fwd: NULL pointer");
  OF_CHECK_ARG(max_disp == 3, "corr: only max_disp=3 (the reference default) is compiled");
  OF_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0, "corr fwd: dims");
  OF_CHECK_ARG(ld1 >= c && ld2 >= c && ldo >= 49, "corr fwd: strides");
  CorrFwdArgs a{};
  a.f1 = f1, a.ld1 = ld1, a.f2 = f2, a.ld2 = ld2, a.h = h, a.w = w, a.c = c;
  a.cv = out, a.ldcv = ldo;
  a.vec = c % 4 == 0 && ld1 % 4 == 0 && ld2 % 4 == 0 && al16(f1) && al16(f2);
  return corr_fwd_launch(a, n, workspace, ws_bytes, stream);
}

int of_corr_bwd(const float* dcv, int lddcv, const float* f1, int ld1, const float* f2, int ld2,
                int n, int h, int w, int c, int max_disp, float* df1, int lddf1, int acc1,
                float* df2, int lddf2, int acc2, void* stream) {
  OF_CHECK_ARG(dcv && f1 && f2, "corr bwd: NULL pointer");
  OF_CHECK_ARG(max_disp == 3, "corr: only max_disp=3 (the reference default) is compiled");
  OF_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0, "corr bwd: dims");
  OF_CHECK_ARG(ld1 >= c && ld2 >= c && lddcv >= 49, "corr bwd: strides");
  hipStream_t s = as_stream(stream);
  int st;
  if (corr_fused_ok(dcv, lddcv, c, f1, ld1, f2, ld2, df1, lddf1, acc1 ? df1 : nullptr, lddf1, df2,
                    lddf2)) {
    OF_CHECK_ARG(lddf1 >= c && lddf2 >= c, "corr bwd: df strides");
    CorrFusedArgs a{};
    a.g = dcv, a.ldg = lddcv, a.f1 = f1, a.ld1 = ld1, a.f2 = f2, a.ld2 = ld2;
    a.df1 = df1, a.lddf1 = lddf1, a.init1 = acc1 ? df1 : nullptr, a.ldinit1 = lddf1;
    a.df2 = df2, a.lddf2 = lddf2, a.init2 = acc2 ? df2 : nullptr, a.ldinit2 = lddf2;
    a.h = h, a.w = w, a.c = c;
    return corr_fused_launch(a, n, s);
  }
  if (df1) {
    OF_CHECK_ARG(lddf1 >= c, "corr bwd: df1 stride");
    CorrBwdArgs a{};
    a.g = dcv, a.ldg = lddcv, a.src = f2, a.lds = ld2, a.h = h, a.w = w, a.c = c;
    a.df = df1, a.lddf = lddf1, a.init = acc1 ? df1 : nullptr, a.ldinit = lddf1;
    a.vec = c % 4 == 0 && ld2 % 4 == 0 && lddf1 % 4 == 0 && al16(f2) && al16(df1);
    if ((st = corr_bwd_launch(1, a, n, s))) return st;
  }
  if (df2) {
    OF_CHECK_ARG(lddf2 >= c, "corr bwd: df2 stride");
    CorrBwdArgs a{};
    a.g = dcv, a.ldg = lddcv, a.src = f1, a.lds = ld1, a.h = h, a.w = w, a.c = c;
    a.df = df2, a.lddf = lddf2, a.init = acc2 ? df2 : nullptr, a.ldinit = lddf2;
    a.vec = c % 4 == 0 && ld1 % 4 == 0 && lddf2 % 4 == 0 && al16(f1) && al16(df2);
    if ((st = corr_bwd_launch(-1, a, n, s))) return st;
  }
  return OF_OK;
}

int of_corr_concat_fwd(const float* f1, const float* f2, const float* flow, int n, int h, int w,
                       int c, int max_disp, float* cat, int cp, void* workspace, size_t ws_bytes,
                       void* stream) {
  OF_CHECK_ARG(f1 && f2 && cat, "corr concat fwd: NULL pointer");
  OF_CHECK_ARG(max_disp == 3, "corr: only max_disp=3 (the reference default) is compiled");
  OF_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0, "corr concat fwd: dims");
  OF_CHECK_ARG(cp >= c + 49 + (flow ? 2 : 0), "corr concat fwd: cp too small");
  CorrFwdArgs a{};
  a.f1 = f1, a.ld1 = c, a.f2 = f2, a.ld2 = c, a.h = h, a.w = w, a.c = c;
  a.cv = cat + c, a.ldcv = cp, a.cat = cat, a.flow = flow;
  a.vec = c % 4 == 0 && cp % 4 == 0 && al16(f1) && al16(f2) && al16(cat);
  return corr_fwd_launch(a, n, workspace, ws_bytes, stream);
}

int of_corr_concat_fwd16(const float* f1, const float* f2, const float* flow, int n, int h,
                         int w, int c, int max_disp, void* cat16, int ld16, void* stream) {
  OF_CHECK_ARG(f1 && f2 && cat16, "corr concat fwd16: NULL pointer");
  OF_CHECK_ARG(max_disp == 3, "corr: only max_disp=3 (the reference default) is compiled");
  OF_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0, "corr concat fwd16: dims");
  OF_CHECK_ARG(ld16 >= c + 49 + (flow ? 2 : 0) && ld16 % 4 == 0, "corr concat fwd16: ld16");
  OF_CHECK_ARG(al16(f1) && al16(f2) && ((uintptr_t)cat16 & 7) == 0, "corr concat fwd16: alignment");
  OF_CHECK_ARG((int64_t)h * w * std::max(c, ld16) < (1LL << 29),
               "corr: one image must hold < 2^29 elements (32-bit buffer offsets)");
  CorrBlkArgs p{};
  p.a.f1 = f1, p.a.ld1 = c, p.a.f2 = f2, p.a.ld2 = c, p.a.h = h, p.a.w = w, p.a.c = c;
  p.a.flow = flow, p.a.vec = 1;
  p.a.cat16 = static_cast<uint16_t*>(cat16), p.a.ld16 = ld16;
  corr_blk_plan(n, h, w, c, p);
  if (p.groups != 1) return fail(OF_EINVAL, "corr concat fwd16: the grid needs slab groups "
                                 "(small level): use of_corr_concat_fwd");
  const int grid = corr_blk_grid(p.items);
  hipLaunchKernelGGL(corr_fwd_blk<true>, dim3(grid), dim3(CB_NT), 0, as_stream(stream), p);
  return check_launch("corr_fwd_blk (bf16 image)");
}

int of_corr_concat_fwd16_ok(int n, int h, int w, int c) {
  CorrBlkArgs p{};
  corr_blk_plan(n, h, w, c, p);
  return c % 4 == 0 && p.groups == 1;
}

int of_corr_concat_bwd(const float* dcat, int cp, const float* f1, const float* f2, int n, int h,
                       int w, int c, int max_disp, float* df1, float* df2, float* dflow,
                       void* stream) {
  OF_CHECK_ARG(dcat && f1 && f2 && df1, "corr concat bwd: NULL pointer");
  OF_CHECK_ARG(max_disp == 3, "corr: only max_disp=3 (the reference default) is compiled");
  OF_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0, "corr concat bwd: dims");
  OF_CHECK_ARG(cp >= c + 49 + (dflow ? 2 : 0), "corr concat bwd: cp too small");
  hipStream_t s = as_stream(stream);
  const bool vec = c % 4 == 0 && cp % 4 == 0 && al16(f1) && al16(f2) && al16(dcat) && al16(df1);
  int st;
  if (corr_fused_ok(dcat + c, cp, c, f1, c, f2, c, df1, c, dcat, cp, df2, c)) {
    CorrFusedArgs f{};
    f.g = dcat + c, f.ldg = cp, f.f1 = f1, f.ld1 = c, f.f2 = f2, f.ld2 = c;
    f.df1 = df1, f.lddf1 = c, f.init1 = dcat, f.ldinit1 = cp;
    f.df2 = df2, f.lddf2 = c;
    f.h = h, f.w = w, f.c = c;
    if ((st = corr_fused_launch(f, n, s))) return st;
    if (dflow)
      return of_copy_strided(dcat + c + 49, cp, dflow, 2, (int64_t)n * h * w, 2, stream);
    return OF_OK;
  }
  CorrBwdArgs a{};
  a.g = dcat + c, a.ldg = cp, a.src = f2, a.lds = c, a.h = h, a.w = w, a.c = c;
  a.df = df1, a.lddf = c, a.init = dcat, a.ldinit = cp, a.vec = vec;
  if ((st = corr_bwd_launch(1, a, n, s))) return st;
  if (df2) {
    a.src = f1, a.df = df2, a.init = nullptr, a.vec = vec && al16(df2);
    if ((st = corr_bwd_launch(-1, a, n, s))) return st;
  }
  if (dflow)
    return of_copy_strided(dcat + c + 49, cp, dflow, 2, (int64_t)n * h * w, 2, stream);
  return OF_OK;
}

static int warp_fwd_impl(const float* inp, int n, int h, int w, int c, const float* flow,
                         float* out, int absolute, void* stream) {
  OF_CHECK_ARG(inp && flow && out, "warp fwd: NULL pointer");
  OF_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0, "warp fwd: dims");
  hipStream_t s = as_stream(stream);
  const int64_t npix = (int64_t)n * h * w;
  if (c % 4 == 0 && ((uintptr_t)inp & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    const int64_t total = npix * (c / 4);
    if (total + (int64_t)grid_for(total) * 256 < (int64_t)UINT32_MAX)
      hipLaunchKernelGGL(warp_fwd_vec<uint32_t>, dim3(grid_for(total)), dim3(256), 0, s, inp, n,
                         h, w, c, flow, out, absolute);
    else
      hipLaunchKernelGGL(warp_fwd_vec<int64_t>, dim3(grid_for(total)), dim3(256), 0, s, inp, n,
                         h, w, c, flow, out, absolute);
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

// dfa (row stride ldfa, 2 channels), when given, is added to d(flow): the gradient of the flow
// through its other consumer (the concat's flow slice), so no separate add pass runs.
static int warp_bwd_impl(const float* dout, const float* inp, int n, int h, int w, int c,
                         const float* flow, float* dinp, float* dflow, int absolute,
                         void* stream, const float* dfa = nullptr, int ldfa = 0) {
  OF_CHECK_ARG(dout && inp && flow && dflow, "warp bwd: NULL pointer");
  OF_CHECK_ARG(!dfa || ldfa >= 2, "warp bwd: ld of the added flow gradient");
  hipStream_t s = as_stream(stream);
  const int64_t npix = (int64_t)n * h * w;
  if (!absolute && c % 64 == 0 && (int64_t)h * w < INT32_MAX) {
    if (c > 64) {     // several 64-channel passes add their d(flow) atomically: preset it
      if (dfa) {
        const int st = of_copy_strided(dfa, ldfa, dflow, 2, npix, 2, stream);
        if (st) return st;
      } else if (hipMemsetAsync(dflow, 0, (size_t)npix * 2 * sizeof(float), s) != hipSuccess) {
        return check_launch("warp_bwd: dflow memset");
      }
    }
    if (g_warp_win) {
      const int64_t blocks =
          (int64_t)n * ((h + WG_T - 1) / WG_T) * ((w + WG_T - 1) / WG_T) * (c / 64);
      OF_CHECK_ARG(blocks < INT32_MAX, "warp bwd: too many tiles");
      hipLaunchKernelGGL(warp_bwd_gather, dim3((unsigned)blocks), dim3(WG_NT), 0, s, dout,
                         inp, n, h, w, c, flow, dinp, dflow, c == 64 ? dfa : nullptr, ldfa);
    } else {
      const int64_t blocks =
          (int64_t)n * ((h + WH_T - 1) / WH_T) * ((w + WH_T - 1) / WH_T) * (c / 64);
      OF_CHECK_ARG(blocks < INT32_MAX, "warp bwd: too many tiles");
      hipLaunchKernelGGL(warp_bwd_agg, dim3((unsigned)blocks), dim3(64 * WH_WAVES), 0, s, dout,
                         inp, n, h, w, c, flow, dinp, dflow, c == 64 ? dfa : nullptr, ldfa);
    }
  } else if (c >= 16) {
    const int g = grid_for(npix * 64, 256, 16384);
    hipLaunchKernelGGL(warp_bwd_wave, dim3(g), dim3(256), 0, s, dout, inp, n, h, w, c, flow,
                       dinp, dflow, absolute, dfa, ldfa);
  } else {
    hipLaunchKernelGGL(warp_bwd_scalar, dim3(grid_for(npix)), dim3(256), 0, s, dout, inp, n, h,
                       w, c, flow, dinp, dflow, absolute, dfa, ldfa);
  }
  return check_launch("warp_bwd");
}

int of_warp_bwd(const float* dout, const float* inp, int n, int h, int w, int c,
                const float* flow, float* dinp, float* dflow, void* stream) {
  return warp_bwd_impl(dout, inp, n, h, w, c, flow, dinp, dflow, 0, stream);
}

int of_warp_bwd_add(const float* dout, const float* inp, int n, int h, int w, int c,
                    const float* flow, float* dinp, float* dflow, const float* dflow_add,
                    int ld_add, void* stream) {
  OF_CHECK_ARG(dflow_add, "warp bwd add: NULL dflow_add");
  return warp_bwd_impl(dout, inp, n, h, w, c, flow, dinp, dflow, 0, stream, dflow_add, ld_add);
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

int of_upscale2x_bwd_ld(const float* dout, int lddo, int n, int h, int w, int c, float scale,
                        float* din, int lddi, int accumulate, void* stream) {
  OF_CHECK_ARG(dout && din && lddo >= c && lddi >= c, "upscale bwd: args");
  const int64_t total = (int64_t)n * h * w * c;
  hipLaunchKernelGGL(upscale2x_bwd_kernel, dim3(grid_for(total)), dim3(256), 0,
                     as_stream(stream), dout, lddo, n, h, w, c, scale, din, accumulate, lddi);
  return check_launch("upscale2x_bwd");
}

int of_upscale2x_bwd(const float* dout, int lddo, int n, int h, int w, int c, float scale,
                     float* din, int accumulate, void* stream) {
  return of_upscale2x_bwd_ld(dout, lddo, n, h, w, c, scale, din, c, accumulate, stream);
}

int of_pyramid6(const float* batch, int n, int h, int w, int levels, float* const* outs,
                void* stream) {
  OF_CHECK_ARG(batch && outs && levels >= 1 && levels <= 8, "pyramid: args");
  OF_CHECK_ARG(h % (1 << levels) == 0 && w % (1 << levels) == 0,
               "pyramid: H and W must be divisible by 2^levels (P17)");
  hipStream_t s = as_stream(stream);
  PyrArgs pa{};
  pa.levels = levels;
  pa.begin[0] = 0;
  for (int l = 1; l <= levels; ++l) {
    OF_CHECK_ARG(outs[l - 1], "pyramid: NULL output");
    pa.out[l - 1] = outs[l - 1];
    pa.begin[l] = pa.begin[l - 1] + (int64_t)n * (h >> l) * (w >> l) * 6;
  }
  hipLaunchKernelGGL(pyramid6_multi, dim3(grid_for(pa.begin[levels])), dim3(256), 0, s, batch, n,
                     h, w, pa);
  return check_launch("pyramid6");
}

int of_photo_l1_fwd_multi(const float* const* img6s, const float* const* flows, int n,
                          const int* hs, const int* ws, int levels, float* partials,
                          void* stream) {
  OF_CHECK_ARG(img6s && flows && hs && ws && partials && levels >= 1 && levels <= 8,
               "photo l1 fwd multi: args");
  PhotoMulti m{};
  m.levels = levels;
  m.beg[0] = 0;
  for (int l = 0; l < levels; ++l) {
    OF_CHECK_ARG(img6s[l] && flows[l], "photo l1 fwd multi: NULL level");
    m.img6[l] = img6s[l];
    m.flow[l] = flows[l];
    m.h[l] = hs[l];
    m.w[l] = ws[l];
    m.beg[l + 1] = m.beg[l] + of_photo_l1_partials(n, hs[l], ws[l]);
  }
  hipLaunchKernelGGL(photo_l1_fwd_multi, dim3((unsigned)m.beg[levels]), dim3(PL_THREADS), 0,
                     as_stream(stream), n, m, partials);
  return check_launch("photo_l1_fwd_multi");
}

int of_photo_l1_bwd_multi(const float* const* img6s, const float* const* flows, int n,
                          const int* hs, const int* ws, int levels, const float* coefs,
                          const float* dloss, float* const* dflows, const int* lds,
                          void* stream) {
  OF_CHECK_ARG(img6s && flows && hs && ws && coefs && dflows && lds && levels >= 1 && levels <= 8,
               "photo l1 bwd multi: args");
  PhotoMulti m{};
  m.levels = levels;
  m.beg[0] = 0;
  for (int l = 0; l < levels; ++l) {
    OF_CHECK_ARG(img6s[l] && flows[l] && dflows[l] && lds[l] >= 2, "photo l1 bwd multi: level");
    m.img6[l] = img6s[l];
    m.flow[l] = flows[l];
    m.dflow[l] = dflows[l];
    m.ld[l] = lds[l];
    m.coef[l] = coefs[l];
    m.h[l] = hs[l];
    m.w[l] = ws[l];
    m.beg[l + 1] = m.beg[l] + (int64_t)n * hs[l] * ws[l];
  }
  hipLaunchKernelGGL(photo_l1_bwd_multi, dim3(grid_for(m.beg[levels])), dim3(256), 0,
                     as_stream(stream), n, m, dloss);
  return check_launch("photo_l1_bwd_multi");
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

int of_photo_l1_bwd_ld(const float* img6, const float* flow, int n, int h, int w, float coef,
                       const float* dloss, float* dflow, int lddf, void* stream) {
  OF_CHECK_ARG(img6 && flow && dflow && lddf >= 2, "photo l1 bwd: args");
  hipLaunchKernelGGL(photo_l1_bwd_kernel, dim3(grid_for((int64_t)n * h * w)), dim3(256), 0,
                     as_stream(stream), img6, flow, n, h, w, coef, dloss, dflow, lddf);
  return check_launch("photo_l1_bwd");
}

int of_photo_l1_bwd(const float* img6, const float* flow, int n, int h, int w, float coef,
                    const float* dloss, float* dflow, void* stream) {
  return of_photo_l1_bwd_ld(img6, flow, n, h, w, coef, dloss, dflow, 2, stream);
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
