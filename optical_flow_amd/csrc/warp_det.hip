// Deterministic feature-warp backward ("a deterministic-mode flag (no atomics in
// the warp bwd)"), the default since round 5 (ops.DETERMINISTIC).
//
// The reference samples with four gather_nd taps (transformations.py:98-129, reached from
// warp_features, model.py:55-73); TF's gradient of a gather is a scatter-add into the feature
// map, whose adds land in whatever order the hardware retires them.  The atomic HIP backward
// (flow_ops.hip warp_bwd_gather) keeps that shape: per-tile sums added with float atomics, so
// two identical steps can differ in the last bit of d(features).  Here the scatter becomes a
// gather with a fixed summation order: every destination row sums w_k * dout[p] over its
// (source p, corner k) entries in ascending code 4 p + k, and is STORED once (no zero-fill,
// no float atomics).  Two ways to find a destination's entries:
//
//   window (own_window, relative flows): every destination scans a window of candidate
//     sources in ascending order, 16 candidates a step over 16 lanes, and sums its hits.
//     Mode A (R <= of_set_tuning key 28, R = floor(max |flow|) + 2 from own_radius): a
//     sample lands within R of its source's transposed position (P1's grid), so the window is
//     (2R+1)^2 around it -- complete by construction.  Mode B (larger flows): the window is
//     (2 WIN_RB + 1)^2 around a source position found by two fixed-point steps on the flow
//     (smooth fields: complete); destinations on the image border scan the whole clipped
//     range.  Mode B counts the hits it found; complete iff the count is 4 n h w (each
//     entry lands on exactly one destination, and no window yields a false hit).
//     Destinations on a pile (the last row when w - h > WIN_PILE in mode A: P1 clips every
//     source beyond h onto it; every border pixel in mode B) get a workgroup each.
//   fixed point (absolute points, key 28 = 0, or a mode-B count short of 4 n h w): every
//     contribution rounded to an int64 at a scale set by max |dout| and added with integer
//     atomics (exact, so in any order the same), tile-aggregated in LDS so that samples piled
//     onto the border add once per workgroup; then scaled back (fix_prep / fix_scatter /
//     fix_convert below).  Its kernels return at once when the window served (~5 us a launch).
//   6. d(flow): per source pixel over all channels in a fixed order (16 lanes x channel quads,
//      then a fixed DPP row reduction), plus the optional addend of of_warp_bwd_add -- in
//      own_window (its loads issued before the window's), or its own kernel.
//
// Bitwise reproducible run to run, in eager mode and inside a captured graph alike (the mode,
// the windows and the path are functions of the flow and dout).
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


// Workspace header (ints, zeroed per call): four banks of DET_SLOTS counters 256 B apart
// (spread atomics: a grid's worth of atomics on one word serialises): the hits mode B found
// (summed), and R, the roughness V and max |dout| (float bits) (each the max over its bank).
constexpr int DET_SLOTS = 32;
constexpr int DET_FOUND = 1, DET_RAD = 33, DET_ROUGH = 65, DET_MAXD = 97;   // bank bases
constexpr int DET_HDR_INTS = 64 * (DET_MAXD + DET_SLOTS);
__device__ __forceinline__ int* det_slot(int* hdr, int s) { return hdr + 64 * (DET_FOUND + s); }
__device__ __forceinline__ int det_bank_max(const int* __restrict__ hdr, int bank) {
  int m = 0;
#pragma unroll 8
  for (int k = 0; k < DET_SLOTS; ++k) m = max(m, hdr[64 * (bank + k)]);
  return m;
}
__device__ __forceinline__ int det_R(const int* __restrict__ hdr) { return det_bank_max(hdr, DET_RAD); }

// The fixed-point path runs unless a window served: mode A (R <= rmax), or mode B with all
// 4 n h w entries found.  rmax < 0: no window was launched.
__device__ __forceinline__ bool own_fallback(const int* __restrict__ hdr, int rmax,
                                             int64_t npix) {
  if (rmax < 0) return true;
  if (det_R(hdr) <= rmax) return false;
  int64_t s = 0;
#pragma unroll 8
  for (int k = 0; k < DET_SLOTS; ++k) s += hdr[64 * (1 + k)];
  return s != 4 * npix;
}

// 0. R = floor(max |flow| + 0.01) + 2 over the batch (INT_MAX for a component that is not
// finite or above DET_HUGE); the margin covers the rounding of (float)j + f near an integer
// for coordinates below 2^16 (the host checks h, w).  And the roughness V = the largest
// change of a flow component between horizontal / vertical neighbours (in 1/1024 px,
// bank DET_ROUGH): mode B is tried only on fields smooth enough for its source estimate.
constexpr float DET_HUGE = 1048576.f;
__global__ __launch_bounds__(256) void own_radius(const float* __restrict__ flow, int64_t npix,
                                                  int h, int w, int* __restrict__ hdr) {
  __shared__ int red[2][4];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int r = 0, v = 0;
  for (int64_t p = t0; p < npix; p += stride) {
    const float2 f = *reinterpret_cast<const float2*>(flow + 2 * p);
    const float ax = fabsf(f.x), ay = fabsf(f.y);
    const bool ok = ax <= DET_HUGE && ay <= DET_HUGE;       // false for NaN
    r = max(r, ok ? (int)(fmaxf(ax, ay) + 0.01f) + 2 : INT_MAX);
    const int j = (int)(p % w), i = (int)((p / w) % h);
    float dv = 0.f;
    if (j + 1 < w) {
      const float2 g = *reinterpret_cast<const float2*>(flow + 2 * (p + 1));
      dv = fmaxf(dv, fmaxf(fabsf(g.x - f.x), fabsf(g.y - f.y)));
    }
    if (i + 1 < h) {
      const float2 g = *reinterpret_cast<const float2*>(flow + 2 * (p + w));
      dv = fmaxf(dv, fmaxf(fabsf(g.x - f.x), fabsf(g.y - f.y)));
    }
    v = max(v, dv <= 1.0e6f ? (int)(dv * 1024.f) : INT_MAX);  // (NaN: INT_MAX)
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    r = max(r, __shfl_xor(r, o, 64));
    v = max(v, __shfl_xor(v, o, 64));
  }
  if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = r, red[1][threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int sl = blockIdx.x % DET_SLOTS;
    atomicMax(hdr + 64 * (DET_RAD + sl), max(max(red[0][0], red[0][1]), max(red[0][2], red[0][3])));
    atomicMax(hdr + 64 * (DET_ROUGH + sl), max(max(red[1][0], red[1][1]), max(red[1][2], red[1][3])));
  }
}

// VEC: rows of float4 quads (c % 4 == 0, 16-byte aligned); else one channel per lane.  Every
// add is an explicit fma, so no path's sums depend on how the compiler packs them.
template <bool VEC>
__device__ __forceinline__ void own_acc(float4& acc, float wr, const float* __restrict__ row,
                                        int k) {
  if (VEC) {
    const float4 g = *reinterpret_cast<const float4*>(row + 4 * k);
    acc.x = fmaf(wr, g.x, acc.x);
    acc.y = fmaf(wr, g.y, acc.y);
    acc.z = fmaf(wr, g.z, acc.z);
    acc.w = fmaf(wr, g.w, acc.w);
  } else {
    acc.x = fmaf(wr, row[k], acc.x);
  }
}

template <bool VEC>
__device__ __forceinline__ void own_store(float* __restrict__ row, int k, const float4& v) {
  if (VEC) *reinterpret_cast<float4*>(row + 4 * k) = v;
  else row[k] = v.x;
}

// The fixed-point fallback (absolute points, key 28 = 0, or a window that did not serve):
// every (pixel, corner) contribution w_k * dout[p] (fp32, as the windows form it) is scaled by
// 2^S and rounded to an int64, and the int64s are added -- integer adds commute, so the sums
// are exact and the same in any order: bitwise reproducible with atomics.  S = 61 - E - L for
// max |dout| <= 2^E and 4 n h w <= 2^L keeps every sum below 2^61 in magnitude; a
// contribution is exact to 2^-S = max|dout| 2^(L - 61) (2^-40 of it at 192 x 256 x 8).
//   fix_prep   : zeroes the accumulator, reduces max |dout| (float bits, atomicMax).
//   fix_scatter: 8 x 8 source tiles and 64 channels per workgroup step (grid-stride, two
//                workgroups per CU: a cheap launch when the window served), one wave per pixel
//                (lanes = channels); corners go through a 128-slot direct-mapped LDS cache of
//                destination rows (int64 LDS adds), a slot collision straight to global int64
//                atomics, and the cache leaves as one 512-B atomic wave-instruction per
//                destination: a tile's samples piled onto the border add once per destination.
//   fix_convert: dinp = acc * 2^-S (NaN everywhere if dout holds a non-finite value or a
//                contribution is not finite: a NaN flow -- the atomic form's NaN rows, louder).
constexpr int FX_T = 8, FX_SLOTS = 128, FX_WAVES = 8;

__global__ __launch_bounds__(256) void fix_prep(const float* __restrict__ dout, int64_t nel,
                                                int4* __restrict__ acc4, int64_t nacc4,
                                                int* __restrict__ hdr, int rmax, int64_t npix) {
  if (!own_fallback(hdr, rmax, npix)) return;
  __shared__ unsigned red[4];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  unsigned m = 0;
  for (int64_t e = t0; e < nel; e += stride)
    m = max(m, __float_as_uint(dout[e]) & 0x7fffffffu);   // NaN > inf > finite as bits
  for (int64_t k = t0; k < nacc4; k += stride) acc4[k] = make_int4(0, 0, 0, 0);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned*>(hdr + 64 * (DET_MAXD + blockIdx.x % DET_SLOTS)),
              max(max(red[0], red[1]), max(red[2], red[3])));
}

// S from max |dout| (0 when it is not finite: fix_convert writes NaN then)
__device__ __forceinline__ int fix_shift(const int* __restrict__ hdr, int lg4n) {
  const float m = __uint_as_float((unsigned)det_bank_max(hdr, DET_MAXD));
  if (!(m <= 3.0e38f)) return 0;
  int e = 0;
  frexpf(m, &e);                                       // m < 2^e
  return 61 - e - lg4n;
}

__global__ __launch_bounds__(64 * FX_WAVES) void fix_scatter(const float* __restrict__ dout,
                                                             const float* __restrict__ flow,
                                                             int n, int h, int w, int c,
                                                             int absolute,
                                                             int* __restrict__ hdr,
                                                             int rmax, int lg4n,
                                                             unsigned long long* __restrict__ acc) {
  const int64_t npix = (int64_t)n * h * w;
  if (!own_fallback(hdr, rmax, npix)) return;
  __shared__ unsigned long long data[FX_SLOTS * 64];
  __shared__ int tag[FX_SLOTS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_i = (h + FX_T - 1) / FX_T, tiles_j = (w + FX_T - 1) / FX_T;
  const int passes = (c + 63) / 64;
  const int S = fix_shift(hdr, lg4n);
  const int nwork = n * tiles_i * tiles_j * passes;
  for (int wk_id = blockIdx.x; wk_id < nwork; wk_id += gridDim.x) {   // (tile, channel pass)
    const int cc = (wk_id % passes) * 64;
    const int tile = wk_id / passes;
    const int b = tile / (tiles_i * tiles_j);
    const int rem = tile - b * tiles_i * tiles_j;
    const int i0 = (rem / tiles_j) * FX_T, j0 = (rem % tiles_j) * FX_T;
    const int64_t img = (int64_t)b * h * w;
    const int e = cc + lane;
    const bool eok = e < c;
    for (int k = tid; k < FX_SLOTS * 64; k += 64 * FX_WAVES) data[k] = 0ull;
    if (tid < FX_SLOTS) tag[tid] = -1;
    __syncthreads();
    for (int pr = wave; pr < FX_T * FX_T; pr += FX_WAVES) {
      const int i = i0 + pr / FX_T, j = j0 + pr % FX_T;
      if (i >= h || j >= w) continue;                  // wave-uniform
      const int64_t p = img + (int64_t)i * w + j;
      const float2 f = *reinterpret_cast<const float2*>(flow + 2 * p);
      const DetCorners t = det_corners(i, j, f.x, f.y, h, w, absolute != 0);
      const float g = eok ? dout[p * c + e] : 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float wk = ((k & 2) ? 1.f - t.a : t.a) * ((k & 1) ? 1.f - t.b : t.b);
        const float ct = wk * g;
        if (!(fabsf(ct) <= 3.0e38f))                   // a non-finite term (NaN / inf flow):
          atomicMax(hdr + 64 * DET_MAXD, 0x7fc00000);  // fix_convert writes NaN, loudly
        const unsigned long long v = (unsigned long long)llrint(ldexp((double)ct, S));
        const int d = t.y[k] * w + t.x[k];
        const int sl = ((t.y[k] & 7) << 4) | (t.x[k] & 15);
        int tg = 0;
        if (lane == 0) tg = atomicCAS(&tag[sl], -1, d);
        tg = __builtin_amdgcn_readfirstlane(tg);
        if (tg == -1 || tg == d)
          atomicAdd(&data[sl * 64 + lane], v);
        else if (eok)
          atomicAdd(acc + (img + d) * c + e, v);
      }
    }
    __syncthreads();
    for (int sl = wave; sl < FX_SLOTS; sl += FX_WAVES) {
      const int d = tag[sl];
      if (d >= 0 && eok) atomicAdd(acc + (img + d) * c + e, data[sl * 64 + lane]);
    }
    __syncthreads();                                   // (the cache is reset for the next tile)
  }
}

__global__ __launch_bounds__(256) void fix_convert(const long long* __restrict__ acc,
                                                   int64_t nel, const int* __restrict__ hdr,
                                                   int rmax, int64_t npix, int lg4n,
                                                   float* __restrict__ dinp) {
  if (!own_fallback(hdr, rmax, npix)) return;
  const float m = __uint_as_float((unsigned)det_bank_max(hdr, DET_MAXD));
  const bool fin = m <= 3.0e38f;
  const int S = fix_shift(hdr, lg4n);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nel; k += stride)
    dinp[k] = fin ? (float)ldexp((double)acc[k], -S) : __builtin_nanf("");
}

// 6. d(flow) (c % 4 == 0): 16 lanes per source pixel, lane q sums channel quads q, q + 16, ...
// in order, then a fixed DPP reduction over the row.  dflow_quad: one quad's terms, explicit
// fmas (the same arithmetic wherever it is inlined).
__device__ __forceinline__ float det_dot_diff(float4 g, float4 u, float4 v) {
  float s = g.x * (u.x - v.x);
  s = fmaf(g.y, u.y - v.y, s);
  s = fmaf(g.z, u.z - v.z, s);
  return fmaf(g.w, u.w - v.w, s);
}
__device__ __forceinline__ void dflow_quad(float& gx, float& gy, float a, float bq, float4 g,
                                           float4 P0, float4 P1, float4 P2, float4 P3) {
  gx -= fmaf(bq, det_dot_diff(g, P0, P2), (1.f - bq) * det_dot_diff(g, P1, P3));
  gy -= fmaf(a, det_dot_diff(g, P0, P1), (1.f - a) * det_dot_diff(g, P2, P3));
}
__device__ __forceinline__ void dflow_store(float gx, float gy, int64_t p, bool ok, int q,
                                            float* __restrict__ dflow,
                                            const float* __restrict__ dfa, int ldfa) {
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

// the four corner rows of pixel p's sample (offsets in floats) and its weights
struct DetTaps {
  int64_t off[4];
  float a, bq;
};
__device__ __forceinline__ DetTaps det_taps(const float* __restrict__ flow, int64_t pp, int h,
                                            int w, int c, int absolute) {
  const int j = (int)(pp % w);
  const int64_t t2 = pp / w;
  const int i = (int)(t2 % h);
  const int64_t img = (t2 / h) * h * w;
  const float2 f = *reinterpret_cast<const float2*>(flow + 2 * pp);
  const DetCorners t = det_corners(i, j, f.x, f.y, h, w, absolute != 0);
  DetTaps T;
#pragma unroll
  for (int k = 0; k < 4; ++k) T.off[k] = (img + (int64_t)t.y[k] * w + t.x[k]) * c;
  T.a = t.a;
  T.bq = t.b;
  return T;
}

// Every lane of the wave calls it (the row reduction reads all 16 lanes).
__device__ __forceinline__ void det_dflow_quads(const float* __restrict__ dout,
                                                const float* __restrict__ inp, int64_t npix,
                                                int h, int w, int c,
                                                const float* __restrict__ flow, int absolute,
                                                float* __restrict__ dflow,
                                                const float* __restrict__ dfa, int ldfa,
                                                int64_t p, int q) {
  const bool ok = p < npix;
  const int64_t pp = ok ? p : npix - 1;
  const DetTaps T = det_taps(flow, pp, h, w, c, absolute);
  float gx = 0.f, gy = 0.f;
  for (int cq = 4 * q; cq < c; cq += 64) {
    const float4 g = *reinterpret_cast<const float4*>(dout + pp * c + cq);
    const float4 P0 = *reinterpret_cast<const float4*>(inp + T.off[0] + cq);
    const float4 P1 = *reinterpret_cast<const float4*>(inp + T.off[1] + cq);
    const float4 P2 = *reinterpret_cast<const float4*>(inp + T.off[2] + cq);
    const float4 P3 = *reinterpret_cast<const float4*>(inp + T.off[3] + cq);
    dflow_quad(gx, gy, T.a, T.bq, g, P0, P1, P2, P3);
  }
  dflow_store(gx, gy, p, ok, q, dflow, dfa, ldfa);
}

__global__ __launch_bounds__(256) void det_dflow_vec(const float* __restrict__ dout,
                                                     const float* __restrict__ inp, int n, int h,
                                                     int w, int c, const float* __restrict__ flow,
                                                     int absolute, float* __restrict__ dflow,
                                                     const float* __restrict__ dfa, int ldfa) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  det_dflow_quads(dout, inp, (int64_t)n * h * w, h, w, c, flow, absolute, dflow, dfa, ldfa,
                  gid >> 4, (int)(gid & 15));
}

// The window gather.  win_accumulate sums a contiguous range of a destination's candidates,
// flattened i-major (ascending source index), over the group's 16 lanes: 4 x 16 candidates per
// batch with their flows loaded together; a candidate's corners landing on (r, x) are its hits,
// appended in (candidate, corner) order -- ascending code 4 p + k -- to
// the group's LDS list (row offset, weight) by a 16-lane prefix sum; the list is summed (flush)
// four rows in flight at a time, in list order, whenever it could overflow and at the end.
// NCB channel blocks of 16 quads (channels when !VEC) per lane; `found` += the hits.  Every
// lane of the wave calls it (wave-wide shuffles); a group with an empty range idles.
constexpr int WIN_CAP = 128;    // list entries per group; flushed above WIN_CAP - 64
constexpr int TILE_CAP = 64;    // sorted bin entries per destination of the tiled mode A
#ifndef WIN_DFLOW_PRE
#define WIN_DFLOW_PRE 0  // 1: own_window issues d(flow)'s loads before the window's (+28 VGPRs)
#endif
constexpr int WIN_PILE = 16;    // mode A: |w - h| above this, the pile row / column
constexpr int WIN_RB = 3;       // mode B window radius around the estimated source
constexpr int WIN_VMAX = 512;   // mode B only for V <= 0.5 px (or rmax == 1: always, tests)

struct WinDest {
  int r, x;                     // the destination
  int ilo, jlo, nj;             // its candidates: i = ilo + k / nj, j = jlo + k % nj
  int k0, k1;                   // the range this group sums
};

template <bool VEC, int NCB>
__device__ __forceinline__ void win_accumulate(float4 (&acc)[NCB], int& found, const WinDest& D,
                                               const float* __restrict__ dimg,
                                               const float* __restrict__ fimg, int h, int w,
                                               int c, int cb0, int* __restrict__ l_off,
                                               float* __restrict__ l_w, int q, int src0) {
  const int nq = VEC ? c >> 2 : c;
#pragma unroll
  for (int b = 0; b < NCB; ++b) acc[b] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int span = max(D.k1 - D.k0, 0);
  const bool interior = D.x >= 1 && D.x <= w - 2 && D.r >= 1 && D.r <= h - 2;
  int pmax = (span + 15) >> 4;
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) pmax = max(pmax, __shfl_xor(pmax, o, 64));
  int cnt = 0;                                         // the group's list length
  auto flush = [&]() {
    int em = cnt;
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) em = max(em, __shfl_xor(em, o, 64));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    for (int e0 = 0; e0 < em; e0 += 4) {
      float4 g[4][NCB];
      float wr[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = e0 + u < cnt;
        const int64_t o = ok ? (int64_t)l_off[e0 + u] * c : 0;
        wr[u] = ok ? l_w[e0 + u] : 0.f;
#pragma unroll
        for (int b = 0; b < NCB; ++b) {
          const int cq = cb0 + 16 * b + q;
          g[u][b] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (ok && cq < nq) {
            if (VEC) g[u][b] = *reinterpret_cast<const float4*>(dimg + o + 4 * cq);
            else g[u][b].x = dimg[o + cq];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (e0 + u < cnt) {
#pragma unroll
          for (int b = 0; b < NCB; ++b) {
            acc[b].x = fmaf(wr[u], g[u][b].x, acc[b].x);   // explicit: a packed
            if (VEC) {                                      // mul + add would round twice
              acc[b].y = fmaf(wr[u], g[u][b].y, acc[b].y);
              acc[b].z = fmaf(wr[u], g[u][b].z, acc[b].z);
              acc[b].w = fmaf(wr[u], g[u][b].w, acc[b].w);
            }
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    cnt = 0;
  };
  // this lane's candidate k = 16 t + q as (row di, column dj) of the window, stepped by 16
  // candidates per batch without a division (one per destination: 16 = s_i nj + s_j)
  const int nj = max(D.nj, 1);
  int di = (D.k0 + q) / nj, dj = (D.k0 + q) - di * nj;
  const int s_i = 16 / nj, s_j = 16 - s_i * nj;
  for (int t0 = 0; t0 < pmax; t0 += 4) {
    float2 f[4];
    int ci[4], cj[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = (t0 + u) * 16 + q;
      const bool in = k < span;
      ci[u] = in ? D.ilo + di : -1;
      cj[u] = D.jlo + dj;
      f[u] = make_float2(0.f, 0.f);
      if (in) f[u] = *reinterpret_cast<const float2*>(fimg + 2 * ((int64_t)ci[u] * w + cj[u]));
      di += s_i, dj += s_j;
      if (dj >= nj) dj -= nj, ++di;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (t0 + u >= pmax) break;
      uint32_t m = 0;
      float ca = 0.f, cbw = 0.f;
      // Interior destination: a candidate hits only if its sample lies in [x - 1, x + 1) x
      // [r - 1, r + 1) (its unclamped corners floor(.) and floor(.) + 1; a clamped corner lands
      // on the border), the same float sums det_corners forms: most lanes skip the corners.
      const bool maybe =
          !interior || ((float)ci[u] + f[u].x >= (float)(D.x - 1) && (float)ci[u] + f[u].x < (float)(D.x + 1) &&
                        (float)cj[u] + f[u].y >= (float)(D.r - 1) && (float)cj[u] + f[u].y < (float)(D.r + 1));
      if (ci[u] >= 0 && maybe) {
        const DetCorners tc = det_corners(ci[u], cj[u], f[u].x, f[u].y, h, w, false);
#pragma unroll
        for (int k = 0; k < 4; ++k) m |= (tc.y[k] == D.r && tc.x[k] == D.x) ? 1u << k : 0u;
        ca = tc.a;
        cbw = tc.b;
      }
      // most batches hit nothing anywhere in the wave: skip the list update (wave-uniform)
      if (__ballot(m != 0) == 0) continue;
      int cm = cnt;
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) cm = max(cm, __shfl_xor(cm, o, 64));
      if (cm > WIN_CAP - 64) flush();
      const int pc = __builtin_popcount(m);
      int incl = pc;                                   // inclusive prefix over the 16 lanes
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const int v = __shfl_up(incl, o, 16);
        if (q >= o) incl += v;
      }
      int pos = cnt + incl - pc;
      const int poff = ci[u] * w + cj[u];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (m & (1u << k)) {
          l_off[pos] = poff;
          l_w[pos] = ((k & 2) ? 1.f - ca : ca) * ((k & 1) ? 1.f - cbw : cbw);
          ++pos;
        }
      }
      const int tot = __shfl(incl, src0 + 15, 64);
      cnt += tot;
      found += tot;
    }
  }
  flush();
}

// Mode A: the candidates of destination (r, x) for radius R (sources within R of the
// transposed position; the last row / column to the far edge).
__device__ __forceinline__ WinDest win_dest_a(int r, int x, int h, int w, int R) {
  WinDest D;
  D.r = r, D.x = x;
  D.ilo = max(0, x - R);
  const int ihi = x == w - 1 ? h - 1 : min(h - 1, x + R);
  D.jlo = max(0, r - R);
  const int jhi = r == h - 1 ? w - 1 : min(w - 1, r + R);
  D.nj = jhi - D.jlo + 1;
  D.k0 = 0;
  D.k1 = ihi >= D.ilo && D.nj > 0 ? (ihi - D.ilo + 1) * D.nj : 0;
  return D;
}

// Mode B: a window of radius WIN_RB around the source estimated by three fixed-point steps
// i <- x - f0(i, j), j <- r - f1(i, j) from the transposed position; along a border the whole
// range a clipped sample can come from (F = R bounds |flow| + 2).
__device__ __forceinline__ WinDest win_dest_b(const float* __restrict__ fimg, int r, int x,
                                              int h, int w, int R) {
  const int F = min(R, 1 << 20);
  int i = min(x, h - 1), j = min(r, w - 1);
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    const float2 f = *reinterpret_cast<const float2*>(fimg + 2 * ((int64_t)i * w + j));
    i = (int)rintf(fminf(fmaxf((float)x - f.x, 0.f), (float)(h - 1)));   // NaN -> 0
    j = (int)rintf(fminf(fmaxf((float)r - f.y, 0.f), (float)(w - 1)));
  }
  WinDest D;
  D.r = r, D.x = x;
  int ilo, ihi, jlo, jhi;
  if (x == 0) ilo = 0, ihi = min(h - 1, F);
  else if (x == w - 1) ilo = max(0, w - 1 - F), ihi = h - 1;
  else ilo = max(0, i - WIN_RB), ihi = min(h - 1, i + WIN_RB);
  if (r == 0) jlo = 0, jhi = min(w - 1, F);
  else if (r == h - 1) jlo = max(0, h - 1 - F), jhi = w - 1;
  else jlo = max(0, j - WIN_RB), jhi = min(w - 1, j + WIN_RB);
  D.ilo = ilo;
  D.jlo = jlo;
  D.nj = jhi - jlo + 1;
  D.k0 = 0;
  D.k1 = ihi >= ilo && D.nj > 0 ? (ihi - ilo + 1) * D.nj : 0;
  return D;
}

// The pile workgroups' destinations per image: row 0 and row h - 1 (w each), then column 0
// and column w - 1 without the corners (h - 2 each); none for an image under 2 x 2.
__device__ __forceinline__ void win_pile_dest(int e, int h, int w, int& r, int& x) {
  if (e < w) r = 0, x = e;
  else if (e < 2 * w) r = h - 1, x = e - w;
  else if (e < 2 * w + h - 2) r = e - 2 * w + 1, x = 0;
  else r = e - (2 * w + h - 2) + 1, x = w - 1;
}

// Is (r, x) a pile destination (a workgroup of its own)?  Mode A: the last row when
// w - h > WIN_PILE, the last column when h - w > WIN_PILE.  Mode B: every border pixel.
__device__ __forceinline__ bool win_piled(bool mode_a, int r, int x, int h, int w) {
  if (h < 2 || w < 2) return false;
  if (mode_a)
    return (w - h > WIN_PILE && r == h - 1) || (h - w > WIN_PILE && x == w - 1);
  return r == 0 || r == h - 1 || x == 0 || x == w - 1;
}

// Mode A by 4 x 4 destination tiles in a kernel of its own (of_set_tuning key 34 = 2): the
// tiled path of own_window below without the scan's LDS list and registers, so more
// workgroups share a CU (the tiled gather is latency-bound: with own_window's 28.8 KB of LDS
// and 92 VGPRs five fit, and fewer measured slower in proportion -- gpurun_out/r6oc).  The
// destinations it cannot bin -- the last row and column of every image (clipped samples come
// from any distance; piles among them) and bins beyond TILE_CAP entries (appended to olist,
// count at hdr[0]) -- are left to own_window's rest pass (tiled = 2).  d(flow) of every
// pixel of the tile as a source (VEC).  Returns at once unless mode A.
#ifndef OWN_TILE_WPE
#define OWN_TILE_WPE 8    // waves per SIMD the registers are sized for (8: two per CU more)
#endif
template <bool VEC, int NCB>
__global__ __launch_bounds__(256, OWN_TILE_WPE) void own_tile(const float* __restrict__ dout,
                                                             const float* __restrict__ inp,
                                                             const float* __restrict__ flow,
                                                             int n, int h, int w, int c,
                                                             int* __restrict__ hdr, int rmax,
                                                             float* __restrict__ dinp,
                                                             float* __restrict__ dflow,
                                                             const float* __restrict__ dfa,
                                                             int ldfa, int* __restrict__ olist) {
  __shared__ int t_cnt[16];
  __shared__ int b_off[16][TILE_CAP];
  __shared__ float b_w[16][TILE_CAP];
  __shared__ int s_off[16][TILE_CAP];
  __shared__ float s_w[16][TILE_CAP];
  const int R = det_R(hdr);
  if (!(R <= rmax)) return;                                            // (grid-uniform)
  const int64_t npix = (int64_t)n * h * w;
  const int64_t hw = (int64_t)h * w;
  const int q = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int nq = VEC ? c >> 2 : c;
  const int tiles_x = (w + 3) >> 2, tiles_y = (h + 3) >> 2;
  const int64_t tb = blockIdx.x;
  if (tb >= (int64_t)n * tiles_x * tiles_y) return;                    // (block-uniform)
  const int img_i = (int)(tb / (tiles_x * tiles_y));
  const int trem = (int)(tb - (int64_t)img_i * tiles_x * tiles_y);
  const int r0 = (trem / tiles_x) * 4, x0 = (trem % tiles_x) * 4;
  const int64_t img = (int64_t)img_i * hw;
  const float* fimg = flow + 2 * img;
  const int r = r0 + (grp >> 2), x = x0 + (grp & 3);
  const bool dlive = r < h && x < w;
  const bool edge = x == w - 1 || r == h - 1;
  const int64_t pix = dlive ? img + (int64_t)r * w + x : npix - 1;
  if (threadIdx.x < 16) t_cnt[threadIdx.x] = 0;
  __syncthreads();
  const int ilo = max(0, x0 - R), ihi = min(h - 1, x0 + 3 + R);
  const int jlo = max(0, r0 - R), jhi = min(w - 1, r0 + 3 + R);
  const int nsj = jhi - jlo + 1;
  const int nsrc = ihi >= ilo && nsj > 0 ? (ihi - ilo + 1) * nsj : 0;
  for (int e = threadIdx.x; e < nsrc; e += 256) {
    const int i = ilo + e / nsj, j = jlo + e % nsj;
    const float2 f = *reinterpret_cast<const float2*>(fimg + 2 * ((int64_t)i * w + j));
    const DetCorners tc = det_corners(i, j, f.x, f.y, h, w, false);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int yr = tc.y[k] - r0, xr = tc.x[k] - x0;
      if ((unsigned)yr < 4u && (unsigned)xr < 4u) {
        const int g = yr * 4 + xr;
        if (r0 + yr == h - 1 || x0 + xr == w - 1) continue;   // edge / pile: the rest pass
        const int pos = atomicAdd(&t_cnt[g], 1);
        if (pos < TILE_CAP) {
          b_off[g][pos] = 4 * (i * w + j) + k;                  // the code
          b_w[g][pos] = ((k & 2) ? 1.f - tc.a : tc.a) * ((k & 1) ? 1.f - tc.b : tc.b);
        }
      }
    }
  }
  __syncthreads();
  const int ne = t_cnt[grp];
  if (dlive && !edge && ne > TILE_CAP) {
    if (q == 0) olist[atomicAdd(hdr, 1)] = (int)pix;    // any order: one list entry per dest.
  } else if (dlive && !edge) {
    for (int e = q; e < ne; e += 16) {                   // sort by code (ranks: distinct)
      const int ce = b_off[grp][e];
      int rank = 0;
      for (int f2 = 0; f2 < ne; ++f2) rank += b_off[grp][f2] < ce;
      s_off[grp][rank] = ce >> 2;
      s_w[grp][rank] = b_w[grp][e];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float* dimg = dout + img * c;
    for (int cb0 = 0; cb0 < nq; cb0 += 16 * NCB) {
      float4 acc[NCB];
#pragma unroll
      for (int b = 0; b < NCB; ++b) acc[b] = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int e0 = 0; e0 < ne; e0 += 4) {
        float4 g[4][NCB];
        float wr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool ok = e0 + u < ne;
          const int64_t o = ok ? (int64_t)s_off[grp][e0 + u] * c : 0;
          wr[u] = ok ? s_w[grp][e0 + u] : 0.f;
#pragma unroll
          for (int b = 0; b < NCB; ++b) {
            const int cq = cb0 + 16 * b + q;
            g[u][b] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (ok && cq < nq) {
              if (VEC) g[u][b] = *reinterpret_cast<const float4*>(dimg + o + 4 * cq);
              else g[u][b].x = dimg[o + cq];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (e0 + u < ne) {
#pragma unroll
            for (int b = 0; b < NCB; ++b) {
              acc[b].x = fmaf(wr[u], g[u][b].x, acc[b].x);   // explicit fmas: win_accumulate's
              if (VEC) {
                acc[b].y = fmaf(wr[u], g[u][b].y, acc[b].y);
                acc[b].z = fmaf(wr[u], g[u][b].z, acc[b].z);
                acc[b].w = fmaf(wr[u], g[u][b].w, acc[b].w);
              }
            }
          }
        }
      }
#pragma unroll
      for (int b = 0; b < NCB; ++b) {
        const int cq = cb0 + 16 * b + q;
        if (cq < nq) own_store<VEC>(dinp + pix * c, cq, acc[b]);
      }
    }
  }
  if (VEC)                   // d(flow) of this pixel as a source (every lane of the wave)
    det_dflow_quads(dout, inp, npix, h, w, c, flow, 0, dflow, dfa, ldfa, dlive ? pix : npix, q);
}

// The window kernel (launched when rmax >= 0).  Blocks [0, n * npb): one workgroup per pile
// destination (win_pile_dest; those that are not piles in this mode return), its 16 groups
// summing contiguous sixteenths of the candidate range, the partials added in group order --
// launched first, as they are the longest.  The other blocks: 16 lanes per destination, four
// per wave, piles skipped; with VEC (c <= 64 NCB) the group also forms d(flow) of pixel d as
// a source, its loads issued before the window's (DFQ quads per lane).  A window that does
// not serve (mode B, a count short of 4 n h w) is overwritten by the fixed-point path; with
// neither mode (R > rmax and V > WIN_VMAX) the kernel forms d(flow) only.
template <bool VEC, int NCB, bool TPRE = false>
__global__ __launch_bounds__(256) void own_window(const float* __restrict__ dout,
                                                  const float* __restrict__ inp,
                                                  const float* __restrict__ flow, int n, int h,
                                                  int w, int c, int* __restrict__ hdr,
                                                  int rmax, float* __restrict__ dinp,
                                                  float* __restrict__ dflow,
                                                  const float* __restrict__ dfa, int ldfa,
                                                  int tiled, const int* __restrict__ olist) {
  __shared__ int l_off[16][WIN_CAP];
  __shared__ float l_w[16][WIN_CAP];
  __shared__ float4 part[16][16 * NCB];
  __shared__ int fsum[16];
  __shared__ int t_cnt[16];
  __shared__ int s_off[16][TILE_CAP];
  __shared__ float s_w[16][TILE_CAP];
  const int64_t npix = (int64_t)n * h * w;
  const int64_t hw = (int64_t)h * w;
  const int lane = threadIdx.x & 63, q = lane & 15, src0 = lane & 48, grp = threadIdx.x >> 4;
  const int nq = VEC ? c >> 2 : c;
  const int R = det_R(hdr);
  const bool mode_a = R <= rmax;                       // uniform over the grid
  const bool mode_b = !mode_a && (det_bank_max(hdr, DET_ROUGH) <= WIN_VMAX || rmax == 1);
  const int npb = h >= 2 && w >= 2 ? 2 * w + 2 * (h - 2) : 0;
  const int npile = n * npb;
  int found = 0;
  if ((int)blockIdx.x < npile) {
    int r, x;
    const int img_i = blockIdx.x / npb;
    win_pile_dest(blockIdx.x % npb, h, w, r, x);
    if (!(mode_a || mode_b) || !win_piled(mode_a, r, x, h, w)) return;   // (block-uniform)
    const int64_t img = (int64_t)img_i * hw;
    WinDest D = mode_a ? win_dest_a(r, x, h, w, R) : win_dest_b(flow + 2 * img, r, x, h, w, R);
    const int seg = (D.k1 + 15) / 16;
    D.k0 = min(grp * seg, D.k1);
    D.k1 = min(D.k0 + seg, D.k1);
    for (int cb0 = 0; cb0 < nq; cb0 += 16 * NCB) {
      float4 acc[NCB];
      int fnd = 0;
      win_accumulate<VEC, NCB>(acc, fnd, D, dout + img * c, flow + 2 * img, h, w, c, cb0,
                               l_off[grp], l_w[grp], q, src0);
      if (cb0 == 0) found = fnd;
#pragma unroll
      for (int b = 0; b < NCB; ++b) part[grp][16 * b + q] = acc[b];
      __syncthreads();
      if (grp == 0) {
#pragma unroll
        for (int b = 0; b < NCB; ++b) {
          float4 t = part[0][16 * b + q];
          for (int g2 = 1; g2 < 16; ++g2) {
            const float4 v = part[g2][16 * b + q];
            t.x += v.x, t.y += v.y, t.z += v.z, t.w += v.w;
          }
          const int cq = cb0 + 16 * b + q;
          if (cq < nq) own_store<VEC>(dinp + (img + (int64_t)r * w + x) * c, cq, t);
        }
      }
      __syncthreads();
    }
    if (mode_b) {
      if (q == 0) fsum[grp] = found;
      __syncthreads();
      if (threadIdx.x == 0) {
        int s = 0;
        for (int g2 = 0; g2 < 16; ++g2) s += fsum[g2];
        atomicAdd(det_slot(hdr, blockIdx.x % DET_SLOTS), s);
      }
    }
    return;
  }
  if (tiled == 2 && mode_a) {
    // ---- the rest of own_tile's mode A (of_set_tuning key 34 = 2): the scan for the last row
    // and column of every image (piles excepted: the blocks above) and for the destinations
    // whose bins overflowed (olist, hdr[0] of them), 16 a block, grid-stride; own_tile formed
    // d(flow)
    const int per = w + h - 1;
    const int64_t nedge = (int64_t)n * per;
    const int64_t total = nedge + hdr[0];
    const int64_t nb = (int64_t)gridDim.x - npile;
    for (int64_t e0 = ((int64_t)blockIdx.x - npile) * 16; e0 < total; e0 += nb * 16) {
      const int64_t e = e0 + grp;
      const bool live = e < total;
      int64_t pix = 0;
      if (e < nedge) {
        const int k = (int)(e % per);
        pix = (e / per) * hw + (k < w ? (int64_t)(h - 1) * w + k : (int64_t)(k - w) * w + (w - 1));
      } else if (live) {
        pix = olist[e - nedge];
      }
      const int64_t img = (pix / hw) * hw;
      const int r = (int)((pix - img) / w), x = (int)((pix - img) % w);
      const bool go = live && !win_piled(true, r, x, h, w);
      WinDest D = win_dest_a(r, x, h, w, R);
      if (!go) D.k1 = 0;
      for (int cb0 = 0; cb0 < nq; cb0 += 16 * NCB) {
        float4 acc[NCB];
        int fnd = 0;
        win_accumulate<VEC, NCB>(acc, fnd, D, dout + img * c, flow + 2 * img, h, w, c, cb0,
                                 l_off[grp], l_w[grp], q, src0);
        if (go) {
#pragma unroll
          for (int b = 0; b < NCB; ++b) {
            const int cq = cb0 + 16 * b + q;
            if (cq < nq) own_store<VEC>(dinp + pix * c, cq, acc[b]);
          }
        }
      }
    }
    return;
  }
  if (tiled == 1 && mode_a) {
    // ---- mode A by destination tiles (of_set_tuning key 34): the block's 16 groups are the
    // 4 x 4 destinations (r0 + g / 4, x0 + g % 4).  Every source of the tile's window -- the
    // union of its destinations' mode-A windows -- is visited ONCE: its corners that land on a
    // destination of the tile go into that destination's LDS bin (position by an LDS atomic:
    // any order), each bin is then sorted by code 4 p + k, and summed in that order -- the
    // order of win_accumulate's list, so the sums are bitwise those of the scan (which reads
    // (2R + 1)^2 candidates per destination instead).  Destinations whose mode-A window is
    // not inside the tile's (the far edge: x = w - 1 or r = h - 1, where clipped samples come
    // from any distance) and bins beyond TILE_CAP entries take the scan; piles are the pile
    // blocks' (above).
    const int tiles_x = (w + 3) >> 2, tiles_y = (h + 3) >> 2;
    const int64_t tb = (int64_t)blockIdx.x - npile;
    if (tb >= (int64_t)n * tiles_x * tiles_y) return;                  // (block-uniform)
    const int img_i = (int)(tb / (tiles_x * tiles_y));
    const int trem = (int)(tb - (int64_t)img_i * tiles_x * tiles_y);
    const int r0 = (trem / tiles_x) * 4, x0 = (trem % tiles_x) * 4;
    const int64_t img = (int64_t)img_i * hw;
    const float* fimg = flow + 2 * img;
    const int r = r0 + (grp >> 2), x = x0 + (grp & 3);
    const bool dlive = r < h && x < w;
    const bool piled = dlive && win_piled(true, r, x, h, w);
    const bool edge = x == w - 1 || r == h - 1;
    const int64_t pix = dlive ? img + (int64_t)r * w + x : npix - 1;
    // TPRE (of_set_tuning key 35): d(flow)'s loads of this pixel issued now, consumed at the
    // end -- in flight across the binning and the gather
    constexpr bool kPre = VEC && TPRE;
    float4 pg[kPre ? NCB : 1], pP[4][kPre ? NCB : 1];
    DetTaps T{};
    const bool pre = kPre && c <= 64 * NCB;
    if (kPre && pre) {
      T = det_taps(flow, pix, h, w, c, 0);
#pragma unroll
      for (int b = 0; b < (kPre ? NCB : 1); ++b) {
        const int cq = 4 * q + 64 * b;
        const bool ok = cq < c;
        pg[b] = ok ? *reinterpret_cast<const float4*>(dout + pix * c + cq) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          pP[k][b] = ok ? *reinterpret_cast<const float4*>(inp + T.off[k] + cq)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if (threadIdx.x < 16) t_cnt[threadIdx.x] = 0;
    __syncthreads();
    // the sources: i in [x0 - R, x0 + 3 + R], j in [r0 - R, r0 + 3 + R] (clipped)
    const int ilo = max(0, x0 - R), ihi = min(h - 1, x0 + 3 + R);
    const int jlo = max(0, r0 - R), jhi = min(w - 1, r0 + 3 + R);
    const int nsj = jhi - jlo + 1;
    const int nsrc = ihi >= ilo && nsj > 0 ? (ihi - ilo + 1) * nsj : 0;
    for (int e = threadIdx.x; e < nsrc; e += 256) {
      const int i = ilo + e / nsj, j = jlo + e % nsj;
      const float2 f = *reinterpret_cast<const float2*>(fimg + 2 * ((int64_t)i * w + j));
      const DetCorners tc = det_corners(i, j, f.x, f.y, h, w, false);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int yr = tc.y[k] - r0, xr = tc.x[k] - x0;
        if ((unsigned)yr < 4u && (unsigned)xr < 4u) {
          const int g = yr * 4 + xr;
          const int rr = r0 + yr, xx = x0 + xr;
          if (rr == h - 1 || xx == w - 1) continue;       // edge / pile: not binned
          const int pos = atomicAdd(&t_cnt[g], 1);
          if (pos < WIN_CAP) {
            l_off[g][pos] = 4 * (i * w + j) + k;          // the code (< 2^31: 4 n h w checked)
            l_w[g][pos] = ((k & 2) ? 1.f - tc.a : tc.a) * ((k & 1) ? 1.f - tc.b : tc.b);
          }
        }
      }
    }
    __syncthreads();
    const int ne = t_cnt[grp];
    const bool scan = dlive && !piled && (edge || ne > TILE_CAP);
    // the scan fallback (wave-wide shuffles inside: all four groups of the wave call it when
    // any of them needs it, the others with an empty range)
    if (__ballot(scan && q == 0) != 0) {
      WinDest D = win_dest_a(dlive ? r : 0, dlive ? x : 0, h, w, R);
      if (!scan) D.k1 = 0;
      for (int cb0 = 0; cb0 < nq; cb0 += 16 * NCB) {
        float4 acc[NCB];
        int fnd = 0;
        win_accumulate<VEC, NCB>(acc, fnd, D, dout + img * c, fimg, h, w, c, cb0,
                                 l_off[grp], l_w[grp], q, src0);
        if (scan) {
#pragma unroll
          for (int b = 0; b < NCB; ++b) {
            const int cq = cb0 + 16 * b + q;
            if (cq < nq) own_store<VEC>(dinp + (img + (int64_t)r * w + x) * c, cq, acc[b]);
          }
        }
      }
    }
    if (dlive && !piled && !scan) {
      // sort the bin by code (ranks: codes are distinct), then sum in that order
      for (int e = q; e < ne; e += 16) {
        const int ce = l_off[grp][e];
        int rank = 0;
        for (int f2 = 0; f2 < ne; ++f2) rank += l_off[grp][f2] < ce;
        s_off[grp][rank] = ce >> 2;
        s_w[grp][rank] = l_w[grp][e];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const float* dimg = dout + img * c;
      for (int cb0 = 0; cb0 < nq; cb0 += 16 * NCB) {
        float4 acc[NCB];
#pragma unroll
        for (int b = 0; b < NCB; ++b) acc[b] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int e0 = 0; e0 < ne; e0 += 4) {
          float4 g[4][NCB];
          float wr[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool ok = e0 + u < ne;
            const int64_t o = ok ? (int64_t)s_off[grp][e0 + u] * c : 0;
            wr[u] = ok ? s_w[grp][e0 + u] : 0.f;
#pragma unroll
            for (int b = 0; b < NCB; ++b) {
              const int cq = cb0 + 16 * b + q;
              g[u][b] = make_float4(0.f, 0.f, 0.f, 0.f);
              if (ok && cq < nq) {
                if (VEC) g[u][b] = *reinterpret_cast<const float4*>(dimg + o + 4 * cq);
                else g[u][b].x = dimg[o + cq];
              }
            }
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (e0 + u < ne) {
#pragma unroll
              for (int b = 0; b < NCB; ++b) {
                acc[b].x = fmaf(wr[u], g[u][b].x, acc[b].x);
                if (VEC) {
                  acc[b].y = fmaf(wr[u], g[u][b].y, acc[b].y);
                  acc[b].z = fmaf(wr[u], g[u][b].z, acc[b].z);
                  acc[b].w = fmaf(wr[u], g[u][b].w, acc[b].w);
                }
              }
            }
          }
        }
#pragma unroll
        for (int b = 0; b < NCB; ++b) {
          const int cq = cb0 + 16 * b + q;
          if (cq < nq) own_store<VEC>(dinp + (img + (int64_t)r * w + x) * c, cq, acc[b]);
        }
      }
    }
    if (kPre && pre) {         // the same quads in the same order as det_dflow_quads
      float gx = 0.f, gy = 0.f;
#pragma unroll
      for (int b = 0; b < (kPre ? NCB : 1); ++b)
        if (4 * q + 64 * b < c) dflow_quad(gx, gy, T.a, T.bq, pg[b], pP[0][b], pP[1][b], pP[2][b], pP[3][b]);
      dflow_store(gx, gy, dlive ? pix : npix, dlive, q, dflow, dfa, ldfa);
    } else if (VEC) {          // d(flow) of this pixel as a source (every lane of the wave)
      det_dflow_quads(dout, inp, npix, h, w, c, flow, 0, dflow, dfa, ldfa,
                      dlive ? img + (int64_t)r * w + x : npix, q);
    }
    return;
  }
  // (a grid sized for the tiles may have more blocks than the scan's 16 destinations each)
  if ((int64_t)blockIdx.x - npile >= (npix + 15) / 16) return;        // (block-uniform)
  const int64_t d = ((blockIdx.x - npile) * (int64_t)blockDim.x + threadIdx.x) >> 4;
  const bool live = d < npix;
  const int64_t dd = live ? d : npix - 1;
#if WIN_DFLOW_PRE
  // d(flow) of pixel d: its loads first (c <= 64 NCB, one quad per channel block)
  constexpr int DFQ = NCB;
  const bool pre = VEC && c <= 64 * DFQ;
  float4 pg[DFQ], pP[4][DFQ];
  DetTaps T;
  if (pre) {
    T = det_taps(flow, dd, h, w, c, 0);
#pragma unroll
    for (int b = 0; b < DFQ; ++b) {
      const int cq = 4 * q + 64 * b;
      const bool ok = cq < c;
      pg[b] = ok ? *reinterpret_cast<const float4*>(dout + dd * c + cq) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        pP[k][b] = ok ? *reinterpret_cast<const float4*>(inp + T.off[k] + cq)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
#else
  constexpr bool pre = false;
#endif
  if (mode_a || mode_b) {
    const int64_t img = dd / hw * hw;
    const int rem = (int)(dd - img);
    const int r = rem / w, x = rem % w;
    const bool skip = !live || win_piled(mode_a, r, x, h, w);
    WinDest D = mode_a ? win_dest_a(r, x, h, w, R) : win_dest_b(flow + 2 * img, r, x, h, w, R);
    if (skip) D.k1 = 0;
    for (int cb0 = 0; cb0 < nq; cb0 += 16 * NCB) {     // every lane runs every iteration
      float4 acc[NCB];
      int fnd = 0;
      win_accumulate<VEC, NCB>(acc, fnd, D, dout + img * c, flow + 2 * img, h, w, c, cb0,
                               l_off[grp], l_w[grp], q, src0);
      if (cb0 == 0) found = fnd;
      if (!skip) {
#pragma unroll
        for (int b = 0; b < NCB; ++b) {
          const int cq = cb0 + 16 * b + q;
          if (cq < nq) own_store<VEC>(dinp + dd * c, cq, acc[b]);
        }
      }
    }
  }
  if (mode_b) {                                        // the wave's hits, one add
    int s = q == 0 ? found : 0;
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0 && s) atomicAdd(det_slot(hdr, (blockIdx.x * 4 + (threadIdx.x >> 6)) % DET_SLOTS), s);
  }
#if WIN_DFLOW_PRE
  if (pre) {
    float gx = 0.f, gy = 0.f;
#pragma unroll
    for (int b = 0; b < DFQ; ++b)
      if (4 * q + 64 * b < c) dflow_quad(gx, gy, T.a, T.bq, pg[b], pP[0][b], pP[1][b], pP[2][b], pP[3][b]);
    dflow_store(gx, gy, d, live, q, dflow, dfa, ldfa);
  } else
#endif
  if (VEC) {
    det_dflow_quads(dout, inp, npix, h, w, c, flow, 0, dflow, dfa, ldfa, d, q);
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


// Workspace layout: the int64 accumulator of the fixed-point path (n h w c), then the header.
struct DetWs {
  size_t acc, hdr, total;
};

void det_layout(int64_t npix, int c, DetWs& L) {
  L.acc = 0;
  L.hdr = (size_t)npix * c * 8;
  L.hdr = (L.hdr + 255) / 256 * 256;
  L.total = L.hdr + DET_HDR_INTS * 4;
}

}  // namespace

int g_det_rmax = 8;
int g_det_tile = 2;   // of_set_tuning key 34: 2 own_tile + rest pass, 1 tiles inside own_window, 0 scan
int g_det_tpre = 0;
// of_set_tuning key 37: workgroups per CU of the fixed-point fallback's grid-stride kernels
// (0: 8 for fix_prep / fix_convert, 2 for fix_scatter).  They run whenever the window may not
// have served and return at once when it did, so their grids cost launch time every call.
int g_det_fx_grid = 0;
// of_set_tuning key 38: extra dynamic LDS bytes per own_window workgroup (an occupancy probe:
// fewer resident workgroups per CU; 0 = default)
int g_det_lds_probe = 0;

extern "C" {

size_t of_warp_bwd_det_workspace(int n, int h, int w, int c) {
  if (n <= 0 || h <= 0 || w <= 0 || c <= 0) return 0;
  DetWs L;
  det_layout((int64_t)n * h * w, c, L);
  return L.total;
}

size_t of_warp_bwd_det_header(int n, int h, int w, int c) {
  if (n <= 0 || h <= 0 || w <= 0 || c <= 0) return 0;
  DetWs L;
  det_layout((int64_t)n * h * w, c, L);
  return L.hdr;
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
  const dim3 gq((unsigned)cdiv(npix * 16, 256));
  const dim3 gp((unsigned)cdiv(npix, 256));
  if (!dinp) {
    if (vec)
      hipLaunchKernelGGL(det_dflow_vec, gq, dim3(256), 0, s, dout, inp, n, h, w, c, flow,
                         absolute, dflow, dflow_add, ld_add);
    else
      hipLaunchKernelGGL(det_dflow_scalar, gp, dim3(256), 0, s, dout, inp, n, h, w, c, flow,
                         absolute, dflow, dflow_add, ld_add);
    return check_launch("warp_bwd_det: dflow");
  }
  DetWs L;
  det_layout(npix, c, L);
  OF_CHECK_ARG(ws && ws_bytes >= L.total, "warp bwd det: workspace too small");
  char* base = static_cast<char*>(ws);
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(base + L.acc);
  int* hdr = reinterpret_cast<int*>(base + L.hdr);
  // the window needs relative flows and coordinates below 2^16 (own_radius's margin)
  const int rmax = absolute || h >= 65536 || w >= 65536 || g_det_rmax == 0 ? -1 : g_det_rmax;
  if (hipMemsetAsync(hdr, 0, DET_HDR_INTS * 4, s) != hipSuccess)
    return check_launch("warp_bwd_det: memset");
  if (rmax >= 0) {
    // R, then the window and d(flow); the fallback's kernels after it read its mode-B count
    const unsigned gr = (unsigned)std::min<int64_t>(cdiv(npix, 256), 4 * device_cus());
    hipLaunchKernelGGL(own_radius, dim3(gr), dim3(256), 0, s, flow, npix, h, w, hdr);
    const int nq = vec ? c / 4 : c;
    auto kw = vec ? (g_det_tpre ? (nq > 16 ? own_window<true, 2, true> : own_window<true, 1, true>)
                                : (nq > 16 ? own_window<true, 2> : own_window<true, 1>))
                  : (nq > 16 ? own_window<false, 2> : own_window<false, 1>);
    const int64_t npile = h >= 2 && w >= 2 ? (int64_t)n * (2 * w + 2 * (h - 2)) : 0;
    const int64_t ntile = g_det_tile ? (int64_t)n * ((h + 3) / 4) * ((w + 3) / 4) : 0;
    // key 34 = 2: own_tile first (mode A's interior destinations), the rest in own_window; the
    // overflow list lives in the fixed-point accumulator's space (unused in mode A)
    int* olist = reinterpret_cast<int*>(base + L.acc);
    if (g_det_tile == 2) {
      auto kt = vec ? (nq > 16 ? own_tile<true, 2> : own_tile<true, 1>)
                    : (nq > 16 ? own_tile<false, 2> : own_tile<false, 1>);
      hipLaunchKernelGGL(kt, dim3((unsigned)ntile), dim3(256), 0, s, dout, inp, flow, n, h, w, c,
                         hdr, rmax, dinp, dflow, dflow_add, ld_add, olist);
      if (int st = check_launch("warp_bwd_det: tiles")) return st;
    }
    const int64_t gw = std::max<int64_t>(gq.x, g_det_tile == 1 ? ntile : 0);
    hipLaunchKernelGGL(kw, dim3((unsigned)(gw + npile)), dim3(256), g_det_lds_probe, s, dout, inp, flow, n,
                       h, w, c, hdr, rmax, dinp, dflow, dflow_add, ld_add, g_det_tile, olist);
    if (int st = check_launch("warp_bwd_det: window")) return st;
  }
  // the fixed-point fallback (each kernel returns at once when the window served)
  int lg4n = 0;
  while ((int64_t(1) << lg4n) < 4 * npix) ++lg4n;
  const int64_t nel = npix * c;
  const int fxg = g_det_fx_grid > 0 ? g_det_fx_grid : 8;
  const unsigned gs = (unsigned)std::min<int64_t>(cdiv(nel, 256), fxg * device_cus());
  hipLaunchKernelGGL(fix_prep, dim3(gs), dim3(256), 0, s, dout, nel,
                     reinterpret_cast<int4*>(acc), (nel + 1) / 2, hdr, rmax, npix);
  const int64_t tiles = (int64_t)n * cdiv(h, FX_T) * cdiv(w, FX_T) * ((c + 63) / 64);
  const unsigned gfx = (unsigned)std::min<int64_t>(tiles, std::min(fxg, 2) * device_cus());   // (grid-stride)
  hipLaunchKernelGGL(fix_scatter, dim3(gfx), dim3(64 * FX_WAVES), 0, s, dout, flow,
                     n, h, w, c, absolute, hdr, rmax, lg4n, acc);
  hipLaunchKernelGGL(fix_convert, dim3(gs), dim3(256), 0, s,
                     reinterpret_cast<const long long*>(acc), nel, hdr, rmax, npix, lg4n, dinp);
  if (int st = check_launch("warp_bwd_det: fixed point")) return st;
  if (rmax >= 0 && vec) return OF_OK;                  // d(flow) formed by own_window
  if (vec)
    hipLaunchKernelGGL(det_dflow_vec, gq, dim3(256), 0, s, dout, inp, n, h, w, c, flow, absolute,
                       dflow, dflow_add, ld_add);
  else
    hipLaunchKernelGGL(det_dflow_scalar, gp, dim3(256), 0, s, dout, inp, n, h, w, c, flow,
                       absolute, dflow, dflow_add, ld_add);
  return check_launch("warp_bwd_det: dflow");
}

}  // extern "C"

}  // namespace oflow
