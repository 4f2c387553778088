// Deterministic feature-warp backward ("a deterministic-mode flag (no atomics in
// the warp bwd)"), the default since round 5 (ops.DETERMINISTIC).
//
// The reference samples with four gather_nd taps (transformations.py:98-129, reached from
// warp_features, model.py:55-73); TF's gradient of a gather is a scatter-add into the feature
// map, whose adds land in whatever order the hardware retires them.  The atomic HIP backward
// (flow_ops.hip warp_bwd_gather) keeps that shape: per-tile sums added with float atomics, so
// two identical steps can differ in the last bit of d(features).  Here the scatter becomes a
// gather with a fixed summation order, all hand-written (a counting sort by destination):
//
//   1. count   : every (source pixel p, corner k) adds 1 to its destination's counter
//                (integer adds: exact in any order);
//   2. scan    : exclusive prefix sums of the counts -> each destination's segment;
//   3. fill    : each entry's code 4 p + k into a slot of its segment (slot order free);
//   4. gather  : per destination, the segment's codes ranked (16 lanes, codes distinct) and
//                w_k * dout[p] summed in ascending code order, STORED -- every row written
//                once, so no zero-fill pass and no float atomics;
//   5. big     : segments of more than 16 entries (a field clipped onto the border) through an
//                LDS bitmap over the code range, visited in code order;
//   6. d(flow) : per source pixel over all channels in a fixed order (16 lanes x channel quads,
//                then a fixed DPP row reduction), plus the optional addend of of_warp_bwd_add.
//
// Bitwise reproducible run to run, in eager mode and inside a captured graph alike.  HBM / L2
// bound: 8 B of flow and 12 B of counters per (pixel, corner) through steps 1-3, the gather
// reads each destination's source rows (mostly L2 hits for smooth flows) and writes d(features)
// once; O(n h w) for any flow field.
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

// 1. count: one thread per source pixel, one integer add per (pixel, corner) on its
// destination's counter (integer adds commute: the counts are exact whatever the order).
__global__ __launch_bounds__(256) void own_count(const float* __restrict__ flow, int n, int h,
                                                 int w, int absolute, int* __restrict__ cnt) {
  const int64_t npix = (int64_t)n * h * w;
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int j = (int)(p % w);
  const int64_t t2 = p / w;
  const int i = (int)(t2 % h);
  const int64_t img = (t2 / h) * h * w;
  const float2 f = *reinterpret_cast<const float2*>(flow + 2 * p);
  const DetCorners t = det_corners(i, j, f.x, f.y, h, w, absolute != 0);
#pragma unroll
  for (int k = 0; k < 4; ++k) atomicAdd(cnt + img + (int64_t)t.y[k] * w + t.x[k], 1);
}

// 2. exclusive scan of the counts (three launches: per-block sums, the block sums in one
// workgroup, per-block scan + block offset).  OWN_SB elements per block.
constexpr int OWN_SB = 2048;
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__global__ __launch_bounds__(256) void own_block_sums(const int* __restrict__ cnt, int64_t total,
                                                      int* __restrict__ bsum) {
  __shared__ int red[4];
  const int64_t base = blockIdx.x * (int64_t)OWN_SB;
  int s = 0;
  for (int k = threadIdx.x; k < OWN_SB; k += 256) {
    const int64_t e = base + k;
    s += e < total ? cnt[e] : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// one workgroup: bsum -> exclusive offsets, in place (nb block sums, any count)
__global__ __launch_bounds__(1024) void own_scan_sums(int* __restrict__ bsum, int nb) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int b0 = 0; b0 < nb; b0 += 1024) {
    const int v = b0 + tid < nb ? bsum[b0 + tid] : 0;
    const int inc = wave_incl_scan(v, lane);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    int before = carry;
    for (int k = 0; k < wv; ++k) before += wsum[k];
    if (b0 + tid < nb) bsum[b0 + tid] = before + inc - v;
    __syncthreads();
    if (tid == 1023) carry = before + inc;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void own_block_scan(const int* __restrict__ cnt, int64_t total,
                                                      const int* __restrict__ boff,
                                                      int* __restrict__ off) {
  __shared__ int wsum[4];
  __shared__ int carry;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t base = blockIdx.x * (int64_t)OWN_SB;
  if (tid == 0) carry = boff[blockIdx.x];
  __syncthreads();
  for (int k0 = 0; k0 < OWN_SB; k0 += 256) {
    const int64_t e = base + k0 + tid;
    const int v = e < total ? cnt[e] : 0;
    const int inc = wave_incl_scan(v, lane);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    int before = carry;
    for (int k = 0; k < wv; ++k) before += wsum[k];
    if (e < total) off[e] = before + inc - v;
    __syncthreads();
    if (tid == 255) carry = before + inc;
    __syncthreads();
  }
}

// 3. fill: each (pixel, corner) entry goes to a slot of its destination's segment.  The slot
// order inside a segment depends on the order of the integer adds; the gather below orders
// every segment itself, so nothing downstream depends on it.  Entry code = 4 p + k (p the
// pixel within its image, k the corner: bit 0 -> row y1, bit 1 -> column x1).
__global__ __launch_bounds__(256) void own_fill(const float* __restrict__ flow, int n, int h,
                                                int w, int absolute, const int* __restrict__ off,
                                                int* __restrict__ cursor,
                                                uint32_t* __restrict__ list) {
  const int64_t npix = (int64_t)n * h * w;
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int j = (int)(p % w);
  const int64_t t2 = p / w;
  const int i = (int)(t2 % h);
  const int64_t img = (t2 / h) * h * w;
  const float2 f = *reinterpret_cast<const float2*>(flow + 2 * p);
  const DetCorners t = det_corners(i, j, f.x, f.y, h, w, absolute != 0);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t d = img + (int64_t)t.y[k] * w + t.x[k];
    list[off[d] + atomicAdd(cursor + d, 1)] = (uint32_t)(4 * (p - img) + k);
  }
}

// the weight of entry `code` of image `img` (the forward's bilinear weights, P2)
__device__ __forceinline__ float own_weight(const float* __restrict__ flow, int64_t img, int h,
                                            int w, int absolute, uint32_t code) {
  const int64_t pi = code >> 2;
  const int k = code & 3;
  const float2 f = *reinterpret_cast<const float2*>(flow + 2 * (img + pi));
  const DetCorners t = det_corners((int)(pi / w), (int)(pi % w), f.x, f.y, h, w, absolute != 0);
  return ((k & 2) ? 1.f - t.a : t.a) * ((k & 1) ? 1.f - t.b : t.b);
}

// 4. gather, destinations with at most 16 entries: 16 lanes per destination (channel quads),
// four destinations per wave.  Lane j < n holds entry j; its rank (the number of smaller codes
// in the segment) orders the sum: sum over codes ascending of w * dout[p] -- the same order
// whatever slots the fill gave them.  A segment of more than 16 entries is listed for step 5.
// Every destination row is written (0 when no entry lands on it): no zero-fill pass.
constexpr int OWN_SMALL = 16;
// VEC: rows of float4 quads (c % 4 == 0, 16-byte aligned); else one channel per lane.
template <bool VEC>
__device__ __forceinline__ void own_acc(float4& acc, float wr, const float* __restrict__ row,
                                        int k) {
  if (VEC) {
    const float4 g = *reinterpret_cast<const float4*>(row + 4 * k);
    acc.x += wr * g.x;
    acc.y += wr * g.y;
    acc.z += wr * g.z;
    acc.w += wr * g.w;
  } else {
    acc.x += wr * row[k];
  }
}

template <bool VEC>
__device__ __forceinline__ void own_store(float* __restrict__ row, int k, const float4& v) {
  if (VEC) *reinterpret_cast<float4*>(row + 4 * k) = v;
  else row[k] = v.x;
}

template <bool VEC>
__global__ __launch_bounds__(256) void own_gather(const float* __restrict__ dout,
                                                  const float* __restrict__ flow, int n, int h,
                                                  int w, int c, int absolute,
                                                  const int* __restrict__ cnt,
                                                  const int* __restrict__ off,
                                                  const uint32_t* __restrict__ list,
                                                  float* __restrict__ dinp,
                                                  int* __restrict__ big_n, int* __restrict__ big) {
  const int64_t npix = (int64_t)n * h * w;
  const int lane = threadIdx.x & 63, g16 = lane >> 4, q = lane & 15;
  const int64_t d = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 4;
  const bool live = d < npix;
  const int64_t dd = live ? d : npix - 1;
  const int ne = live ? cnt[dd] : 0;
  const int64_t img = dd / ((int64_t)h * w) * h * w;
  const bool small = ne <= OWN_SMALL;
  if (live && !small && q == 0) big[atomicAdd(big_n, 1)] = (int)dd;
  const uint32_t code = small && q < ne ? list[off[dd] + q] : 0xffffffffu;
  // rank among the segment's codes (codes are distinct)
  int rank = 0;
  const int src0 = lane & 48;
#pragma unroll
  for (int k = 0; k < OWN_SMALL; ++k) {
    const uint32_t o = (uint32_t)__shfl((int)code, src0 + k, 64);
    rank += o < code ? 1 : 0;
  }
  const float wt = small && q < ne ? own_weight(flow, img, h, w, absolute, code) : 0.f;
  // max entries over the four destinations of the wave: the loop bound
  int nmax = small ? ne : 0;
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) nmax = max(nmax, __shfl_xor(nmax, o, 64));
  const int nq = VEC ? c >> 2 : c;                     // quads, or channels
  for (int cb = 0; cb < nq; cb += 16) {                // every lane runs every iteration
    const int cq = cb + q;
    const bool cok = cq < nq;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < nmax; ++r) {
      // the lane of this group holding rank r (none when this group's segment is shorter)
      const uint64_t bal = __ballot(small && q < ne && rank == r);
      const int sl = (int)((bal >> (16 * g16)) & 0xffffull);
      const bool has = sl != 0;
      const int src = src0 + (has ? __builtin_ctz(sl) : 0);
      const uint32_t cd = (uint32_t)__shfl((int)code, src, 64);
      const float wr = __shfl(wt, src, 64);
      if (has && cok) own_acc<VEC>(acc, wr, dout + (img + (cd >> 2)) * c, cq);
    }
    if (live && small && cok) own_store<VEC>(dinp + dd * c, cq, acc);
  }
}

// 5. gather, destinations with more than 16 entries (a clipped flow field piles samples onto
// the border): one workgroup per listed destination.  The segment's codes are marked in an
// LDS bitmap over a window of the image's code range (all of it when 4 h w <= OWN_WBITS), the
// four waves each sum a contiguous quarter of the window in code order, and the quarters are
// added in order: a fixed order for any n.
constexpr int OWN_WBITS = 1 << 20;    // 128 KB of bitmap
template <bool VEC>
__global__ __launch_bounds__(256) void own_gather_big(const float* __restrict__ dout,
                                                      const float* __restrict__ flow, int h,
                                                      int w, int c, int absolute,
                                                      const int* __restrict__ cnt,
                                                      const int* __restrict__ off,
                                                      const uint32_t* __restrict__ list,
                                                      const int* __restrict__ big_n,
                                                      const int* __restrict__ big,
                                                      float* __restrict__ dinp) {
  extern __shared__ uint32_t bm[];
  __shared__ float4 part[4][64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t codes = 4 * (int64_t)h * w;
  const int64_t wbits = codes < OWN_WBITS ? (codes + 31) / 32 * 32 : OWN_WBITS;
  const int nwords = (int)(wbits / 32);
  const int nb = *big_n;
  for (int bi = blockIdx.x; bi < nb; bi += gridDim.x) {
    const int64_t d = big[bi];
    const int64_t img = d / ((int64_t)h * w) * h * w;
    const int ne = cnt[d];
    const int64_t o0 = off[d];
    const int nq = VEC ? c >> 2 : c;
    for (int qb = 0; qb < nq; qb += 64) {                // 64 channel quads (channels) a sweep
      const int cq = qb + lane;
      const bool cok = cq < nq;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int64_t w0 = 0; w0 < codes; w0 += wbits) {   // code windows
        for (int k = tid; k < nwords; k += 256) bm[k] = 0u;
        __syncthreads();
        for (int e = tid; e < ne; e += 256) {
          const int64_t cd = (int64_t)list[o0 + e] - w0;
          if (cd >= 0 && cd < wbits) atomicOr(&bm[cd >> 5], 1u << (cd & 31));
        }
        __syncthreads();
        // wave wv: words [wv * nwords / 4, (wv + 1) * nwords / 4), in order; 64 words per
        // step, the nonzero ones visited in lane order
        const int k0 = (int)((int64_t)wv * nwords / 4), k1 = (int)((int64_t)(wv + 1) * nwords / 4);
        for (int kb = k0; kb < k1; kb += 64) {
          const uint32_t myw = kb + lane < k1 ? bm[kb + lane] : 0u;
          uint64_t nzm = __ballot(myw != 0u);
          while (nzm) {
            const int l = __builtin_ctzll(nzm);
            nzm &= nzm - 1;
            uint32_t word = (uint32_t)__shfl((int)myw, l, 64);
            while (word) {
              const int bit = __builtin_ctz(word);
              word &= word - 1;
              const uint32_t cd = (uint32_t)(w0 + 32 * (int64_t)(kb + l) + bit);
              const float wr = own_weight(flow, img, h, w, absolute, cd);
              if (cok) own_acc<VEC>(acc, wr, dout + (img + (cd >> 2)) * c, cq);
            }
          }
        }
        __syncthreads();                                // the bitmap is reused
      }
      part[wv][lane] = acc;
      __syncthreads();
      if (wv == 0 && cok) {
        float4 s = part[0][lane];
#pragma unroll
        for (int u = 1; u < 4; ++u) {
          s.x += part[u][lane].x;
          s.y += part[u][lane].y;
          s.z += part[u][lane].z;
          s.w += part[u][lane].w;
        }
        own_store<VEC>(dinp + d * c, cq, s);
      }
      __syncthreads();
    }
  }
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

// Workspace layout (256-byte aligned pieces): per destination pixel a count, a segment
// offset and a fill cursor (4 B each), the entry list (4 B per (pixel, corner)), the block
// sums of the scan, and the list of destinations with long segments + its length.
struct DetWs {
  size_t cnt, off, cursor, list, bsum, big, big_n, total;
  int nblk;
};

void det_layout(int64_t npix, DetWs& L) {
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  L.nblk = (int)cdiv(npix, OWN_SB);
  size_t o = 0;
  L.cnt = o, o += al(npix * 4);
  L.cursor = o, o += al(npix * 4);     // (cnt and cursor adjacent: one memset)
  L.off = o, o += al(npix * 4);
  L.list = o, o += al(4 * npix * 4);
  L.bsum = o, o += al((size_t)L.nblk * 4);
  L.big = o, o += al(npix * 4);
  L.big_n = o, o += 256;
  L.total = o;
}

}  // namespace

extern "C" {

size_t of_warp_bwd_det_workspace(int n, int h, int w, int c) {
  (void)c;
  if (n <= 0 || h <= 0 || w <= 0) return 0;
  DetWs L;
  det_layout((int64_t)n * h * w, L);
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
    det_layout(npix, L);
    OF_CHECK_ARG(ws && ws_bytes >= L.total, "warp bwd det: workspace too small");
    char* base = static_cast<char*>(ws);
    int* cnt = reinterpret_cast<int*>(base + L.cnt);
    int* cursor = reinterpret_cast<int*>(base + L.cursor);
    int* off = reinterpret_cast<int*>(base + L.off);
    uint32_t* list = reinterpret_cast<uint32_t*>(base + L.list);
    int* bsum = reinterpret_cast<int*>(base + L.bsum);
    int* big = reinterpret_cast<int*>(base + L.big);
    int* big_n = reinterpret_cast<int*>(base + L.big_n);
    if (hipMemsetAsync(cnt, 0, L.off - L.cnt, s) != hipSuccess ||
        hipMemsetAsync(big_n, 0, sizeof(int), s) != hipSuccess)
      return check_launch("warp_bwd_det: memset");
    const dim3 gp((unsigned)cdiv(npix, 256));
    hipLaunchKernelGGL(own_count, gp, dim3(256), 0, s, flow, n, h, w, absolute, cnt);
    hipLaunchKernelGGL(own_block_sums, dim3(L.nblk), dim3(256), 0, s, cnt, npix, bsum);
    hipLaunchKernelGGL(own_scan_sums, dim3(1), dim3(1024), 0, s, bsum, L.nblk);
    hipLaunchKernelGGL(own_block_scan, dim3(L.nblk), dim3(256), 0, s, cnt, npix, bsum, off);
    hipLaunchKernelGGL(own_fill, gp, dim3(256), 0, s, flow, n, h, w, absolute, off, cursor, list);
    if (int st = check_launch("warp_bwd_det: sort")) return st;
    if (vec)
      hipLaunchKernelGGL(own_gather<true>, dim3((unsigned)cdiv(npix * 16, 256)), dim3(256), 0, s,
                         dout, flow, n, h, w, c, absolute, cnt, off, list, dinp, big_n, big);
    else
      hipLaunchKernelGGL(own_gather<false>, dim3((unsigned)cdiv(npix * 16, 256)), dim3(256), 0, s,
                         dout, flow, n, h, w, c, absolute, cnt, off, list, dinp, big_n, big);
    const int64_t codes = 4 * (int64_t)h * w;
    const size_t bm_bytes =
        (size_t)(codes < OWN_WBITS ? (codes + 31) / 32 * 32 : OWN_WBITS) / 8;
    static bool attr = false;
    if (!attr) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(own_gather_big<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              OWN_WBITS / 8) != hipSuccess ||
          hipFuncSetAttribute(reinterpret_cast<const void*>(own_gather_big<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              OWN_WBITS / 8) != hipSuccess)
        return check_launch("warp_bwd_det: LDS attribute");
      attr = true;
    }
    if (vec)
      hipLaunchKernelGGL(own_gather_big<true>, dim3(2 * device_cus()), dim3(256), bm_bytes, s,
                         dout, flow, h, w, c, absolute, cnt, off, list, big_n, big, dinp);
    else
      hipLaunchKernelGGL(own_gather_big<false>, dim3(2 * device_cus()), dim3(256), bm_bytes, s,
                         dout, flow, h, w, c, absolute, cnt, off, list, big_n, big, dinp);
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
