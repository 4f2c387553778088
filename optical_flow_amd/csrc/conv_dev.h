// Device-side pieces shared by the conv kernel files (conv_f32.hip, conv_ws.hip): the GEMM
// argument block, the fused epilogues, and the bf16 staging helpers.
#pragma once
#include "common.h"

namespace oflow {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

// The 16-byte epilogues of conv_tile_bf16, conv_gemm_bf16 and conv_gemm_x3 (conv_f32.hip):
// rows in groups through epilogue_rows4c (1) or one row at a time (0, the round-2 form; A/B
// builds)
#ifndef EPC_BATCH
#define EPC_BATCH 1
#endif
constexpr int BK = 16;
constexpr int MAX_GROUPS = 4;

// A group = GEMM rows sharing one tap list (dgrad stride-2 phase classes); plain convs have
// a single identity group.
struct Group {
  int tiles_begin;   // first m-tile of this group in the flattened tile space
  int m_tiles;
  int M;             // rows of the group
  int hc, wc;        // phase mode: rows are (b, u, v), input pixel (2u+ry, 2v+rx)
  int ry, rx;
  int r0, s0, ns;    // taps (r0 + dt*(t/ns), s0 + dt*(t%ns)), t < ntaps
  int ntaps;
  int K;             // K of the group (multiple of BK)
  int64_t b_off;     // first packed-B row of the group
};

struct GemmArgs {
  int n, h, w, ho, wo;
  int kh, kw, stride, pt, pl;
  int kc;                 // channels per tap along K (fwd: cin_p, dgrad: cout_p) / M (wgrad)
  int dt;                 // tap step inside a group (1, or 2 for phase groups)
  int phase;              // dgrad phase-group mode (stride 2)
  int M, N, K;            // wgrad: M = taps*cin_p, K = output pixels
  const float* A; int lda; int64_t a_bytes;
  const float* B; int ldb; int nb; int64_t b_bytes;
  int64_t b_plane;        // conv_tile_x3: elements between the hi / mid / lo weight planes
  float* C; int ldc;      // final output (epilogue)
  const float* bias;
  const float* bn_g; const float* bn_b; const float* bn_m; const float* bn_v; float bn_eps;
  const float* res; int ldr;
  float* z; int ldz;
  int act; float alpha;
  const float* act_src; int ld_act;
  int splits;             // K slices over workgroups
  int k_per_split;        // elements of K per slice (multiple of BK)
  float* slab; int slab_ld;   // partials (wgrad always; fwd/dgrad when splits > 1)
  int64_t split_stride;
  int n_tiles;
  int tiles_total;        // sum over groups of m_tiles * n_tiles
  int colsum;             // wgrad: column sums of B (bias grad) into slab row M
  int bm;                 // M tile of the launched configuration
  int bn_tile;            // conv_tile_x3: N tile when not pick_bn(N) (0: pick_bn)
  // conv_wgrad_stem_x3<NP, true>: dz formed on load from the stem's max-pool / BN / ReLU
  // backward inputs (pooled gradient, the out0 gradient or NULL, the stem output y)
  const float* st_dyp; const float* st_g; const float* st_y;
  float* pool_out;        // conv_stem_x3: also the 2x2 / stride-2 max-pool of the output (ld N)
  int ngroups;
  int vec_ep;             // tile kernels: 4-column epilogue (N, every ld a multiple of 4,
                          // every row pointer 16-byte aligned)
  int act_post;           // dgrad: dx = act'(act_src) * (sum + res) instead of act' * sum + res
  // bf16 activation images (conv_b16i.hip): output image (C16, ldc16 bf16 per pixel; C may then
  // be NULL), the dgrad activation source as an image (act16; its sign is all act' needs), and
  // per-M-tile column sums of the dgrad output (col_part [m tile][N]: bias-gradient partials)
  uint16_t* C16; int ldc16;
  const uint16_t* act16; int ld_act16;
  float* col_part;
  int abl;                // conv_b16i.hip timing ablations (of_set_tuning key 21; 0 = none)
  // conv_b16i.hip direct epilogue (bf16 image output only): fwd writes its output's act' signs
  // (mask_out), the next layer's input gradient reads them (mask_in) instead of act16
  int direct16;
  uint4* mask_out;
  const uint4* mask_in;
  // fused BN backward partial sums (conv_tile_x3 input gradient, one K slice): the output t
  // (the gradient at the BN layer's output, after act') is also summed per channel, with
  // zhat = (act_src - bnp_res - beta) / gamma, into bnp [m tile][2][N] (sum t, sum t zhat)
  float* bnp;
  const float* bnp_res; int ld_bnp_res;
  const float* bnp_g; const float* bnp_b;
  Group grp[MAX_GROUPS];
};

// dgrad epilogue value: the input gradient v times the producer's activation derivative at s,
// plus an added gradient r -- or, with act_post, the derivative applied to the sum (the
// gradient of a ReLU output that has several consumers: encoder block inputs).
__device__ __forceinline__ float dgrad_ep(const GemmArgs& a, float v, float s, float r) {
  const float d = s > 0.f ? 1.f : (a.act == OF_ACT_LEAKY ? a.alpha : 0.f);
  return a.act_post ? (v + r) * d : v * d + r;
}

__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

// Input-gradient store of one row's channel quad n (one K slice) with the BN partial sums of
// the layer whose output is act_src: t = act'(s) (v + r) (act_post) or act'(s) v + r, then
// sb += t, sg += t zhat with zhat = (s - res_bn - beta) / gamma (bn_act_bwd_partial<true>'s
// recovery of the normalised value from the layer output).  ig = 1 / gamma, bt = beta.
__device__ __forceinline__ void dgrad_store4_bnp(const GemmArgs& a, int64_t row, int n,
                                                 float4 v4, const float4& bt, const float4& ig,
                                                 float4& sb, float4& sg) {
  const float4 s4 = *reinterpret_cast<const float4*>(&a.act_src[row * a.ld_act + n]);
  float4 r4 = make_float4(0.f, 0.f, 0.f, 0.f), q4 = r4;
  if (a.res) r4 = *reinterpret_cast<const float4*>(&a.res[row * a.ldr + n]);
  if (a.bnp_res) q4 = *reinterpret_cast<const float4*>(&a.bnp_res[row * a.ld_bnp_res + n]);
  const float4 t = make_float4(dgrad_ep(a, v4.x, s4.x, r4.x), dgrad_ep(a, v4.y, s4.y, r4.y),
                               dgrad_ep(a, v4.z, s4.z, r4.z), dgrad_ep(a, v4.w, s4.w, r4.w));
  *reinterpret_cast<float4*>(&a.C[row * a.ldc + n]) = t;
  add4(sb, t);
  sg.x += t.x * ((s4.x - q4.x - bt.x) * ig.x);
  sg.y += t.y * ((s4.y - q4.y - bt.y) * ig.y);
  sg.z += t.z * ((s4.z - q4.z - bt.z) * ig.z);
  sg.w += t.w * ((s4.w - q4.w - bt.w) * ig.w);
}

__device__ __forceinline__ float act_fwd(float v, int act, float alpha) {
  if (act == OF_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == OF_ACT_LEAKY) return v > 0.f ? v : alpha * v;
  return v;
}

// Output pixel row of group-local GEMM row m (identity unless dgrad phase groups).
__device__ __forceinline__ int64_t out_row(const GemmArgs& a, const Group& g, int m) {
  if (!a.phase) return m;
  const int hw = g.hc * g.wc;
  const int b = m / hw, rem = m - b * hw;
  const int u = rem / g.wc, v = rem - u * g.wc;
  return ((int64_t)b * a.h + 2 * u + g.ry) * a.w + 2 * v + g.rx;
}

// The epilogue's second input for one element: the residual (fwd) or the producer's output
// whose activation derivative scales dx (dgrad).  Call sites gather all of a lane's values
// before the first store: interleaved, every load would wait behind the previous store (the
// compiler cannot prove a.C does not alias them).
// dgrad: s = the producer's output (activation derivative), r = a gradient to add (the
// residual branch's, so the autograd sum of the two input gradients needs no extra pass).
struct EpAux {
  float s, r;
};
template <int MODE>
__device__ __forceinline__ EpAux epilogue_aux(const GemmArgs& a, int64_t row, int n) {
  if (MODE == MODE_FWD) return {a.res ? a.res[row * a.ldr + n] : 0.f, 0.f};
  if (MODE == MODE_DGRAD)
    return {a.act_src ? a.act_src[row * a.ld_act + n] : 1.f, a.res ? a.res[row * a.ldr + n] : 0.f};
  return {0.f, 0.f};
}

// Aux values gathered ahead of the stores: the whole 16-value MFMA fragment for dgrad (the
// decoder's act_src on every layer); 4 for fwd, whose residual only the encoder has and whose
// epilogue registers set the kernels' occupancy.
#ifndef OF_EPG_FWD
#define OF_EPG_FWD 4
#endif
#ifndef OF_EPG_DGRAD
#define OF_EPG_DGRAD 8
#endif
template <int MODE>
constexpr int EP_GATHER = MODE == MODE_DGRAD ? OF_EPG_DGRAD : OF_EPG_FWD;

// Fused epilogue for one element (fwd / dgrad), v = the full K sum, aux = epilogue_aux.
template <int MODE>
__device__ __forceinline__ void epilogue_store(const GemmArgs& a, int64_t row, int n, float v,
                                               float bias, float scale, float shift, EpAux aux) {
  if (MODE == MODE_FWD) {
    v += bias;
    if (a.z) a.z[row * a.ldz + n] = v;
    if (a.bn_g) v = v * scale + shift;
    v += aux.s;
    v = act_fwd(v, a.act, a.alpha);
  } else if (MODE == MODE_DGRAD) {
    v = dgrad_ep(a, v, aux.s, aux.r);
  }
  a.C[row * a.ldc + n] = v;
}

template <int MODE>
__device__ __forceinline__ void column_params(const GemmArgs& a, int n, float& bias,
                                              float& scale, float& shift);

// The fused epilogue of epilogue_store for four consecutive columns n .. n + 3 of one row,
// with 16-byte loads and stores (a.vec_ep: N and every leading dimension a multiple of 4,
// 16-byte aligned bases).  splits > 1 writes the raw sums to this K slice's slab row.
template <int MODE>
__device__ __forceinline__ void epilogue_store4(const GemmArgs& a, int split, int64_t row, int n,
                                                float4 v4) {
  if (a.splits > 1) {
    *reinterpret_cast<float4*>(&a.slab[(int64_t)split * a.split_stride + row * a.slab_ld + n]) = v4;
    return;
  }
  float v[4] = {v4.x, v4.y, v4.z, v4.w};
  if (MODE == MODE_FWD) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float bias, scale, shift;
      column_params<MODE>(a, n + e, bias, scale, shift);
      v[e] += bias;
      (void)scale;
      (void)shift;
    }
    if (a.z) *reinterpret_cast<float4*>(&a.z[row * a.ldz + n]) = make_float4(v[0], v[1], v[2], v[3]);
    if (a.bn_g) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float bias, scale, shift;
        column_params<MODE>(a, n + e, bias, scale, shift);
        v[e] = v[e] * scale + shift;
      }
    }
    if (a.res) {
      const float4 r = *reinterpret_cast<const float4*>(&a.res[row * a.ldr + n]);
      v[0] += r.x;
      v[1] += r.y;
      v[2] += r.z;
      v[3] += r.w;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = act_fwd(v[e], a.act, a.alpha);
  } else if (MODE == MODE_DGRAD) {
    float4 s4 = make_float4(1.f, 1.f, 1.f, 1.f), r4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.act_src) s4 = *reinterpret_cast<const float4*>(&a.act_src[row * a.ld_act + n]);
    if (a.res) r4 = *reinterpret_cast<const float4*>(&a.res[row * a.ldr + n]);
    v[0] = dgrad_ep(a, v[0], s4.x, r4.x);
    v[1] = dgrad_ep(a, v[1], s4.y, r4.y);
    v[2] = dgrad_ep(a, v[2], s4.z, r4.z);
    v[3] = dgrad_ep(a, v[3], s4.w, r4.w);
  }
  *reinterpret_cast<float4*>(&a.C[row * a.ldc + n]) = make_float4(v[0], v[1], v[2], v[3]);
}

// epilogue_store4 for R rows of one lane's column quad n .. n + 3 (row[r] valid where bit r of
// ok is set): the column parameters are loaded once, and every row's residual / activation-
// source quad before the first store.  (In epilogue_store4's per-row form the compiler cannot
// prove a.C does not alias those inputs, so each row's loads wait behind the previous row's
// store and their latency is exposed once per row.)
template <int MODE, int R>
__device__ __forceinline__ void epilogue_rows4(const GemmArgs& a, int split, const int64_t* row,
                                               unsigned ok, int n, const float4* v) {
  if (a.splits > 1) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if ((ok >> r) & 1)
        *reinterpret_cast<float4*>(&a.slab[(int64_t)split * a.split_stride + row[r] * a.slab_ld + n]) = v[r];
    return;
  }
  float4 s4[R], r4[R];
  if (MODE == MODE_FWD) {
    float bias[4], scale[4], shift[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) column_params<MODE>(a, n + e, bias[e], scale[e], shift[e]);
#pragma unroll
    for (int r = 0; r < R; ++r)
      r4[r] = a.res && ((ok >> r) & 1) ? *reinterpret_cast<const float4*>(&a.res[row[r] * a.ldr + n])
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!((ok >> r) & 1)) continue;
      float x[4] = {v[r].x + bias[0], v[r].y + bias[1], v[r].z + bias[2], v[r].w + bias[3]};
      if (a.z) *reinterpret_cast<float4*>(&a.z[row[r] * a.ldz + n]) = make_float4(x[0], x[1], x[2], x[3]);
      const float rr[4] = {r4[r].x, r4[r].y, r4[r].z, r4[r].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (a.bn_g) x[e] = x[e] * scale[e] + shift[e];
        x[e] = act_fwd(x[e] + rr[e], a.act, a.alpha);
      }
      *reinterpret_cast<float4*>(&a.C[row[r] * a.ldc + n]) = make_float4(x[0], x[1], x[2], x[3]);
    }
  } else if (MODE == MODE_DGRAD) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool k = (ok >> r) & 1;
      s4[r] = a.act_src && k ? *reinterpret_cast<const float4*>(&a.act_src[row[r] * a.ld_act + n])
                             : make_float4(1.f, 1.f, 1.f, 1.f);
      r4[r] = a.res && k ? *reinterpret_cast<const float4*>(&a.res[row[r] * a.ldr + n])
                         : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!((ok >> r) & 1)) continue;
      *reinterpret_cast<float4*>(&a.C[row[r] * a.ldc + n]) =
          make_float4(dgrad_ep(a, v[r].x, s4[r].x, r4[r].x), dgrad_ep(a, v[r].y, s4[r].y, r4[r].y),
                      dgrad_ep(a, v[r].z, s4[r].z, r4[r].z), dgrad_ep(a, v[r].w, s4[r].w, r4[r].w));
    }
  }
}

// epilogue_rows4 for rows and a column clamped into the tensors (row[r] always a valid pixel,
// nl = min(n, N - 4)): every residual / activation-source quad is loaded unconditionally, all
// of them before the first store, and only the stores are masked by ok -- a guarded load per
// row was compiled to a branch and a wait per row (the loads reuse the address registers).
template <int MODE, int R>
__device__ __forceinline__ void epilogue_rows4c(const GemmArgs& a, int split, const int64_t* row,
                                                unsigned ok, int n, int nl, const float4* v) {
  if (a.splits > 1) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if ((ok >> r) & 1)
        *reinterpret_cast<float4*>(&a.slab[(int64_t)split * a.split_stride + row[r] * a.slab_ld + n]) = v[r];
    return;
  }
  float4 s4[R], r4[R];
#pragma unroll
  for (int r = 0; r < R; ++r) s4[r] = make_float4(1.f, 1.f, 1.f, 1.f), r4[r] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (MODE == MODE_DGRAD && a.act_src) {
#pragma unroll
    for (int r = 0; r < R; ++r) s4[r] = *reinterpret_cast<const float4*>(&a.act_src[row[r] * a.ld_act + nl]);
  }
  if (a.res) {
#pragma unroll
    for (int r = 0; r < R; ++r) r4[r] = *reinterpret_cast<const float4*>(&a.res[row[r] * a.ldr + nl]);
  }
  if (MODE == MODE_FWD) {
    float bias[4], scale[4], shift[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) column_params<MODE>(a, nl + e, bias[e], scale[e], shift[e]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!((ok >> r) & 1)) continue;
      float x[4] = {v[r].x + bias[0], v[r].y + bias[1], v[r].z + bias[2], v[r].w + bias[3]};
      if (a.z) *reinterpret_cast<float4*>(&a.z[row[r] * a.ldz + n]) = make_float4(x[0], x[1], x[2], x[3]);
      const float rr[4] = {r4[r].x, r4[r].y, r4[r].z, r4[r].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (a.bn_g) x[e] = x[e] * scale[e] + shift[e];
        x[e] = act_fwd(x[e] + rr[e], a.act, a.alpha);
      }
      *reinterpret_cast<float4*>(&a.C[row[r] * a.ldc + n]) = make_float4(x[0], x[1], x[2], x[3]);
    }
  } else if (MODE == MODE_DGRAD) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!((ok >> r) & 1)) continue;
      *reinterpret_cast<float4*>(&a.C[row[r] * a.ldc + n]) =
          make_float4(dgrad_ep(a, v[r].x, s4[r].x, r4[r].x), dgrad_ep(a, v[r].y, s4[r].y, r4[r].y),
                      dgrad_ep(a, v[r].z, s4[r].z, r4[r].z), dgrad_ep(a, v[r].w, s4[r].w, r4[r].w));
    }
  }
}

// epilogue_rows4c's input gradient (one K slice) with dgrad_store4_bnp's BN partial sums: the
// act' source, added-gradient and BN residual quads of all R rows loaded (clamped, unmasked)
// before the first store; stores and sums masked by ok.
template <int R>
__device__ __forceinline__ void dgrad_rows4c_bnp(const GemmArgs& a, const int64_t* row,
                                                 unsigned ok, int n, int nl, const float4* v,
                                                 const float4& bt, const float4& ig, float4& sb,
                                                 float4& sg) {
  float4 s4[R], r4[R], q4[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    s4[r] = *reinterpret_cast<const float4*>(&a.act_src[row[r] * a.ld_act + nl]);
    r4[r] = a.res ? *reinterpret_cast<const float4*>(&a.res[row[r] * a.ldr + nl])
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    q4[r] = a.bnp_res ? *reinterpret_cast<const float4*>(&a.bnp_res[row[r] * a.ld_bnp_res + nl])
                      : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (!((ok >> r) & 1)) continue;
    const float4 t = make_float4(dgrad_ep(a, v[r].x, s4[r].x, r4[r].x), dgrad_ep(a, v[r].y, s4[r].y, r4[r].y),
                                 dgrad_ep(a, v[r].z, s4[r].z, r4[r].z), dgrad_ep(a, v[r].w, s4[r].w, r4[r].w));
    *reinterpret_cast<float4*>(&a.C[row[r] * a.ldc + n]) = t;
    add4(sb, t);
    sg.x += t.x * ((s4[r].x - q4[r].x - bt.x) * ig.x);
    sg.y += t.y * ((s4[r].y - q4[r].y - bt.y) * ig.y);
    sg.z += t.z * ((s4[r].z - q4[r].z - bt.z) * ig.z);
    sg.w += t.w * ((s4[r].w - q4[r].w - bt.w) * ig.w);
  }
}

// One wave's 32 x 32 accumulator block in the v_mfma_f32_32x32x* layout (column lane & 31,
// rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5)) through a private 4 KB LDS image E, back as
// float4 rows: f(row 0..31, column quad 0..7, value) for the 4 rows x 1 quad each lane owns.
// Unpadded 32-float rows: the ds_write_b32 of a lane group cover one row (32 banks) and the
// ds_read_b128 groups (rows 4 apart sharing a slot base) hit 16 distinct slots.
template <typename F>
__device__ __forceinline__ void transpose32(float* E, const f32x16& acc, int lane, F&& f) {
  const int lrow = lane & 31, lk = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) E[((r & 3) + 8 * (r >> 2) + 4 * lk) * 32 + lrow] = acc[r];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int c4 = lane & 7, rr = lane >> 3;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = 8 * q + rr;
    f(row, c4, *reinterpret_cast<const float4*>(&E[row * 32 + 4 * c4]));
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // reads done before the next block
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int MODE>
__device__ __forceinline__ void column_params(const GemmArgs& a, int n, float& bias,
                                              float& scale, float& shift) {
  bias = 0.f;
  scale = 1.f;
  shift = 0.f;
  if (MODE == MODE_FWD) {
    if (a.bias) bias = a.bias[n];
    if (a.bn_g) {
      scale = a.bn_g[n] * rsqrtf(a.bn_v[n] + a.bn_eps);
      shift = a.bn_b[n] - a.bn_m[n] * scale;
    }
  }
}


typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifndef OF_TF_H
#define OF_TF_H 4
#define OF_TF_W 32
#endif
constexpr int TF_H = OF_TF_H, TF_W = OF_TF_W;

__device__ __forceinline__ int x3_sw(int p) { return ((p >> 2) & 1) << 1; }

// One LDS-DMA wave-instruction (buffer_load_dwordx4 ... lds): lane L's 16 bytes at byte
// offset voff + soff of r land at dst + 16 L (dst wave-uniform); out-of-range lanes write 0.
__device__ __forceinline__ void dma16_to_lds(rsrc_t r, uint4* dst, uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16,
                                           voff, soff, 0, 0);
}

// LDS byte address of a __shared__ pointer, and a 16-byte LDS read in inline asm: no memory
// operand, so hipcc does not wait for in-flight LDS DMAs (vmcnt) before it -- the caller
// orders it (counted vmcnt + barrier before, s_waitcnt lgkmcnt(0) + sched_barrier(0) after).
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ uint4 ds_read16(uint32_t addr) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return make_uint4(r[0], r[1], r[2], r[3]);
}

// 4 fp32 -> 4 bf16 (RNE, v_cvt_pk_bf16_f32), element 0 in the low half of .x
__device__ __forceinline__ uint2 pack_bf16x4(const float4& v) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 r;
  r[0] = (__bf16)v.x;
  r[1] = (__bf16)v.y;
  r[2] = (__bf16)v.z;
  r[3] = (__bf16)v.w;
  return __builtin_bit_cast(uint2, r);
}

// Direct fp32 forward epilogue of a 16x16x32-MFMA tile kernel (conv_f32.hip tile_x3_body;
// conv_b16i.hip has its own, with the bf16 image and sign-mask outputs): bias / BN / act on
// the accumulators in their MFMA layout (lane: column 16 j + l16, rows 16 i + 4 lq + r),
// adjacent columns swapped between lane pairs (DPP) so each lane writes 2 rows x 2 columns
// with 64-bit LDS writes into the wave's row image (half the rows per pass, 32-byte padded
// pitch: conflict-free), then whole 16-byte row chunks to C: every store instruction writes
// full 128-byte lines, where the per-pass transposes store 64-byte row pieces.  lds: this
// wave's region, (WM / 2) * (WN * 4 + 32) bytes.  Rows: tile pixel m -> (oy0 + m / TW,
// ox0 + m % TW) of image `img` (OH x OW).
template <int SM, int SN, int WM, int WN, int TW>
__device__ __forceinline__ void direct_fwd_f32(const GemmArgs& a, f32x4 (&acc)[SM][SN], char* lds,
                                               int lane, int wm0, int wn0, int n0, int oy0,
                                               int ox0, int OH, int OW, int64_t img) {
  static_assert(SM % 2 == 0, "two passes of SM / 2 row blocks");
  constexpr int P = WN * 4 + 32, LR = WN / 4, NR = WM / 2;
  static_assert((NR * LR) % 64 == 0, "whole store instructions");
  const int l16 = lane & 15, lq = lane >> 4;
  const bool even = !(l16 & 1);
  float cb[SN], cs[SN], ct[SN];
#pragma unroll
  for (int j = 0; j < SN; ++j) {
    const int n = n0 + wn0 + 16 * j + l16;
    cb[j] = 0.f, cs[j] = 1.f, ct[j] = 0.f;
    if (n < a.N) column_params<MODE_FWD>(a, n, cb[j], cs[j], ct[j]);
  }
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int ii = 0; ii < SM / 2; ++ii) {
      const int i = hf * (SM / 2) + ii;
#pragma unroll
      for (int j = 0; j < SN; ++j) {
        float x[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t = acc[i][j][r] + cb[j];
          if (a.bn_g) t = t * cs[j] + ct[j];
          x[r] = act_fwd(t, a.act, a.alpha);
        }
        const float p0 = even ? x[2] : x[0], p1 = even ? x[3] : x[1];
        const float q0 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
                                                       __builtin_bit_cast(int, p0), 0xB1, 0xF, 0xF, false));
        const float q1 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
                                                       __builtin_bit_cast(int, p1), 0xB1, 0xF, 0xF, false));
        const int row0 = 16 * ii + 4 * lq + (even ? 0 : 2);
        char* d = lds + row0 * P + (16 * j + (l16 & ~1)) * 4;
        *reinterpret_cast<float2*>(d) = even ? make_float2(x[0], q0) : make_float2(q0, x[2]);
        *reinterpret_cast<float2*>(d + P) = even ? make_float2(x[1], q1) : make_float2(q1, x[3]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int it = 0; it < NR * LR / 64; ++it) {
      const int c = lane + 64 * it, row = c / LR, part = c - row * LR;
      const uint4 v = *reinterpret_cast<const uint4*>(lds + row * P + 16 * part);
      const int mt = wm0 + 16 * (hf * (SM / 2)) + row;
      const int oy = oy0 + mt / TW, ox = ox0 + mt % TW;
      const int ch = n0 + wn0 + 4 * part;
      if (oy < OH && ox < OW && ch < a.N)
        *reinterpret_cast<uint4*>(&a.C[(img + (int64_t)oy * OW + ox) * a.ldc + ch]) = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// Direct fp32 input-gradient epilogue, the counterpart of direct_fwd_f32: the raw sums go
// through the same row image; then each lane takes whole 16-byte row chunks, loads the
// activation source and residual quads of all its chunks first (addresses clamped into the
// tensors, so no load sits behind a branch and all are in flight together), and stores
// dgrad_ep of each element -- full 128-byte lines for the loads and the stores, where the
// per-pass transposes move 64-byte row pieces with one chunk's loads in flight.
template <int SM, int SN, int WM, int WN, int TW>
__device__ __forceinline__ void direct_dgrad_f32(const GemmArgs& a, f32x4 (&acc)[SM][SN],
                                                 char* lds, int lane, int wm0, int wn0, int n0,
                                                 int oy0, int ox0, int OH, int OW, int64_t img) {
  static_assert(SM % 2 == 0, "two passes of SM / 2 row blocks");
  constexpr int P = WN * 4 + 32, LR = WN / 4, NR = WM / 2, IT = NR * LR / 64;
  static_assert((NR * LR) % 64 == 0, "whole store instructions");
  const int l16 = lane & 15, lq = lane >> 4;
  const bool even = !(l16 & 1);
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int ii = 0; ii < SM / 2; ++ii) {
      const int i = hf * (SM / 2) + ii;
#pragma unroll
      for (int j = 0; j < SN; ++j) {
        const f32x4 x = acc[i][j];
        const float p0 = even ? x[2] : x[0], p1 = even ? x[3] : x[1];
        const float q0 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
                                                       __builtin_bit_cast(int, p0), 0xB1, 0xF, 0xF, false));
        const float q1 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
                                                       __builtin_bit_cast(int, p1), 0xB1, 0xF, 0xF, false));
        const int row0 = 16 * ii + 4 * lq + (even ? 0 : 2);
        char* d = lds + row0 * P + (16 * j + (l16 & ~1)) * 4;
        *reinterpret_cast<float2*>(d) = even ? make_float2(x[0], q0) : make_float2(q0, x[2]);
        *reinterpret_cast<float2*>(d + P) = even ? make_float2(x[1], q1) : make_float2(q1, x[3]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // chunks in groups of G: the group's activation-source / residual quads are all loaded
    // before its first store (G = 4 bounds the registers: 8 chunks spilled the 4-wave form)
    constexpr int G = IT < 4 ? IT : 4;
    static_assert(IT % G == 0, "whole groups");
#pragma unroll
    for (int g0 = 0; g0 < IT; g0 += G) {
      int64_t prow[G];
      int chs[G];
      bool ok[G];
      float4 s4[G], r4[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int c = lane + 64 * (g0 + g), row = c / LR, part = c - row * LR;
        const int mt = wm0 + 16 * (hf * (SM / 2)) + row;
        const int oy = oy0 + mt / TW, ox = ox0 + mt % TW;
        const int ch = n0 + wn0 + 4 * part;
        ok[g] = oy < OH && ox < OW && ch < a.N;
        prow[g] = img + (int64_t)min(oy, OH - 1) * OW + min(ox, OW - 1);
        chs[g] = min(ch, a.N - 4);
        s4[g] = a.act_src ? *reinterpret_cast<const float4*>(&a.act_src[prow[g] * a.ld_act + chs[g]])
                          : make_float4(1.f, 1.f, 1.f, 1.f);
        r4[g] = a.res ? *reinterpret_cast<const float4*>(&a.res[prow[g] * a.ldr + chs[g]])
                      : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int c = lane + 64 * (g0 + g), row = c / LR, part = c - row * LR;
        const float4 v = *reinterpret_cast<const float4*>(lds + row * P + 16 * part);
        if (ok[g])
          *reinterpret_cast<float4*>(&a.C[prow[g] * a.ldc + chs[g]]) =
              make_float4(dgrad_ep(a, v.x, s4[g].x, r4[g].x), dgrad_ep(a, v.y, s4[g].y, r4[g].y),
                          dgrad_ep(a, v.z, s4[g].z, r4[g].z), dgrad_ep(a, v.w, s4[g].w, r4[g].w));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// conv_ws.hip: launch conv_tile_ws for a planned bf16 3x3 fwd / dgrad (no timing, no split-K
// epilogue: the caller's)
int launch_tile_ws_kernel(const GemmArgs& a, int mode, hipStream_t s);

}  // namespace oflow
