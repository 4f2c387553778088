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
//         stride 2 = the transposed convolution, run as 4 "phase groups": the input pixels
//         of one (row, col) parity only see the taps of matching parity, so each group's
//         K loop visits exactly its taps (no zero-masked MACs) and the packed Wd holds the
//         taps grouped by phase.
//   WGRAD C[m=(tap,ci)][n=cout]  = sum_{k=out pixel} x[pix(k,tap)][ci] * dy[k][n]
//         (split-K over pixels into fp32 slabs, reduced deterministically; the bias
//          gradient = column sums of dy rides along in the same pass).
//
// Tiling: BM x BN x 16 per 256-thread workgroup (4 waves), each wave an (BM/WAVES_M) x
// (BN/WAVES_N) block of 32x32 MFMA tiles.  LDS holds both operands k-major ([k][m], [k][n]) so
// the MFMA operand fetch is one conflict-free ds_read_b32 per lane (lanes 0-31 row k,
// lanes 32-63 row k+1); the fragments of k-step s+1 are read while the MFMAs of step s issue.
// Global->LDS is register-staged and double-buffered: the loads of chunk c+1 are issued
// before the MFMAs of chunk c, one barrier per chunk.  Grids with fewer tiles than the chip
// has CUs split K over workgroups into fp32 slabs; a separate pass sums them and runs the
// epilogue.  Fused epilogues: bias, BN-inference affine, residual add, ReLU/LeakyReLU (fwd);
// the producer layer's activation derivative (dgrad).  Work-group ids are remapped so that
// consecutive tiles (and all tiles of one K slice) run on one XCD and share its L2.
#include "common.h"
#include "conv_dev.h"
#include "conv_narrow.h"

#include <algorithm>

namespace oflow {

// (shared device helpers: conv_dev.h)
template <int BM, int BN, int WAVES_M, int WAVES_N, int MODE>
__global__ __launch_bounds__(256, 2) void conv_gemm_f32(GemmArgs a) {
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  static_assert(TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "tile");
  constexpr bool A_KCONTIG = (MODE != MODE_WGRAD);
  constexpr int SA = BM + 4;
  constexpr int SB = BN + 4;
  constexpr int A_SLOTS = BM * BK / 4 / 256;
  constexpr int B_QUADS = BK * BN / 4;
  constexpr int B_SLOTS = (B_QUADS + 255) / 256;
  static_assert(A_SLOTS >= 1, "BM >= 64");

  // One LDS array: both operand buffers, and after the main loop the epilogue's 4 KB
  // per-wave transpose images.
  static_assert(2 * BK * (SA + SB) >= 4 * 1024, "epilogue images fit LDS");
  __shared__ float smem[2 * BK * (SA + SB)];
  float (*As)[BK * SA] = reinterpret_cast<float (*)[BK * SA]>(smem);
  float (*Bs)[BK * SB] = reinterpret_cast<float (*)[BK * SB]>(smem + 2 * BK * SA);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // XCD-aware bijective remap: consecutive work ids -> one XCD's L2 (cdna guide T1).
  // Stride-2 input gradients (phase groups of 4 / 2 / 2 / 1 taps, contiguous in the tile
  // space) skip the XCD remap: it would hand each XCD the tiles of one or two groups (the
  // 4-tap group's XCDs then run 1.8x the average), while block order deals every group
  // evenly over the 8 XCDs and starts the longest tiles first.
  const int wgid = a.phase ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  // work id = split * tiles_total + tile: all tiles of one K slice are consecutive.
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_n = tile % a.n_tiles;
  const int tile_mg = tile / a.n_tiles;
  int gi = 0;
#pragma unroll
  for (int g = 1; g < MAX_GROUPS; ++g)
    if (g < a.ngroups && tile_mg >= a.grp[g].tiles_begin) gi = g;
  const Group& G = a.grp[gi];
  const int tile_m = tile_mg - G.tiles_begin;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int M = G.M;

  // ---------------- K range -------------------------------------------------------------
  const int Kg = (MODE == MODE_WGRAD) ? a.K : G.K;
  const int k_begin = split * a.k_per_split;
  const int k_end = min(Kg, k_begin + a.k_per_split);
  const int nchunks = k_end > k_begin ? (k_end - k_begin + BK - 1) / BK : 0;

  const rsrc_t ra_src = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rb_src = make_rsrc(a.B, a.b_bytes);

  // ---------------- A loader state ------------------------------------------------------
  // fwd/dgrad: wave w loads k-quad w of every chunk (4 channels of one tap) for rows
  //   lane + 64*i; the tap walk (t, ci) is wave-uniform (scalar), each row keeps a byte
  //   offset of its tap-origin pixel and a bitmask of its in-bounds taps, so one chunk costs
  //   an add and a select per load (out-of-bounds -> past num_records -> 0).
  // wgrad: thread -> (mq = tid % (BM/4), krow = tid/(BM/4) + i*256/(BM/4)), fixed (tap, ci).
  int a_off[A_SLOTS];                 // fwd/dgrad: byte offset of tap (0,0) of the row
  uint64_t a_msk[A_SLOTS];            // fwd/dgrad: in-bounds taps
  int ks_t = 0, ks_tr = 0, ks_ts = 0, ks_ci = 0;
  int tap_step = 0;                   // koff(bytes) = tap_sign*(tr*src_w + ts)*lda*4 + ci*4
  int wm_r = 0, wm_s = 0, wm_ci = 0;  // wgrad: per-thread fixed m
  bool wm_ok = false;
  int a_oy[A_SLOTS], a_ox[A_SLOTS], a_b[A_SLOTS], a_kb[A_SLOTS];   // wgrad: pixel state

  if constexpr (A_KCONTIG) {
    const int src_h = (MODE == MODE_DGRAD) ? a.ho : a.h;
    const int src_w = (MODE == MODE_DGRAD) ? a.wo : a.w;
#pragma unroll
    for (int i = 0; i < A_SLOTS; ++i) {
      const int m = m0 + lane + 64 * i;
      const bool okm = m < M;
      const int mm = okm ? m : 0;
      int b, yb, xb;   // tap-origin source pixel (may be outside the image)
      if (MODE == MODE_FWD) {
        const int hw = a.ho * a.wo;
        b = mm / hw;
        const int rem = mm - b * hw;
        const int oy = rem / a.wo, ox = rem - oy * a.wo;
        yb = oy * a.stride - a.pt;
        xb = ox * a.stride - a.pl;
      } else if (a.phase) {
        const int hw = G.hc * G.wc;
        b = mm / hw;
        const int rem = mm - b * hw;
        const int u = rem / G.wc, v = rem - u * G.wc;
        yb = (2 * u + G.ry + a.pt - G.r0) >> 1;
        xb = (2 * v + G.rx + a.pl - G.s0) >> 1;
      } else {
        const int hw = a.h * a.w;
        b = mm / hw;
        const int rem = mm - b * hw;
        const int iy = rem / a.w, ix = rem - iy * a.w;
        yb = iy + a.pt;
        xb = ix + a.pl;
      }
      a_off[i] = (int)(((int64_t)(b * src_h + yb) * src_w + xb) * a.lda * 4);
      uint64_t msk = 0;
      if (okm) {
        // taps are row-major over (tr, ts); mask = in-bounds rows x in-bounds columns
        uint64_t colmask = 0;
        for (int ts = 0; ts < G.ns; ++ts) {
          const int sx = (MODE == MODE_FWD) ? xb + ts : xb - ts;
          if ((unsigned)sx < (unsigned)src_w) colmask |= (uint64_t)1 << ts;
        }
        int t = 0;
        for (int tr = 0; t < G.ntaps; ++tr, t += G.ns) {
          const int sy = (MODE == MODE_FWD) ? yb + tr : yb - tr;
          if ((unsigned)sy < (unsigned)src_h) msk |= colmask << t;
        }
        if (G.ntaps < 64) msk &= ((uint64_t)1 << G.ntaps) - 1;
      }
      a_msk[i] = msk;
    }
    const int k0 = k_begin + wave * 4;
    ks_t = k0 / a.kc;
    ks_ci = k0 - ks_t * a.kc;
    ks_tr = ks_t / G.ns;
    ks_ts = ks_t - ks_tr * G.ns;
    tap_step = (MODE == MODE_FWD ? 1 : -1) * src_w * a.lda * 4;   // bytes per tap row
  } else {
    constexpr int MQ = BM / 4;
    const int mq = tid % MQ;
    const int m = m0 + 4 * mq;
    wm_ok = m < M;
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
      const bool tap_ok = ks_t < G.ntaps;
      const int koff = (ks_tr * tap_step) + (MODE == MODE_FWD ? 1 : -1) * ks_ts * a.lda * 4 +
                       ks_ci * 4;
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        const bool ok = tap_ok && ((a_msk[i] >> ks_t) & 1);
        ra[i] = bload4(ra_src, ok ? (uint32_t)(a_off[i] + koff) : kOOB);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        const int sy = a_oy[i] * a.stride - a.pt + wm_r;
        const int sx = a_ox[i] * a.stride - a.pl + wm_s;
        const bool ok = wm_ok && a_kb[i] < k_end && (unsigned)sy < (unsigned)a.h &&
                        (unsigned)sx < (unsigned)a.w;
        const int off = (((a_b[i] * a.h + sy) * a.w + sx) * a.lda + wm_ci) * 4;
        ra[i] = bload4(ra_src, ok ? (uint32_t)off : kOOB);
      }
    }
  };
  auto advance_a = [&]() {
    if constexpr (A_KCONTIG) {
      ks_ci += BK;
      while (ks_ci >= a.kc) {
        ks_ci -= a.kc;
        ++ks_t;
        if (++ks_ts >= G.ns) {
          ks_ts = 0;
          ++ks_tr;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        a_kb[i] += BK;
        a_ox[i] += BK;
        if (a_ox[i] >= a.wo) {           // row wrap (rare: every wo/BK chunks)
          const int q = a_ox[i] / a.wo;
          a_ox[i] -= q * a.wo;
          a_oy[i] += q;
          if (a_oy[i] >= a.ho) {
            const int q2 = a_oy[i] / a.ho;
            a_oy[i] -= q2 * a.ho;
            a_b[i] += q2;
          }
        }
      }
    }
  };
  auto store_a = [&](int buf) {
    if constexpr (A_KCONTIG) {
      // 64 consecutive rows of one k per wave-instruction: conflict-free ds_write_b32
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        float* p = &As[buf][(wave * 4) * SA + lane + 64 * i];
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
  // per slot a fixed byte offset (row krow, column quad); the chunk adds b_k rows.
  const int64_t b_base = (MODE == MODE_WGRAD) ? 0 : G.b_off;
  uint32_t b_off[B_SLOTS];
  int b_row[B_SLOTS];
#pragma unroll
  for (int i = 0; i < B_SLOTS; ++i) {
    constexpr int NQ = BN / 4;
    const int slot = tid + 256 * i;
    const int krow = slot / NQ, nq = slot - krow * NQ;
    const int n = n0 + 4 * nq;
    b_row[i] = krow;
    b_off[i] = (slot < B_QUADS && n < a.nb) ? (uint32_t)(((b_base + krow) * a.ldb + n) * 4)
                                            : kOOB;
  }
  int b_k = k_begin;   // first k row of the current chunk
  auto load_b = [&]() {
    const uint32_t kadd = (uint32_t)b_k * (uint32_t)a.ldb * 4u;
#pragma unroll
    for (int i = 0; i < B_SLOTS; ++i) {
      bool ok = b_off[i] != kOOB;
      if (MODE == MODE_WGRAD) ok = ok && (b_k + b_row[i] < k_end);
      rb[i] = bload4(rb_src, ok ? b_off[i] + kadd : kOOB);
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

  const bool do_colsum = (MODE == MODE_WGRAD) && a.colsum && tile_m == 0;
  float colacc = 0.f;

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
    if (do_colsum && tid < BN) {
#pragma unroll
      for (int k = 0; k < BK; ++k) colacc += bs[k * SB + tid];
    }
    // Operand fragments of k-step st+1 are read while the MFMAs of step st issue.
    float av[2][TM], bv[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) av[0][i] = as[lk * SA + wm0 + 32 * i + lrow];
#pragma unroll
    for (int j = 0; j < TN; ++j) bv[0][j] = bs[lk * SB + wn0 + 32 * j + lrow];
#pragma unroll
    for (int st = 0; st < BK / 2; ++st) {
      const int cur = st & 1;
      if (st + 1 < BK / 2) {
        const int kk = 2 * (st + 1) + lk;
#pragma unroll
        for (int i = 0; i < TM; ++i) av[cur ^ 1][i] = as[kk * SA + wm0 + 32 * i + lrow];
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[cur ^ 1][j] = bs[kk * SB + wn0 + 32 * j + lrow];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] =
              __builtin_amdgcn_mfma_f32_32x32x2f32(av[cur][i], bv[cur][j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_a(buf ^ 1);
      store_b(buf ^ 1);
    }
    __syncthreads();
  }

  // ---------------- epilogue ---------------------------------------------------------------
  if (a.vec_ep) {
    // 16-byte rows through LDS (transpose32; the loop's last barrier freed the operand
    // buffers): slab rows, or the fused epilogue on output rows
    float* E = smem + wave * 1024;
    float* S = a.slab + (int64_t)split * a.split_stride;
    const int row_base = (MODE == MODE_WGRAD) ? 0 : G.tiles_begin * BM;
    const bool slab = MODE == MODE_WGRAD || a.splits > 1;
    if (do_colsum && tid < BN && n0 + tid < a.N) S[(int64_t)M * a.slab_ld + n0 + tid] = colacc;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        transpose32(E, acc[i][j], lane, [&](int row, int c4, float4 v) {
          const int m = m0 + wm0 + 32 * i + row, n = n0 + wn0 + 32 * j + 4 * c4;
          if (m >= M || n >= a.N) return;
          if (slab)
            *reinterpret_cast<float4*>(&S[(int64_t)(row_base + m) * a.slab_ld + n]) = v;
          else
            epilogue_store4<MODE>(a, 0, out_row(a, G, m), n, v);
        });
    return;
  }
  if (MODE == MODE_WGRAD || a.splits > 1) {
    // raw partial sums into this K slice's slab; rows of group g start at tiles_begin*BM
    float* S = a.slab + (int64_t)split * a.split_stride;
    const int row_base = (MODE == MODE_WGRAD) ? 0 : G.tiles_begin * BM;
    if (do_colsum && tid < BN && n0 + tid < a.N) S[(int64_t)M * a.slab_ld + n0 + tid] = colacc;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn0 + 32 * j + lrow;
      if (n >= a.N) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
          if (m < M) S[(int64_t)(row_base + m) * a.slab_ld + n] = acc[i][j][r];
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + 32 * j + lrow;
    if (n >= a.N) continue;
    float bias, scale, shift;
    column_params<MODE>(a, n, bias, scale, shift);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r0 = 0; r0 < 16; r0 += EP_GATHER<MODE>) {
        EpAux aux[EP_GATHER<MODE>];
#pragma unroll
        for (int r = r0; r < r0 + EP_GATHER<MODE>; ++r) {
          const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
          aux[r - r0] = m < M ? epilogue_aux<MODE>(a, out_row(a, G, m), n) : EpAux{0.f, 0.f};
        }
#pragma unroll
        for (int r = r0; r < r0 + EP_GATHER<MODE>; ++r) {
          const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
          if (m >= M) continue;
          epilogue_store<MODE>(a, out_row(a, G, m), n, acc[i][j][r], bias, scale, shift,
                               aux[r - r0]);
        }
      }
    }
  }
}

// ===================================================================== bf16 MFMA variant ===
// fwd / dgrad with bf16 operands (fp32 activations converted while staging, RNE; bf16 packed
// weights), fp32 accumulation: v_mfma_f32_32x32x16_bf16, 16x the f32-MFMA rate per clock.
// Same implicit-GEMM geometry, split-K and epilogues as conv_gemm_f32.  Differences:
//   * K chunk 32 (two MFMA k-steps); LDS operand images are [row][k] with k contiguous
//     (80-byte rows: the ds_read_b128 fragment reads of a wave are conflict-free);
//   * wave w stages k-octet w of every chunk: two channel quads, each with its own tap walk
//     (kc need only be a multiple of 4);
//   * packed weights are bf16 [n][k] (k contiguous, K padded to 32 per group).
constexpr int BKH = 32;                  // bf16 chunk
constexpr int SROW16 = 5;                // LDS row stride in 16-byte units (40 bf16 = 80 B)

__device__ __forceinline__ uint4 pack_bf16x8(const float4& lo, const float4& hi) {
  bf16x8 v;
  v[0] = (__bf16)lo.x;
  v[1] = (__bf16)lo.y;
  v[2] = (__bf16)lo.z;
  v[3] = (__bf16)lo.w;
  v[4] = (__bf16)hi.x;
  v[5] = (__bf16)hi.y;
  v[6] = (__bf16)hi.z;
  v[7] = (__bf16)hi.w;
  return __builtin_bit_cast(uint4, v);
}

template <int BM, int BN, int WAVES_M, int WAVES_N, int MODE>
__global__ __launch_bounds__(256, 2) void conv_gemm_bf16(GemmArgs a) {
  static_assert(MODE == MODE_FWD || MODE == MODE_DGRAD, "bf16: fwd / dgrad");
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  static_assert(TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "tile");
  constexpr int A_SLOTS = BM / 64;               // rows per lane
  constexpr int B_OCTS = BN * (BKH / 8);         // 16-byte octets of the B chunk
  constexpr int B_SLOTS = (B_OCTS + 255) / 256;
  static_assert(A_SLOTS >= 1, "BM >= 64");

  // One LDS array: both operand buffers, then the epilogue's 4 KB per-wave transpose images.
  static_assert(2 * (BM + BN) * SROW16 * 16 >= 4 * 4096, "epilogue images fit LDS");
  __shared__ uint4 smem[2 * (BM + BN) * SROW16];
  uint4 (*As)[BM * SROW16] = reinterpret_cast<uint4 (*)[BM * SROW16]>(smem);
  uint4 (*Bs)[BN * SROW16] = reinterpret_cast<uint4 (*)[BN * SROW16]>(smem + 2 * BM * SROW16);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // Stride-2 input gradients (phase groups of 4 / 2 / 2 / 1 taps, contiguous in the tile
  // space) skip the XCD remap: it would hand each XCD the tiles of one or two groups (the
  // 4-tap group's XCDs then run 1.8x the average), while block order deals every group
  // evenly over the 8 XCDs and starts the longest tiles first.
  const int wgid = a.phase ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_n = tile % a.n_tiles;
  const int tile_mg = tile / a.n_tiles;
  int gi = 0;
#pragma unroll
  for (int g = 1; g < MAX_GROUPS; ++g)
    if (g < a.ngroups && tile_mg >= a.grp[g].tiles_begin) gi = g;
  const Group& G = a.grp[gi];
  const int tile_m = tile_mg - G.tiles_begin;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int M = G.M;

  const int k_begin = split * a.k_per_split;
  const int k_end = min(G.K, k_begin + a.k_per_split);
  const int nchunks = k_end > k_begin ? (k_end - k_begin + BKH - 1) / BKH : 0;

  const rsrc_t ra_src = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rb_src = make_rsrc(a.B, a.b_bytes);

  // ---------------- A rows (same geometry as the f32 kernel) --------------------------------
  const int src_h = (MODE == MODE_DGRAD) ? a.ho : a.h;
  const int src_w = (MODE == MODE_DGRAD) ? a.wo : a.w;
  int a_off[A_SLOTS];
  uint64_t a_msk[A_SLOTS];
#pragma unroll
  for (int i = 0; i < A_SLOTS; ++i) {
    const int m = m0 + lane + 64 * i;
    const bool okm = m < M;
    const int mm = okm ? m : 0;
    int b, yb, xb;
    if (MODE == MODE_FWD) {
      const int hw = a.ho * a.wo;
      b = mm / hw;
      const int rem = mm - b * hw;
      const int oy = rem / a.wo, ox = rem - oy * a.wo;
      yb = oy * a.stride - a.pt;
      xb = ox * a.stride - a.pl;
    } else if (a.phase) {
      const int hw = G.hc * G.wc;
      b = mm / hw;
      const int rem = mm - b * hw;
      const int u = rem / G.wc, v = rem - u * G.wc;
      yb = (2 * u + G.ry + a.pt - G.r0) >> 1;
      xb = (2 * v + G.rx + a.pl - G.s0) >> 1;
    } else {
      const int hw = a.h * a.w;
      b = mm / hw;
      const int rem = mm - b * hw;
      const int iy = rem / a.w, ix = rem - iy * a.w;
      yb = iy + a.pt;
      xb = ix + a.pl;
    }
    a_off[i] = (int)(((int64_t)(b * src_h + yb) * src_w + xb) * a.lda * 4);
    uint64_t msk = 0;
    if (okm) {
      uint64_t colmask = 0;
      for (int ts = 0; ts < G.ns; ++ts) {
        const int sx = (MODE == MODE_FWD) ? xb + ts : xb - ts;
        if ((unsigned)sx < (unsigned)src_w) colmask |= (uint64_t)1 << ts;
      }
      int t = 0;
      for (int tr = 0; t < G.ntaps; ++tr, t += G.ns) {
        const int sy = (MODE == MODE_FWD) ? yb + tr : yb - tr;
        if ((unsigned)sy < (unsigned)src_h) msk |= colmask << t;
      }
      if (G.ntaps < 64) msk &= ((uint64_t)1 << G.ntaps) - 1;
    }
    a_msk[i] = msk;
  }
  // Two wave-uniform tap walkers: channel quads 2w and 2w+1 of the chunk.
  int ks_t[2], ks_tr[2], ks_ts[2], ks_ci[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k0 = k_begin + wave * 8 + 4 * h;
    ks_t[h] = k0 / a.kc;
    ks_ci[h] = k0 - ks_t[h] * a.kc;
    ks_tr[h] = ks_t[h] / G.ns;
    ks_ts[h] = ks_t[h] - ks_tr[h] * G.ns;
  }
  const int sgn = MODE == MODE_FWD ? 1 : -1;
  const int tap_step = sgn * src_w * a.lda * 4;

  float4 ra[A_SLOTS][2];
  uint4 rb[B_SLOTS];

  auto load_a = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool tap_ok = ks_t[h] < G.ntaps;
      const int koff = ks_tr[h] * tap_step + sgn * ks_ts[h] * a.lda * 4 + ks_ci[h] * 4;
#pragma unroll
      for (int i = 0; i < A_SLOTS; ++i) {
        const bool ok = tap_ok && ((a_msk[i] >> ks_t[h]) & 1);
        ra[i][h] = bload4(ra_src, ok ? (uint32_t)(a_off[i] + koff) : kOOB);
      }
    }
  };
  auto advance_a = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ks_ci[h] += BKH;
      while (ks_ci[h] >= a.kc) {
        ks_ci[h] -= a.kc;
        ++ks_t[h];
        if (++ks_ts[h] >= G.ns) {
          ks_ts[h] = 0;
          ++ks_tr[h];
        }
      }
    }
  };
  auto store_a = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_SLOTS; ++i)
      As[buf][(lane + 64 * i) * SROW16 + wave] = pack_bf16x8(ra[i][0], ra[i][1]);
  };

  // ---------------- B (packed bf16 weights [n][k]) -------------------------------------------
  uint32_t b_off[B_SLOTS];
#pragma unroll
  for (int i = 0; i < B_SLOTS; ++i) {
    const int slot = tid + 256 * i;
    const int row = slot >> 2, oct = slot & 3;
    const int n = n0 + row;
    b_off[i] = (slot < B_OCTS && n < a.nb) ? (uint32_t)((((int64_t)n * a.ldb) + G.b_off + 8 * oct) * 2)
                                           : kOOB;
  }
  int b_k = k_begin;
  auto load_b = [&]() {
#pragma unroll
    for (int i = 0; i < B_SLOTS; ++i)
      rb[i] = __builtin_bit_cast(uint4, bload4(rb_src, b_off[i] != kOOB ? b_off[i] + 2u * b_k : kOOB));
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int i = 0; i < B_SLOTS; ++i) {
      const int slot = tid + 256 * i;
      if (slot < B_OCTS) Bs[buf][(slot >> 2) * SROW16 + (slot & 3)] = rb[i];
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
      b_k += BKH;
      load_a();
      load_b();
    }
#pragma unroll
    for (int st = 0; st < BKH / 16; ++st) {
      bf16x8 av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        av[i] = __builtin_bit_cast(bf16x8, As[buf][(wm0 + 32 * i + lrow) * SROW16 + 2 * st + lk]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bv[j] = __builtin_bit_cast(bf16x8, Bs[buf][(wn0 + 32 * j + lrow) * SROW16 + 2 * st + lk]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_a(buf ^ 1);
      store_b(buf ^ 1);
    }
    __syncthreads();
  }

  // ---------------- epilogue (as conv_gemm_f32) ----------------------------------------------
  if (a.vec_ep) {
    float* E = reinterpret_cast<float*>(smem) + wave * 1024;
    float* S = a.slab + (int64_t)split * a.split_stride;
    const int row_base = G.tiles_begin * BM;
    if constexpr (!EPC_BATCH) {        // the round-2 form (one row at a time), for A/B builds
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          transpose32(E, acc[i][j], lane, [&](int row, int c4, float4 v) {
            const int m = m0 + wm0 + 32 * i + row, n = n0 + wn0 + 32 * j + 4 * c4;
            if (m >= M || n >= a.N) return;
            if (a.splits > 1)
              *reinterpret_cast<float4*>(&S[(int64_t)(row_base + m) * a.slab_ld + n]) = v;
            else
              epilogue_store4<MODE>(a, 0, out_row(a, G, m), n, v);
          });
      return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        // one 32 x 32 block's 4 rows per lane through epilogue_rows4c (the aux quads loaded
        // before the first store; row by row each load waited behind its row's guard)
        float4 vv[4];
        int64_t rows[4];
        unsigned ok = 0;
        int ncol = 0;
        transpose32(E, acc[i][j], lane, [&](int row, int c4, float4 v) {
          const int q = row >> 3;
          const int m = m0 + wm0 + 32 * i + row, n = n0 + wn0 + 32 * j + 4 * c4;
          if (a.splits > 1) {
            if (m < M && n < a.N)
              *reinterpret_cast<float4*>(&S[(int64_t)(row_base + m) * a.slab_ld + n]) = v;
            return;
          }
          rows[q] = out_row(a, G, min(m, M - 1));
          ok |= (m < M && n < a.N ? 1u : 0u) << q;
          vv[q] = v;
          ncol = n;
        });
        if (a.splits == 1) epilogue_rows4c<MODE, 4>(a, 0, rows, ok, ncol, min(ncol, a.N - 4), vv);
      }
    return;
  }
  if (a.splits > 1) {
    float* S = a.slab + (int64_t)split * a.split_stride;
    const int row_base = G.tiles_begin * BM;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn0 + 32 * j + lrow;
      if (n >= a.N) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
          if (m < M) S[(int64_t)(row_base + m) * a.slab_ld + n] = acc[i][j][r];
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + 32 * j + lrow;
    if (n >= a.N) continue;
    float bias, scale, shift;
    column_params<MODE>(a, n, bias, scale, shift);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r0 = 0; r0 < 16; r0 += EP_GATHER<MODE>) {
        EpAux aux[EP_GATHER<MODE>];
#pragma unroll
        for (int r = r0; r < r0 + EP_GATHER<MODE>; ++r) {
          const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
          aux[r - r0] = m < M ? epilogue_aux<MODE>(a, out_row(a, G, m), n) : EpAux{0.f, 0.f};
        }
#pragma unroll
        for (int r = r0; r < r0 + EP_GATHER<MODE>; ++r) {
          const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
          if (m >= M) continue;
          epilogue_store<MODE>(a, out_row(a, G, m), n, acc[i][j][r], bias, scale, shift,
                               aux[r - r0]);
        }
      }
    }
  }
}

// ---- bf16, 3x3 stride 1: 2-D output tiles with an LDS-staged input halo -----------------
// The implicit-GEMM kernels above re-read the input once per tap (9x for 3x3) through L2;
// with bf16 MFMA that traffic, not the MFMA, bounds them.  Here a workgroup owns an 8 x 16
// output-pixel tile (BM = 128 GEMM rows) and, per 32-channel chunk, stages the 10 x 18 input
// halo once (fp32 -> bf16) and takes all 9 taps' A fragments from it at shifted positions;
// the 3 taps of one kernel row share a B stage (3 x BN x 32 bf16, double-buffered).
// fwd:   out(oy, ox) += in(oy + r - pt, ox + s - pl) . W[r][s]
// dgrad: out(iy, ix) += dy(iy + pt - r, ix + pl - s) . W[r][s]^T
// GEMM K = channel chunks: a.K = chunks, a.k_per_split = chunks per K slice.
constexpr int TT_H = 8, TT_W = 16;   // wgrad halo tiles
// fwd / dgrad halo tiles (conv_tile_bf16): 4 rows x 32 px.  A wave's 32 A-fragment rows are
// then 32 consecutive halo pixels of one row: with the 80-byte pixel pitch their ds_read_b128
// 16-byte slots (5 p mod 16) are distinct in every 16-lane bank group.  An 8 x 16 tile puts
// lanes 16-31 on the next halo row (18 px later) and collides in 2 of 16 slots per group
// (SQ_LDS_BANK_CONFLICT was 40 % of the LDS cycles).
#ifndef OF_X3_TH0
#define OF_X3_TH0 8
#endif
constexpr int X3_TH0 = OF_X3_TH0;   // conv_tile_x3 BN = 128 tiles: X3_TH0 rows x 32 px
// Timing ablations of conv_tile_x3 (tools/ab_build.sh -DX3_ABL=mask; wrong results by
// design, never in the shipped build): 1 no barriers in the tap loop, 2 no B restaging,
// 4 no halo restaging, 8 one MFMA per fragment pair instead of six.
#ifndef X3_ABL
#define X3_ABL 0
#endif
// conv_tile_x3 B staging by LDS DMA (buffer_load ... lds) in the double-buffered forms
// (measured against register staging, same box: dec3.c0 fwd / dgrad -5 / -4 %, dec3.c3 fwd
// -6 %, enc.l4 -7 %; -DX3_BDMA=0 builds the register-staged form)
#ifndef X3_BDMA
#define X3_BDMA 1
#endif
// tile_x3_body's 16-byte epilogue: rows per epilogue_rows4c batch (1: one row per
// epilogue_store4, the round-2 form).  (Round 2 measured 4 at -0.3 % on the fp32 step, but
// with guarded loads that the compiler still waited for one by one; round 4 batches them
// unguarded, epilogue_rows4c.)
#ifndef X3_EPB
#define X3_EPB 1
#endif

// tile_x3_body's 4-wave split form recomputes its halo slot offsets per chunk (1) instead of
// keeping them live (0: the round-3 form, 14-16 VGPRs spilled to scratch and reloaded at every
// chunk's halo store behind a vmcnt(0)); -DX3_HREC=0 builds the old form for A/B timing
#ifndef X3_HREC
#define X3_HREC 1
#endif


// PF (of_set_tuning key 20, default 1): the MFMA loop's fragments read one sub-step ahead.
template <int BN, int WAVES_M, int WAVES_N, int MODE, int TH = OF_TF_H, int PF = 1>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N, 256 / (32 * WAVES_M * WAVES_N)) void conv_tile_bf16(GemmArgs a) {
  constexpr bool g_tile16_pf_dev = PF != 0;
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int BM = TH * TF_W, KS = 3;
  constexpr int HH = TH + KS - 1, HW = TF_W + KS - 1, HP = HH * HW;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert((NT == 256 || NT == 512) && TM >= 1 && TN >= 1, "tile");
  constexpr int HQ = HP * 8, HS = (HQ + NT - 1) / NT;        // halo quads (32 ch)
  constexpr int BOCT = KS * BN * 4, BSL = (BOCT + NT - 1) / NT; // B octets per kernel row
  // One LDS array: the halo, the B buffers, then the epilogue's 4 KB per-wave images.
  static_assert((HP + 2 * KS * BN) * SROW16 * 16 >= (NT / 64) * 4096, "epilogue images fit LDS");
  __shared__ uint4 smem[(HP + 2 * KS * BN) * SROW16];
  uint4* Ah = smem;
  uint4 (*Bs)[KS * BN * SROW16] = reinterpret_cast<uint4 (*)[KS * BN * SROW16]>(smem + HP * SROW16);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_n = tile % a.n_tiles;
  const int tile_m = tile / a.n_tiles;
  const int n0 = tile_n * BN;
  const int OH = MODE == MODE_FWD ? a.ho : a.h, OW = MODE == MODE_FWD ? a.wo : a.w;
  const int SH = MODE == MODE_FWD ? a.h : a.ho, SW = MODE == MODE_FWD ? a.w : a.wo;
  const int tiles_x = (OW + TF_W - 1) / TF_W, tiles_y = (OH + TH - 1) / TH;
  const int b = tile_m / (tiles_x * tiles_y);
  const int trem = tile_m - b * tiles_x * tiles_y;
  const int oy0 = (trem / tiles_x) * TH, ox0 = (trem % tiles_x) * TF_W;
  const int hy0 = MODE == MODE_FWD ? oy0 - a.pt : oy0 + a.pt - (KS - 1);
  const int hx0 = MODE == MODE_FWD ? ox0 - a.pl : ox0 + a.pl - (KS - 1);
  const int c_begin = split * a.k_per_split;
  const int c_end = min(a.K, c_begin + a.k_per_split);
  const int steps = c_end > c_begin ? (c_end - c_begin) * KS : 0;

  const rsrc_t ra_src = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rb_src = make_rsrc(a.B, a.b_bytes);

  // ---- halo slots: quad (q & 7) of halo pixel (q >> 3)
  int h_off[HS];
  unsigned h_ok = 0;
  const int hcq = tid & 7;
#pragma unroll
  for (int j = 0; j < HS; ++j) {
    const int q = tid + NT * j;
    const int hp = q >> 3;
    const int sy = hy0 + hp / HW, sx = hx0 + hp % HW;
    const bool ok = q < HQ && (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW;
    h_off[j] = ok ? (((b * SH + sy) * SW + sx) * a.lda + 4 * hcq) * 4 : 0;
    h_ok |= (ok ? 1u : 0u) << j;
  }
  float4 hv[HS];
  auto load_halo = [&](int c) {
    const bool cok = 32 * c + 4 * hcq < a.kc;
#pragma unroll
    for (int j = 0; j < HS; ++j)
      hv[j] = bload4(ra_src, cok && ((h_ok >> j) & 1) ? (uint32_t)(h_off[j] + 128 * c) : kOOB);
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int j = 0; j < HS; ++j) {
      const int q = tid + NT * j;
      if (q < HQ) {
        bf16x8 t;   // low 4 used: one quad -> 8 bytes
        const float4 v = hv[j];
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 u;
        u[0] = (__bf16)v.x;
        u[1] = (__bf16)v.y;
        u[2] = (__bf16)v.z;
        u[3] = (__bf16)v.w;
        (void)t;
        *reinterpret_cast<bf16x4*>(reinterpret_cast<char*>(Ah) + (q >> 3) * (SROW16 * 16) +
                                   8 * (q & 7)) = u;
      }
    }
  };
  // ---- B slots: (tap s of the kernel row, weight row, octet)
  uint4 rb[BSL];
  auto load_b = [&](int c, int r) {
#pragma unroll
    for (int j = 0; j < BSL; ++j) {
      const int o = tid + NT * j;
      const int s = o / (BN * 4), rem = o - s * (BN * 4);
      const int n = n0 + (rem >> 2), oct = rem & 3;
      const bool ok = o < BOCT && n < a.nb;
      const int k = (r * KS + s) * a.kc + 32 * c + 8 * oct;
      rb[j] = __builtin_bit_cast(uint4,
                                 bload4(rb_src, ok ? (uint32_t)(((int64_t)n * a.ldb + k) * 2) : kOOB));
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int j = 0; j < BSL; ++j) {
      const int o = tid + NT * j;
      if (o < BOCT) {
        const int s = o / (BN * 4), rem = o - s * (BN * 4);
        Bs[buf][(s * BN + (rem >> 2)) * SROW16 + (rem & 3)] = rb[j];
      }
    }
  };

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
  int a_hp[TM];   // halo pixel of this lane's A row at tap (0, 0)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = wm0 + 32 * i + lrow;
    const int ty = m / TF_W, tx = m % TF_W;
    a_hp[i] = MODE == MODE_FWD ? ty * HW + tx : (ty + KS - 1) * HW + tx + KS - 1;
  }

  if (steps > 0) {
    load_halo(c_begin);
    load_b(c_begin, 0);
    store_halo();
    store_b(0);
  }
  __syncthreads();
  // The next chunk's halo is fetched at the first step of the current chunk and stored after
  // its last step (KS steps of latency cover); B one step ahead into the other buffer.  Only
  // the halo store needs the pre-store barrier: the B buffer written at step q was last read
  // at step q-1, which every wave finished before step q-1's closing barrier.
  for (int q = 0; q < steps; ++q) {
    const int r = q % KS, buf = q & 1;
    const bool more = q + 1 < steps;
    const int nq = q + 1;
    const int nc = c_begin + nq / KS, nr = nq % KS;
    if (more) load_b(nc, nr);
    if (r == 0 && q + KS < steps) load_halo(c_begin + q / KS + 1);
    // sub-step k = (tap s, K half st): its TM A and TN B fragments
    auto frags = [&](int k, bf16x8 (&av)[TM], bf16x8 (&bv)[TN]) {
      const int s = k >> 1, st = k & 1;
      const int dh = MODE == MODE_FWD ? r * HW + s : -(r * HW + s);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        av[i] = __builtin_bit_cast(bf16x8, Ah[(a_hp[i] + dh) * SROW16 + 2 * st + lk]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bv[j] = __builtin_bit_cast(
            bf16x8, Bs[buf][(s * BN + wn0 + 32 * j + lrow) * SROW16 + 2 * st + lk]);
    };
    if (g_tile16_pf_dev) {
      // fragments one sub-step ahead of their MFMAs (the scheduler otherwise sinks each read
      // to its first MFMA, a ds_read latency exposed per TM x TN MFMAs); sched_barrier fences
      bf16x8 av[2][TM], bv[2][TN];
      frags(0, av[0], bv[0]);
#pragma unroll
      for (int k = 0; k < 2 * KS; ++k) {
        const int cur = k & 1;
        if (k + 1 < 2 * KS) frags(k + 1, av[cur ^ 1], bv[cur ^ 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[cur][i], bv[cur][j], acc[i][j],
                                                                0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 2 * KS; ++k) {
        bf16x8 av[TM], bv[TN];
        frags(k, av, bv);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more && nr == 0) __syncthreads();           // all reads of this chunk's halo done
    if (more) {
      store_b(buf ^ 1);
      if (nr == 0) store_halo();
    }
    __syncthreads();
  }

  // ---- epilogue
  const int64_t img = (int64_t)b * OH * OW;
  if (a.vec_ep && !EPC_BATCH) {   // the round-2 form (one row at a time), for A/B builds
    float* E = reinterpret_cast<float*>(smem) + wave * 1024;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        transpose32(E, acc[i][j], lane, [&](int row, int c4, float4 v) {
          const int mt = wm0 + 32 * i + row, n = n0 + wn0 + 32 * j + 4 * c4;
          const int oy = oy0 + mt / TF_W, ox = ox0 + mt % TF_W;
          if (oy < OH && ox < OW && n < a.N)
            epilogue_store4<MODE>(a, split, img + (int64_t)oy * OW + ox, n, v);
        });
    return;
  }
  if (MODE == MODE_DGRAD && a.vec_ep && a.bnp != nullptr) {
    // the same with the BN partial sums of the layer whose output is act_src (one K slice,
    // host-checked): per lane its column quads' sums over its rows, then over the lanes of a
    // column quad (shuffles), the WAVES_M waves of a column block in wave order (LDS), one
    // partial row per output tile and channel -- fixed order, no atomics
    float* E = reinterpret_cast<float*>(smem) + wave * 1024;
    const int c4 = lane & 7;
    float4 bsb[TN], bsg[TN], bt[TN], ig[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bsb[j] = bsg[j] = bt[j] = ig[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      const int n = n0 + wn0 + 32 * j + 4 * c4;
      if (n < a.N) {
        bt[j] = *reinterpret_cast<const float4*>(&a.bnp_b[n]);
        const float4 gm = *reinterpret_cast<const float4*>(&a.bnp_g[n]);
        ig[j] = make_float4(1.f / gm.x, 1.f / gm.y, 1.f / gm.z, 1.f / gm.w);
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float4 vv[4];
        int64_t rows[4];
        unsigned ok = 0;
        int ncol = 0;
        transpose32(E, acc[i][j], lane, [&](int row, int c4r, float4 v) {
          const int q = row >> 3;
          const int mt = wm0 + 32 * i + row, n = n0 + wn0 + 32 * j + 4 * c4r;
          const int oy = oy0 + mt / TF_W, ox = ox0 + mt % TF_W;
          rows[q] = img + (int64_t)min(oy, OH - 1) * OW + min(ox, OW - 1);
          ok |= (oy < OH && ox < OW && n < a.N ? 1u : 0u) << q;
          vv[q] = v;
          ncol = n;
        });
        dgrad_rows4c_bnp<4>(a, rows, ok, ncol, min(ncol, a.N - 4), vv, bt[j], ig[j], bsb[j], bsg[j]);
      }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        bsb[j].x += __shfl_xor(bsb[j].x, o, 64), bsb[j].y += __shfl_xor(bsb[j].y, o, 64);
        bsb[j].z += __shfl_xor(bsb[j].z, o, 64), bsb[j].w += __shfl_xor(bsb[j].w, o, 64);
        bsg[j].x += __shfl_xor(bsg[j].x, o, 64), bsg[j].y += __shfl_xor(bsg[j].y, o, 64);
        bsg[j].z += __shfl_xor(bsg[j].z, o, 64), bsg[j].w += __shfl_xor(bsg[j].w, o, 64);
      }
    __syncthreads();                      // every wave's E image reads are done
    float4* red = reinterpret_cast<float4*>(smem);   // [2][WAVES_M][BN / 4]
    const int wmi = wave / WAVES_N;
    if (lane < 8) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int lq = (wn0 + 32 * j) / 4 + c4;
        red[wmi * (BN / 4) + lq] = bsb[j];
        red[(WAVES_M + wmi) * (BN / 4) + lq] = bsg[j];
      }
    }
    __syncthreads();
    if (tid < BN / 4 && n0 + 4 * tid < a.N) {
      float4 sb = red[tid], sg = red[WAVES_M * (BN / 4) + tid];
      for (int w2 = 1; w2 < WAVES_M; ++w2) {
        add4(sb, red[w2 * (BN / 4) + tid]);
        add4(sg, red[(WAVES_M + w2) * (BN / 4) + tid]);
      }
      float* prow = a.bnp + (int64_t)tile_m * 2 * a.N + n0 + 4 * tid;
      *reinterpret_cast<float4*>(prow) = sb;
      *reinterpret_cast<float4*>(prow + a.N) = sg;
    }
    return;
  }
  if (a.vec_ep) {   // 16-byte rows through LDS (the loop's last barrier freed the images)
    float* E = reinterpret_cast<float*>(smem) + wave * 1024;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        // the block's 4 rows per lane through epilogue_rows4: their residual / activation-
        // source quads are loaded before the first store (one row at a time, each row's load
        // sat behind a branch and waited: 4 TM TN serial memory round trips per tile)
        float4 vv[4];
        int64_t rows[4];
        unsigned ok = 0;
        int ncol = 0;
        transpose32(E, acc[i][j], lane, [&](int row, int c4, float4 v) {
          const int q = row >> 3;
          const int mt = wm0 + 32 * i + row, n = n0 + wn0 + 32 * j + 4 * c4;
          const int oy = oy0 + mt / TF_W, ox = ox0 + mt % TF_W;
          rows[q] = img + (int64_t)min(oy, OH - 1) * OW + min(ox, OW - 1);
          ok |= (oy < OH && ox < OW && n < a.N ? 1u : 0u) << q;
          vv[q] = v;
          ncol = n;
        });
        epilogue_rows4c<MODE, 4>(a, split, rows, ok, ncol, min(ncol, a.N - 4), vv);
      }
    return;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + 32 * j + lrow;
    if (n >= a.N) continue;
    float bias = 0.f, scale = 1.f, shift = 0.f;
    if (a.splits == 1) column_params<MODE>(a, n, bias, scale, shift);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      EpAux aux[16];
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int m = wm0 + 32 * i + (rr & 3) + 8 * (rr >> 2) + 4 * lk;
        const int oy = oy0 + m / TF_W, ox = ox0 + m % TF_W;
        aux[rr] = a.splits == 1 && oy < OH && ox < OW
                      ? epilogue_aux<MODE>(a, img + (int64_t)oy * OW + ox, n) : EpAux{0.f, 0.f};
      }
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int m = wm0 + 32 * i + (rr & 3) + 8 * (rr >> 2) + 4 * lk;
        const int oy = oy0 + m / TF_W, ox = ox0 + m % TF_W;
        if (oy >= OH || ox >= OW) continue;
        const int64_t row = img + (int64_t)oy * OW + ox;
        if (a.splits > 1)
          a.slab[(int64_t)split * a.split_stride + row * a.slab_ld + n] = acc[i][j][rr];
        else
          epilogue_store<MODE>(a, row, n, acc[i][j][rr], bias, scale, shift, aux[rr]);
      }
    }
  }
}

// ---- fp32 on bf16 MFMA by a three-term split, 3x3 stride 1 -------------------------------
// Every fp32 operand is cut exactly into three bf16 terms, x = hi + mid + lo (8 + 8 + 8
// significand bits: hi = x with the low 16 bits cleared, mid = the same of x - hi,
// lo = x - hi - mid), and a.b is accumulated as the six products whose magnitude can reach
// 2^-16 |a||b|: hi.hi, hi.mid, mid.hi, mid.mid, hi.lo, lo.hi.  bf16 x bf16 products are
// exact, the MFMA accumulates in fp32, and the dropped terms (mid.lo, lo.mid, lo.lo) are
// below 2^-23 |a||b| together: the error per product is that of one fp32 rounding.  Six
// v_mfma_f32_32x32x16_bf16 do the work of 8 v_mfma_f32_32x32x2_f32 at 16/6 of their peak.
// Structure as conv_tile_bf16 (4 x 32 output tiles, LDS halo, 9 taps per chunk) with three
// halo planes and B staged one tap per step (3 planes x BN rows x 32 channels) to fit LDS;
// the packed weights are three bf16 planes a.b_plane elements apart.
__device__ __forceinline__ void split3x4(const float4& v, uint2& h, uint2& m, uint2& l) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  uint32_t hb[4], mb[4], lb[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hb[e] = __float_as_uint(x[e]) & 0xffff0000u;
    const float r = x[e] - __uint_as_float(hb[e]);
    mb[e] = __float_as_uint(r) & 0xffff0000u;
    lb[e] = __float_as_uint(r - __uint_as_float(mb[e]));   // <= 8 significant bits: exact
  }
  // upper halves of (e0, e1) -> one dword, element 0 low: one v_perm_b32 per pair
  auto hi2 = [](uint32_t e0, uint32_t e1) { return __builtin_amdgcn_perm(e1, e0, 0x07060302u); };
  h = make_uint2(hi2(hb[0], hb[1]), hi2(hb[2], hb[3]));
  m = make_uint2(hi2(mb[0], mb[1]), hi2(mb[2], mb[3]));
  l = make_uint2(hi2(lb[0], lb[1]), hi2(lb[2], lb[3]));
}

// NB = B buffers: 2 (double-buffered, one barrier per tap) or 1 (TH = 4: 64 KB of LDS, so two
// 4-wave workgroups share a CU; two barriers per tap).
// LDS images (halo pixels, B rows) are rows of 32 bf16 = four 16-byte octets, unpadded; octet
// o of row p sits in slot o ^ x3_sw(p).  A v_mfma_f32_16x16x32_bf16 fragment read (lanes
// l & 15 = 16 consecutive rows from ANY start, lanes l >> 4 = the octet) then touches 16
// distinct 16-byte bank slots in each ds_read_b128 lane group: rows 4 apart share a slot
// base, and of the four such rows in a group two read octet q and two octet q ^ 1; the
// swizzle alternates with bit 2 of the row, so the four land on q, q ^ 2, q ^ 1, q ^ 3.  (The
// 80-byte padded rows that suit the 32 x 32 layout leave 3 of 16 slots 2-way in every group.)
// The halo-tiled 3x3 stride-1 body shared by the fp32 split kernel (NP = 3 planes: hi / mid /
// lo, six MFMAs per fragment pair) and the bf16 one (NP = 1: activations rounded to bf16 RNE
// while staged, the bf16 packed weights, one MFMA per fragment pair).
template <int BN, int WAVES_M, int WAVES_N, int MODE, int TH, int NB, int NP>
__device__ __forceinline__ void tile_x3_body(const GemmArgs& a) {
  constexpr int BM = TH * TF_W, KS = 3;
  static_assert(NP == 1 || NP == 3, "planes");
  constexpr int HH = TH + KS - 1, HW = TF_W + KS - 1, HP = HH * HW;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int SM = WM / 16, SN = WN / 16;                    // 16 x 16 MFMA tiles per wave
  constexpr int NT = 64 * WAVES_M * WAVES_N;                   // 4-12 waves
  static_assert(NT % 64 == 0 && NT <= 1024 && WM % 16 == 0 && WN % 16 == 0 && SM >= 1 && SN >= 1,
                "tile");
  constexpr int HQ = HP * 8, HS = (HQ + NT - 1) / NT;          // halo quads (32 ch)
  constexpr int BOCT = NP * BN * 4, BSL = (BOCT + NT - 1) / NT; // B octets per tap
  // One LDS array: the halo planes, the B buffers, and after the main loop the epilogue's
  // per-wave transpose images (WM rows x 16 EJ floats, EJ column blocks per pass; unpadded:
  // rows 4 apart share a bank-slot base, and the float4 reads of a ds_read_b128 lane group
  // (4 EJ lanes per row) cover 16 distinct slots; the 2-way ds_write_b32 conflict is free).
  constexpr int AH_U4 = NP * HP * 4, BS_U4 = NB * NP * BN * 4;
  // (one plane can leave the loop's images smaller than one 16-column epilogue pass: the
  // array is then sized for that pass)
  constexpr int EP1_U4 = (NT / 64) * WM * 16 * 4 / 16;
  constexpr int SM_U4 = AH_U4 + BS_U4 > EP1_U4 ? AH_U4 + BS_U4 : EP1_U4;
  constexpr int LDS_B = SM_U4 * 16;
  constexpr int EJ = (NT / 64) * WM * 16 * SN * 4 <= LDS_B ? SN
                     : (NT / 64) * WM * 8 * SN * 4 <= LDS_B ? SN / 2 : 1;
  constexpr int EPW = 16 * EJ;
  static_assert(SN % EJ == 0 && (NT / 64) * WM * EPW * 4 <= LDS_B, "epilogue image fits LDS");
  __shared__ uint4 smem[SM_U4];
  uint4* Ah = smem;                      // [plane][halo pixel][4 octets]
  uint4* Bs = smem + AH_U4;              // [buf][plane][BN rows][4 octets]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_n = tile % a.n_tiles;
  const int tile_m = tile / a.n_tiles;
  const int n0 = tile_n * BN;
  const int OH = MODE == MODE_FWD ? a.ho : a.h, OW = MODE == MODE_FWD ? a.wo : a.w;
  const int SH = MODE == MODE_FWD ? a.h : a.ho, SW = MODE == MODE_FWD ? a.w : a.wo;
  const int tiles_x = (OW + TF_W - 1) / TF_W, tiles_y = (OH + TH - 1) / TH;
  const int b = tile_m / (tiles_x * tiles_y);
  const int trem = tile_m - b * tiles_x * tiles_y;
  const int oy0 = (trem / tiles_x) * TH, ox0 = (trem % tiles_x) * TF_W;
  const int hy0 = MODE == MODE_FWD ? oy0 - a.pt : oy0 + a.pt - (KS - 1);
  const int hx0 = MODE == MODE_FWD ? ox0 - a.pl : ox0 + a.pl - (KS - 1);
  const int c_begin = split * a.k_per_split;
  const int c_end = min(a.K, c_begin + a.k_per_split);

  const rsrc_t ra_src = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rb_src = make_rsrc(a.B, a.b_bytes);

  // ---- halo slots: quad (q & 7) of halo pixel (q >> 3)
  float4 hv[HS];
  // HREC (the 4-wave split form): the slot offsets recomputed per chunk from a lane index made
  // opaque there, instead of HS offsets live through the main loop (that form spilled)
  constexpr bool HREC = X3_HREC && NT == 256 && NP == 3;
  int h_off[HREC ? 1 : HS];
  unsigned h_ok = 0;
  const int hcq = tid & 7;
  auto halo_slot = [&](int t, int j, bool& ok) {
    const int q = t + NT * j;
    const int hp = q >> 3;
    const int sy = hy0 + hp / HW, sx = hx0 + hp % HW;
    ok = q < HQ && (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW;
    return ok ? (((b * SH + sy) * SW + sx) * a.lda + 4 * (t & 7)) * 4 : 0;
  };
  if constexpr (!HREC) {
#pragma unroll
    for (int j = 0; j < HS; ++j) {
      bool ok;
      h_off[j] = halo_slot(tid, j, ok);
      h_ok |= (ok ? 1u : 0u) << j;
    }
  }
  auto load_halo = [&](int c) {
    const bool cok = 32 * c + 4 * hcq < a.kc;
    if constexpr (HREC) {
      int t = tid;
      asm volatile("" : "+v"(t));
#pragma unroll
      for (int j = 0; j < HS; ++j) {
        bool ok;
        const int off = halo_slot(t, j, ok);
        hv[j] = bload4(ra_src, cok && ok ? (uint32_t)(off + 128 * c) : kOOB);
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < HS; ++jj)
        hv[jj] = bload4(ra_src, cok && ((h_ok >> jj) & 1) ? (uint32_t)(h_off[jj] + 128 * c) : kOOB);
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int j = 0; j < HS; ++j) {
      const int q = tid + NT * j;
      if (q < HQ) {
        const int hp = q >> 3;
        const int off = hp * 64 + ((((q & 7) >> 1) ^ x3_sw(hp)) << 4) + 8 * (q & 1);
        char* base = reinterpret_cast<char*>(Ah);
        if constexpr (NP == 1) {
          *reinterpret_cast<uint2*>(base + off) = pack_bf16x4(hv[j]);
        } else {
          uint2 h, m, l;
          split3x4(hv[j], h, m, l);
          *reinterpret_cast<uint2*>(base + off) = h;
          *reinterpret_cast<uint2*>(base + HP * 64 + off) = m;
          *reinterpret_cast<uint2*>(base + 2 * HP * 64 + off) = l;
        }
      }
    }
  };
  // ---- B slots: (plane, weight row, octet) of one tap; the (tap, chunk) part of the offset
  // is uniform and rides in the buffer load's scalar offset.
  uint32_t b_off[BSL];
  int b_lds[BSL];
#pragma unroll
  for (int j = 0; j < BSL; ++j) {
    const int o = tid + NT * j;
    const int p = o / (BN * 4), rem = o - p * (BN * 4);
    const int row = rem >> 2, oct = rem & 3;
    const int n = n0 + row;
    const bool ok = o < BOCT && n < a.nb;
    b_off[j] = ok ? (uint32_t)(((int64_t)p * a.b_plane + (int64_t)n * a.ldb + 8 * oct) * 2) : kOOB;
    b_lds[j] = o < BOCT ? (p * BN + row) * 4 + (oct ^ x3_sw(row)) : -1;
  }
  uint4 rb[BSL];
  auto load_b = [&](int c, int t) {
    const int so = (t * a.kc + 32 * c) * 2;
#pragma unroll
    for (int j = 0; j < BSL; ++j)
      rb[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rb_src, b_off[j], so, 0));
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int j = 0; j < BSL; ++j)
      if (BOCT % NT == 0 || b_lds[j] >= 0) Bs[buf * NP * BN * 4 + b_lds[j]] = rb[j];
  };
  // X3_BDMA (double-buffered forms): B goes global -> LDS by buffer_load ... lds, no VGPR
  // staging and no ds_write: one wave-instruction fills 16 rows x 64 bytes (lane-linear), so
  // lane L loads octet (L & 3) ^ x3_sw(L >> 2) of its row to keep the swizzled image.
  constexpr bool BDMA = X3_BDMA && NB == 2;
  constexpr int NW = NT / 64, BDI = NP * BN / 16, BDW = (BDI + NW - 1) / NW;
  uint32_t bd_off[BDW];
  int bd_lds[BDW];
#pragma unroll
  for (int k = 0; k < BDW; ++k) {
    const int g = wave + NW * k;
    const int p = g / (BN / 16), rbk = g % (BN / 16);
    const int n = rbk * 16 + (lane >> 2), o = (lane & 3) ^ x3_sw(lane >> 2);
    bd_off[k] = g < BDI && n0 + n < a.nb
                    ? (uint32_t)(((int64_t)p * a.b_plane + (int64_t)(n0 + n) * a.ldb + 8 * o) * 2)
                    : kOOB;
    bd_lds[k] = g < BDI ? (p * BN + rbk * 16) * 4 : -1;
  }
  auto dma_b = [&](int c, int t, int buf) {
    const int so = (t * a.kc + 32 * c) * 2;
#pragma unroll
    for (int k = 0; k < BDW; ++k)
      if (BDI % NW == 0 || bd_lds[k] >= 0)
        dma16_to_lds(rb_src, Bs + buf * NP * BN * 4 + bd_lds[k], bd_off[k], so);
  };

  f32x4 acc4[SM][SN];
#pragma unroll
  for (int i = 0; i < SM; ++i)
#pragma unroll
    for (int j = 0; j < SN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc4[i][j][r] = 0.f;
  const int wm0 = (wave / WAVES_N) * WM;
  const int wn0 = (wave % WAVES_N) * WN;
  const int l16 = lane & 15, lq = lane >> 4;
  int a_hp16[SM];        // halo pixel of this lane's A row at tap (0, 0)
#pragma unroll
  for (int i = 0; i < SM; ++i) {
    const int m = wm0 + 16 * i + l16;
    const int ty = m / TF_W, tx = m % TF_W;
    a_hp16[i] = MODE == MODE_FWD ? ty * HW + tx : (ty + KS - 1) * HW + tx + KS - 1;
  }
  // B fragment rows wn0 + 16 j + l16: the swizzle depends on l16 only
  const int b_frag = (wn0 + l16) * 4 + (lq ^ x3_sw(l16));

  if (c_end > c_begin) {
    load_halo(c_begin);
    if constexpr (BDMA) dma_b(c_begin, 0, 0);
    else load_b(c_begin, 0);
    store_halo();
    if constexpr (!BDMA) store_b(0);
  }
  if constexpr (BDMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // Chunk loop with the 9 taps unrolled (fragment offsets are immediates).  Step (chunk, tap)
  // reads B buffer (chunk + tap) & 1 (9 steps per chunk) and fetches the next step's B; the
  // next chunk's halo is fetched at tap 0 and stored after tap 8.
  for (int c = c_begin; c < c_end; ++c) {
    const int cc = c - c_begin;
    const bool more_c = c + 1 < c_end;
    if (more_c && !(X3_ABL & 4)) load_halo(c + 1);
#pragma unroll
    for (int t = 0; t < KS * KS; ++t) {
      const int buf = NB == 2 ? (cc + t) & 1 : 0;
      const bool more = t + 1 < KS * KS || more_c;
      if (more && !(X3_ABL & 2)) {
        if constexpr (BDMA) dma_b(t + 1 < KS * KS ? c : c + 1, t + 1 < KS * KS ? t + 1 : 0, buf ^ 1);
        else load_b(t + 1 < KS * KS ? c : c + 1, t + 1 < KS * KS ? t + 1 : 0);
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of this step's MFMAs
      const int r = t / KS, s = t % KS;
      const int dh = MODE == MODE_FWD ? r * HW + s : -(r * HW + s);
      bf16x8 av[NP][SM], bv[NP][SN];
#pragma unroll
      for (int i = 0; i < SM; ++i) {
        const int px = a_hp16[i] + dh;
        const int ai = px * 4 + (lq ^ x3_sw(px));
#pragma unroll
        for (int p = 0; p < NP; ++p) av[p][i] = __builtin_bit_cast(bf16x8, Ah[p * HP * 4 + ai]);
      }
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int j = 0; j < SN; ++j)
          bv[p][j] = __builtin_bit_cast(bf16x8, Bs[(buf * NP + p) * BN * 4 + 64 * j + b_frag]);
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SN; ++j) {
          f32x4 x = acc4[i][j];
          if constexpr (NP == 1) {
            acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], x, 0, 0, 0);
            continue;
          } else {
          if (X3_ABL & 8) {      // ablation: one product (the MFMA count of a bf16 conv)
            asm volatile("" ::"v"(av[1][i]), "v"(av[2][i]), "v"(bv[1][j]), "v"(bv[2][j]));
            acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], x, 0, 0, 0);
            continue;
          }
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[2][i], bv[0][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[2][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1][i], bv[1][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1][i], bv[0][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[1][j], x, 0, 0, 0);
          acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], x, 0, 0, 0);
          }
        }
      __builtin_amdgcn_sched_barrier(0);   // the stores wait for the prefetch: after the MFMAs
      // single B buffer: every wave must be done with it; double: only with the halo
      if (!(X3_ABL & 1) && (NB == 1 ? more : (t + 1 == KS * KS && more_c))) __syncthreads();
      if (more) {
        if (!(X3_ABL & 2) && !BDMA) store_b(NB == 2 ? buf ^ 1 : 0);
        if (t + 1 == KS * KS && more_c && !(X3_ABL & 4)) store_halo();
      }
      if constexpr (BDMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // own B DMA landed
      if (!(X3_ABL & 1)) __syncthreads();
    }
  }

  // ---- epilogue (16 x 16 C layout: column = lane & 15, rows 4 (lane >> 4) + r)
  const int64_t img = (int64_t)b * OH * OW;
  if constexpr (X3_ABL & 16) {   // ablation: one store per lane instead of 4 SM SN
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j) v += acc4[i][j][0] + acc4[i][j][1] + acc4[i][j][2] + acc4[i][j][3];
    a.C[(img + (int64_t)oy0 * OW + ox0) * a.ldc + (n0 + wn0 + (lane & 31)) % a.N] = v;
    return;
  }
  if constexpr (MODE == MODE_FWD && SM % 2 == 0 &&
                (NT / 64) * (WM / 2) * (WN * 4 + 32) <= LDS_B &&
                ((WM / 2) * (WN / 4)) % 64 == 0) {
    if (a.direct16) {      // fp32 forward, one output, no residual / z: conv_dev.h
      direct_fwd_f32<SM, SN, WM, WN, TF_W>(
          a, acc4, reinterpret_cast<char*>(smem) + wave * (WM / 2) * (WN * 4 + 32), lane, wm0,
          wn0, n0, oy0, ox0, OH, OW, img);
      return;
    }
  }
  // (not the 4-wave forms: at 256 VGPRs already, the chunk registers raised their spills)
  if constexpr (MODE == MODE_DGRAD && NT >= 512 && SM % 2 == 0 &&
                (NT / 64) * (WM / 2) * (WN * 4 + 32) <= LDS_B &&
                ((WM / 2) * (WN / 4)) % 64 == 0) {
    if (a.direct16) {      // fp32 input gradient, one K slice: conv_dev.h
      direct_dgrad_f32<SM, SN, WM, WN, TF_W>(
          a, acc4, reinterpret_cast<char*>(smem) + wave * (WM / 2) * (WN * 4 + 32), lane, wm0,
          wn0, n0, oy0, ox0, OH, OW, img);
      return;
    }
  }
  if (a.vec_ep) {
    // The wave's accumulator block goes through a private LDS image, EJ column blocks per
    // pass (every wave passed the main loop's last barrier after its last halo / B read), and
    // comes back as rows of float4: 16-byte loads and stores, 4 EJ lanes per pixel row (the
    // MFMA layout holds 4 rows of one column per lane: 4-byte accesses on 64-byte segments).
    float* E = reinterpret_cast<float*>(smem) + wave * WM * EPW;
    constexpr int LPR = 4 * EJ, RPI = 64 / LPR;            // lanes per row, rows per pass
    const int c4 = lane % LPR, rr = lane / LPR;
    // fused BN partial sums (a.bnp: input gradient, one K slice, the host checked)
    constexpr int NPASS = SN / EJ;
    const bool bnp = MODE == MODE_DGRAD && a.bnp != nullptr;
    float4 bsb[NPASS], bsg[NPASS];
#pragma unroll
    for (int p = 0; p < NPASS; ++p) bsb[p] = bsg[p] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int jp = 0; jp < SN; jp += EJ) {
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < EJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            E[(16 * i + 4 * lq + r) * EPW + 16 * j + l16] = acc4[i][jp + j][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int n = n0 + wn0 + 16 * jp + 4 * c4;
      if constexpr (X3_EPB > 1 && (WM / RPI) % X3_EPB == 0) {
        // rows in batches of X3_EPB (epilogue_rows4: the aux loads ahead of the stores)
#pragma unroll
        for (int q0 = 0; q0 < WM / RPI; q0 += X3_EPB) {
          float4 v[X3_EPB];
          int64_t row[X3_EPB];
          unsigned ok = 0;
#pragma unroll
          for (int g = 0; g < X3_EPB; ++g) {
            const int m = (q0 + g) * RPI + rr;
            v[g] = *reinterpret_cast<const float4*>(&E[m * EPW + 4 * c4]);
            const int mt = wm0 + m;
            const int oy = oy0 + mt / TF_W, ox = ox0 + mt % TF_W;
            row[g] = img + (int64_t)min(oy, OH - 1) * OW + min(ox, OW - 1);   // clamped: loads
            ok |= (oy < OH && ox < OW && n < a.N ? 1u : 0u) << g;
          }
          epilogue_rows4c<MODE, X3_EPB>(a, split, row, ok, n, min(n, a.N - 4), v);
        }
      } else if (MODE == MODE_DGRAD && bnp) {
        float4 bt = make_float4(0.f, 0.f, 0.f, 0.f), ig = bt;
        if (n < a.N) {
          bt = *reinterpret_cast<const float4*>(&a.bnp_b[n]);
          const float4 gm = *reinterpret_cast<const float4*>(&a.bnp_g[n]);
          ig = make_float4(1.f / gm.x, 1.f / gm.y, 1.f / gm.z, 1.f / gm.w);
        }
#pragma unroll
        for (int q = 0; q < WM / RPI; ++q) {
          const int m = q * RPI + rr;
          const float4 v = *reinterpret_cast<const float4*>(&E[m * EPW + 4 * c4]);
          const int mt = wm0 + m;
          const int oy = oy0 + mt / TF_W, ox = ox0 + mt % TF_W;
          if (oy < OH && ox < OW && n < a.N)
            dgrad_store4_bnp(a, img + (int64_t)oy * OW + ox, n, v, bt, ig, bsb[jp / EJ],
                             bsg[jp / EJ]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < WM / RPI; ++q) {
          const int m = q * RPI + rr;
          const float4 v = *reinterpret_cast<const float4*>(&E[m * EPW + 4 * c4]);
          const int mt = wm0 + m;
          const int oy = oy0 + mt / TF_W, ox = ox0 + mt % TF_W;
          if (oy < OH && ox < OW && n < a.N)
            epilogue_store4<MODE>(a, split, img + (int64_t)oy * OW + ox, n, v);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (MODE == MODE_DGRAD && bnp) {
      // the wave's rows (lanes c4 + LPR rr), then the WAVES_M waves of a column block in wave
      // order through LDS, then one partial row per tile and channel: fixed order, no atomics
      constexpr int NWM = (NT / 64) / WAVES_N;
#pragma unroll
      for (int p = 0; p < NPASS; ++p)
#pragma unroll
        for (int o = LPR; o < 64; o <<= 1) {
          bsb[p].x += __shfl_xor(bsb[p].x, o, 64), bsb[p].y += __shfl_xor(bsb[p].y, o, 64);
          bsb[p].z += __shfl_xor(bsb[p].z, o, 64), bsb[p].w += __shfl_xor(bsb[p].w, o, 64);
          bsg[p].x += __shfl_xor(bsg[p].x, o, 64), bsg[p].y += __shfl_xor(bsg[p].y, o, 64);
          bsg[p].z += __shfl_xor(bsg[p].z, o, 64), bsg[p].w += __shfl_xor(bsg[p].w, o, 64);
        }
      __syncthreads();                    // every wave's E image reads are done
      float4* red = reinterpret_cast<float4*>(smem);       // [2][NWM][BN / 4]
      const int wmi = wave / WAVES_N;
      if (rr == 0) {
#pragma unroll
        for (int p = 0; p < NPASS; ++p) {
          const int lq = (wn0 + 16 * EJ * p) / 4 + c4;
          red[wmi * (BN / 4) + lq] = bsb[p];
          red[(NWM + wmi) * (BN / 4) + lq] = bsg[p];
        }
      }
      __syncthreads();
      const int tid = threadIdx.x;
      if (tid < BN / 4 && n0 + 4 * tid < a.N) {
        float4 sb = red[tid], sg = red[NWM * (BN / 4) + tid];
        for (int w2 = 1; w2 < NWM; ++w2) {
          add4(sb, red[w2 * (BN / 4) + tid]);
          add4(sg, red[(NWM + w2) * (BN / 4) + tid]);
        }
        float* prow = a.bnp + (int64_t)tile_m * 2 * a.N + n0 + 4 * tid;
        *reinterpret_cast<float4*>(prow) = sb;
        *reinterpret_cast<float4*>(prow + a.N) = sg;
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < SN; ++j) {
    const int n = n0 + wn0 + 16 * j + l16;
    if (n >= a.N) continue;
    float bias = 0.f, scale = 1.f, shift = 0.f;
    if (a.splits == 1) column_params<MODE>(a, n, bias, scale, shift);
    EpAux aux[SM * 4];
#pragma unroll
    for (int q = 0; q < SM * 4; ++q) {
      const int m = wm0 + 16 * (q >> 2) + 4 * lq + (q & 3);
      const int oy = oy0 + m / TF_W, ox = ox0 + m % TF_W;
      aux[q] = a.splits == 1 && oy < OH && ox < OW
                   ? epilogue_aux<MODE>(a, img + (int64_t)oy * OW + ox, n) : EpAux{0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < SM * 4; ++q) {
      const int m = wm0 + 16 * (q >> 2) + 4 * lq + (q & 3);
      const int oy = oy0 + m / TF_W, ox = ox0 + m % TF_W;
      if (oy >= OH || ox >= OW) continue;
      const int64_t row = img + (int64_t)oy * OW + ox;
      const float v = acc4[q >> 2][j][q & 3];
      if (a.splits > 1)
        a.slab[(int64_t)split * a.split_stride + row * a.slab_ld + n] = v;
      else
        epilogue_store<MODE>(a, row, n, v, bias, scale, shift, aux[q]);
    }
  }
}

template <int BN, int WAVES_M, int WAVES_N, int MODE, int TH, int NB = 2>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N, NB == 1 ? 2 : 1) void conv_tile_x3(GemmArgs a) {
  tile_x3_body<BN, WAVES_M, WAVES_N, MODE, TH, NB, 3>(a);
}

// bf16 (configs 3-5) 3x3 stride-1 fwd / dgrad on the same structure, one plane: 16x16x32
// fragments on 64-byte swizzled rows, B by LDS DMA one tap ahead, the 16-byte epilogue.  One
// plane takes a third of the split kernel's LDS (38 KB at 8 x 32 x 128), so two workgroups
// share a CU and one's staging / barrier / epilogue overlaps the other's MFMAs.
// (__launch_bounds__'s second argument is the minimum waves per SIMD: two workgroups of W
// waves per CU need W / 2.  Waves with more than 48 accumulator registers (the 8 x 32 x 128
// tile: 64) spill under that bound, and the 12-wave form exceeds 32 waves per CU: those keep
// one workgroup per CU.)
constexpr int b16_min_waves(int w, int acc) { return w <= 8 && acc <= 48 ? (w + 1) / 2 : (w + 3) / 4; }
template <int BN, int WAVES_M, int WAVES_N, int MODE, int TH>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N,
                             b16_min_waves(WAVES_M * WAVES_N,
                                           (TH * TF_W / WAVES_M / 16) * (BN / WAVES_N / 16) * 4))
void conv_tile_b16(GemmArgs a) {
  tile_x3_body<BN, WAVES_M, WAVES_N, MODE, TH, 2, 1>(a);
}

// ---- the stem (7x7 stride 2, 3 -> 4 padded input channels, 64 outputs) on the split-bf16
// MFMA.  conv_gemm_x3's im2col staging gathers 16-byte (one pixel's 4 channels) pieces per tap;
// here a 32-deep K chunk is one kernel row r: lane octet sp holds taps (r, 2 sp), (r, 2 sp + 1)
// x 4 channels = two horizontally adjacent input pixels, i.e. one aligned 16-byte read of the
// bf16 halo image (tap 7 is a zero weight column).  The workgroup stages the whole K (7 rows x
// 32) of B once, 3 planes x 64 rows with a 464-byte pitch (fragment reads conflict-free), and
// the tile's input halo ((2 TH + 5) x (2 TW + 6) pixels) once as 3 split planes; then 7 chunks
// of 6 MFMAs per fragment pair, the epilogue through per-wave LDS images (16-byte stores).
// CO = 64: 8 waves, 4 x 2 of 64 pixels (2 tile rows) x 32 output channels, 125 KB of LDS;
// CO = 32: each workgroup takes half the output channels with 4 waves and 80 KB, so two share
// a CU and one's staging / epilogue overlaps the other's MFMAs.
// NP = 1 is the bf16 path (configs 3-5): one plane of each operand (the halo rounded to bf16
// as conv_gemm_bf16 rounds its A, the packed bf16 weights), one MFMA per fragment pair and
// 32 KB of LDS, so four workgroups share a CU: the stem is then bound by its HBM pass
// (the 4-channel input read, the 64-channel output written once).
constexpr int ST_TH = 8, ST_TW = 32;
constexpr int ST_HH = 2 * ST_TH + 5, ST_HW = 2 * ST_TW + 6, ST_HWP = 72;
constexpr int ST_BROW = 232;      // bf16 per B row: 7 x 32 + 8

template <int CO, int NP = 3>
__global__ __launch_bounds__(CO * 8, CO == 64 ? 1 : NP == 1 ? 4 : 2) void conv_stem_x3(GemmArgs a, int ntiles) {
  constexpr int SM = 4, SN = 2, WM = 64, WN = 32, NW = CO / 8, NT = 64 * NW;
  static_assert(NP == 3 || NP == 1, "three split planes (fp32) or one (bf16)");
  constexpr int B_U4 = CO * ST_BROW / 8;              // uint4 per B plane
  constexpr int HWP = ST_HW;                          // halo pitch: B + halo 79.8 KB (fp32 CO 32)
  constexpr int H_PIX = ST_HH * HWP;                  // halo pixels (8 bytes each) per plane
  constexpr int HB_U4 = NP * H_PIX / 2, EP_U4 = NW * WM * WN * 4 / 16;
  constexpr int W_U4 = HB_U4 > EP_U4 ? HB_U4 : EP_U4; // halo planes, then the epilogue images
  // B stays for the workgroup's whole tile walk; the halo region is reused per tile
  __shared__ uint4 smem[NP * B_U4 + W_U4];
  char* Bs = reinterpret_cast<char*>(smem);                          // [plane][co][k']
  char* Hs = reinterpret_cast<char*>(smem + NP * B_U4);              // [plane][hy][hx] 8 B

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Persistent over tiles: the 64 / CO workgroups of a channel group share co0; workgroup w
  // walks tiles w / groups, + gridDim.x / groups, ...  (grid = tiles * groups: one tile each)
  constexpr int GROUPS = 64 / CO;
  const int wgid0 = xcd_remap(blockIdx.x, gridDim.x);
  const int co0 = (wgid0 % GROUPS) * CO;
  const int tstride = gridDim.x / GROUPS;
  const int tiles_x = (a.wo + ST_TW - 1) / ST_TW, tiles_y = (a.ho + ST_TH - 1) / ST_TH;
  int t = wgid0 / GROUPS;
  if (t >= ntiles) return;

  // ---- B: entry (plane, co, kernel row r, octet sp) <- taps (r, 2 sp), (r, 2 sp + 1) of the
  // x3 fwd image W16_f[co][tap * 4 + ci] (8-byte aligned pieces; tap 7 is zero), once.
  constexpr int BE = NP * CO * 28, BQ = (BE + NT - 1) / NT;
  constexpr int HE = ST_HH * ST_HW, HQ = (HE + NT - 1) / NT;
  const rsrc_t rb = make_rsrc(a.B, a.b_bytes);
  const rsrc_t ra = make_rsrc(a.A, a.a_bytes);
  float4 hv[HQ];
  // this tile's halo: input pixel (iy0 + hy, ix0 + hx), 4 channels, into registers
  auto load_halo = [&](int tt) {
    const int b = tt / (tiles_x * tiles_y);
    const int trem = tt - b * tiles_x * tiles_y;
    const int iy0 = 2 * ((trem / tiles_x) * ST_TH) - a.pt, ix0 = 2 * ((trem % tiles_x) * ST_TW) - a.pl;
#pragma unroll
    for (int k = 0; k < HQ; ++k) {
      const int q = tid + NT * k;
      const int hy = q / ST_HW, hx = q - hy * ST_HW;
      const int iy = iy0 + hy, ix = ix0 + hx;
      const bool ok = q < HE && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
      hv[k] = bload4(ra, ok ? (uint32_t)((((int64_t)b * a.h + iy) * a.w + ix) * a.lda * 4) : kOOB);
    }
  };
  auto store_halo = [&]() {                // (split into 3 planes for fp32)
#pragma unroll
    for (int k = 0; k < HQ; ++k) {
      const int q = tid + NT * k;
      if (HE % NT == 0 || q < HE) {
        const int hy = q / ST_HW, hx = q - hy * ST_HW;
        const int o = (hy * HWP + hx) * 8;
        if (NP == 1) {
          *reinterpret_cast<uint2*>(Hs + o) = pack_bf16x4(hv[k]);
        } else {
          uint2 h, m, l;
          split3x4(hv[k], h, m, l);
          *reinterpret_cast<uint2*>(Hs + o) = h;
          *reinterpret_cast<uint2*>(Hs + H_PIX * 8 + o) = m;
          *reinterpret_cast<uint2*>(Hs + 2 * H_PIX * 8 + o) = l;
        }
      }
    }
  };
  {
    // every load of B and the first halo issued before any LDS store (a load -> store loop
    // keeps one load in flight per thread: the stem is latency-bound on its staging)
    uint2 blo[BQ], bhi[BQ];
#pragma unroll
    for (int k = 0; k < BQ; ++k) {
      const int e = tid + NT * k;
      const int p = e / (CO * 28), rem = e - p * (CO * 28);
      const int co = rem / 28, rs = rem - co * 28, r = rs >> 2, sp = rs & 3;
      const uint32_t src =
          (uint32_t)((p * a.b_plane + (int64_t)(co0 + co) * a.ldb + (r * 7 + 2 * sp) * 4) * 2);
      const bool ok = e < BE && co0 + co < a.nb;
      blo[k] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rb, ok ? src : kOOB, 0, 0));
      bhi[k] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rb, ok && sp < 3 ? src + 8 : kOOB, 0, 0));
    }
    load_halo(t);
#pragma unroll
    for (int k = 0; k < BQ; ++k) {
      const int e = tid + NT * k;
      if (BE % NT == 0 || e < BE) {
        const int p = e / (CO * 28), rem = e - p * (CO * 28);
        const int co = rem / 28, rs = rem - co * 28, r = rs >> 2, sp = rs & 3;
        *reinterpret_cast<uint4*>(Bs + ((p * CO + co) * ST_BROW + r * 32 + sp * 8) * 2) =
            make_uint4(blo[k].x, blo[k].y, bhi[k].x, bhi[k].y);
      }
    }
  }

  const int wm = CO == 64 ? wave >> 1 : wave, wn = CO == 64 ? wave & 1 : 0;
  const int l16 = lane & 15, sp = lane >> 4;
  // A block i: output row 2 wm + (i >> 1), columns 16 (i & 1) + l16 -> halo pixel at kernel row 0
  int a_off[SM];
#pragma unroll
  for (int i = 0; i < SM; ++i)
    a_off[i] = ((2 * (2 * wm + (i >> 1))) * HWP + 2 * (16 * (i & 1) + l16) + 2 * sp) * 8;
  const int b_off = ((wn * WN + l16) * ST_BROW + sp * 8) * 2;
  constexpr int EPW = 32, LPR = 8, RPI = 8;
  float* E = reinterpret_cast<float*>(smem + NP * B_U4) + wave * WM * EPW;
  const int lq = lane >> 4;
  const int c4 = lane % LPR, rr = lane / LPR;
  const int n = co0 + wn * WN + 4 * c4;

  for (; t < ntiles; t += tstride) {
    const int b = t / (tiles_x * tiles_y);
    const int trem = t - b * tiles_x * tiles_y;
    const int oy0 = (trem / tiles_x) * ST_TH, ox0 = (trem % tiles_x) * ST_TW;
    store_halo();
    __syncthreads();
    // the next tile's halo loads stay in flight during this tile's MFMAs and epilogue
    if (t + tstride < ntiles) load_halo(t + tstride);

    f32x4 acc4[SM][SN];
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc4[i][j][r] = 0.f;
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      bf16x8 av[NP][SM], bv[NP][SN];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int i = 0; i < SM; ++i)
          av[p][i] = *reinterpret_cast<const bf16x8*>(Hs + p * H_PIX * 8 + a_off[i] + r * HWP * 8);
#pragma unroll
        for (int j = 0; j < SN; ++j)
          bv[p][j] = *reinterpret_cast<const bf16x8*>(Bs + p * B_U4 * 16 + b_off + (16 * j * ST_BROW + r * 32) * 2);
      }
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SN; ++j) {
          f32x4 x = acc4[i][j];
          if (NP == 3) {
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP - 1][i], bv[0][j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[NP - 1][j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP / 2][i], bv[NP / 2][j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP / 2][i], bv[0][j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[NP / 2][j], x, 0, 0, 0);
          }
          acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], x, 0, 0, 0);
        }
    }
    __syncthreads();                      // halo reads done: the halo region becomes E images

    // ---- epilogue: the wave's 64 x 32 block through a private LDS image, float4 rows
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) E[(16 * i + 4 * lq + r) * EPW + 16 * j + l16] = acc4[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t img = (int64_t)b * a.ho * a.wo;
#pragma unroll
    for (int q = 0; q < WM / RPI; ++q) {
      const int m = q * RPI + rr;
      const float4 v = *reinterpret_cast<const float4*>(&E[m * EPW + 4 * c4]);
      const int oy = oy0 + 2 * wm + m / 32, ox = ox0 + m % 32;
      if (oy < a.ho && ox < a.wo && n < a.N)
        epilogue_store4<MODE_FWD>(a, 0, img + (int64_t)oy * a.wo + ox, n, v);
    }
    if (a.pool_out) {
      // MaxPool2D (model.py:17) of the two output rows this wave owns (even rows: the 2 x 2
      // windows never straddle waves or tiles): the epilogue's value of each of the four pixels
      // (bias, BN, ReLU as epilogue_store4 computes it) and the max in maxpool2_fwd_kernel's
      // order, so the pooled tensor is the separate pass's bit for bit, without re-reading the
      // output.
      const int pho = a.ho / 2, pwo = a.wo / 2;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int it = lane + 64 * u;                 // 16 pooled columns x 8 channel quads
        const int pc = it >> 3, qq = it & 7;
        const int nn = co0 + wn * WN + 4 * qq;
        const int py = (oy0 + 2 * wm) / 2, px = ox0 / 2 + pc;
        if (py >= pho || px >= pwo || nn >= a.N) continue;
        float bias[4], scale[4], shift[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) column_params<MODE_FWD>(a, nn + e, bias[e], scale[e], shift[e]);
        float rv[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {                 // (0,0), (0,1), (1,0), (1,1)
          const int m = (k >> 1) * 32 + 2 * pc + (k & 1);
          const float4 v = *reinterpret_cast<const float4*>(&E[m * EPW + 4 * qq]);
          const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float x = vv[e] + bias[e];
            if (a.bn_g) x = x * scale[e] + shift[e];
            rv[k][e] = act_fwd(x, a.act, a.alpha);
          }
        }
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = fmaxf(fmaxf(rv[0][e], rv[1][e]), fmaxf(rv[2][e], rv[3][e]));
        *reinterpret_cast<float4*>(&a.pool_out[(((int64_t)b * pho + py) * pwo + px) * a.N + nn]) =
            make_float4(o[0], o[1], o[2], o[3]);
      }
    }
    __syncthreads();                      // E reads done before the next tile's halo store
  }
}

// of_set_tuning key 8: the stem on conv_stem_x3 (1: two 32-channel workgroups per CU,
// default; 2: one 64-channel workgroup) or on conv_gemm_x3 (0).
static int g_stem_x3 = 1;
// of_set_tuning key 31: conv_stem_x3 persistent with this many workgroups per CU (-1: the
// default, 2 fp32 / 3 bf16 / 1 for the 64-channel form; 0: one tile per workgroup).
static int g_stem_persist = -1;
// of_set_tuning key 15: the bf16 stem (forward and weight gradient) on the one-plane
// conv_stem_x3<32, 1> / conv_wgrad_stem_x3<1> (1, default) or on the bf16 GEMMs (0).
static int g_stem_bf16 = 1;
// of_set_tuning key 18: bf16 3x3 input gradients with BN = 128 on the tall (X3_TH0 x 32)
// output tiles of conv_tile_bf16 where the grid allows (1), as the forward does, or on 4 x 32
// tiles (0, default).
static int g_tall16_dgrad = 0;
// of_set_tuning key 20: conv_tile_bf16 with its fragments read one sub-step ahead (1, default)
// or right before their MFMAs (0, the round-1 schedule).
static int g_tile16_pf = 1;
bool stem_x3_ok(const of_conv_desc* d) {
  return d->kh == 7 && d->kw == 7 && d->stride == 2 && d->cin_p == 4 && d->cout == 64 &&
         d->pad_top >= 0 && d->pad_top <= 3 && d->pad_left >= 0 && d->pad_left <= 3;
}

// ---- fp32 on bf16 MFMA by the three-term split: implicit-GEMM fwd / dgrad ------------------
// The shapes the halo tiles do not cover (the 7x7 stride-2 stem, the 3x3 stride-2 block
// convs and the 1x1 stride-2 projections, with the stride-2 input gradient as phase groups):
// conv_gemm_bf16's geometry (tap walkers, phase groups, K in 32-deep chunks of the packed
// [n][k] images, split-K slabs) with the operands cut into the hi / mid / lo planes of
// conv_tile_x3 and six v_mfma_f32_16x16x32_bf16 per fragment pair.  A (activations) is
// register-staged and split while it is stored; B (the x3 weight planes) comes in by LDS DMA;
// both LDS images are double-buffered rows of four octets in the x3_sw swizzle (one barrier
// per chunk).  Waves own WM x WN blocks of 16 x 16 tiles.  Wave w stages octet w & 3 of every
// chunk (two channel quads with their own tap walks) for row group w >> 2.
// NP = 1 is the bf16 path (configs 3-5, the stride-2 block convs and projections): one plane
// of each operand (A rounded to bf16 as conv_gemm_bf16 rounds it, B the packed bf16 image,
// which has the x3 hi plane's layout), one MFMA per fragment pair, and with a third of the
// LDS two workgroups per CU.
template <int BM, int BN, int WAVES_M, int WAVES_N, int MODE, int NP = 3, int RING = 3>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N, NP == 1 || RING == 2 ? 2 : 1)
void conv_gemm_x3(GemmArgs a) {
  static_assert(MODE == MODE_FWD || MODE == MODE_DGRAD, "x3 GEMM: fwd / dgrad");
  static_assert(NP == 3 || NP == 1, "three split planes (fp32) or one (bf16)");
  constexpr int NT = 64 * WAVES_M * WAVES_N, NW = NT / 64;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, SM = WM / 16, SN = WN / 16;
  static_assert(NW % 4 == 0 && SM >= 1 && SN >= 1 && WM % 16 == 0 && WN % 16 == 0, "tile");
  constexpr int RG = NW / 4;                     // row groups (4 waves each: one per octet)
  constexpr int A_SL = BM / (64 * RG);           // A rows per lane
  static_assert(A_SL >= 1 && BM % (64 * RG) == 0, "BM");
  constexpr int A_U4 = NP * BM * 4, B_U4 = NP * BN * 4;
  constexpr int BDI = NP * BN / 16, BDW = (BDI + NW - 1) / NW;   // B DMA wave-instructions
  constexpr int OP_U4 = 2 * (A_U4 + B_U4), EP_U4 = NW * WM * WN * 4 / 16;
  // DA (RING = slots 2 / 3, of_set_tuning key 30; where the LDS allows): A comes by LDS DMA
  // too, as raw fp32 rows in [quad][row] images split (fp32) or rounded (bf16) while its
  // fragments are read, and (A, B) chunks cycle through an NS-slot ring with NS - 2 chunks in
  // flight across each barrier (counted vmcnt, raw s_barrier); NS = 2 leaves room for two
  // workgroups per CU.  (A register-staged ring cannot go deeper than one chunk: hipcc drains
  // every LDS DMA (vmcnt(0)) at the first use of an ordinary load's registers.)  Measured: the
  // 3-slot ring alone is even with the register form -- the loop was not waiting on its loads
  // (SQ: 37 % of wave-cycles parked at waits / barriers, 32 % issue-stalled, MFMA ~25 % busy,
  // eight barrier-locked waves per CU) -- and the 2-slot ring's second workgroup per CU is
  // what gains (-10..-15 % on the stride-2 layers).
  constexpr int AF_U4 = BM * 8, SLOT_U4 = AF_U4 + B_U4;
  constexpr int NS = RING == 2 && 2 * 2 * SLOT_U4 * 16 <= 160 * 1024 ? 2
                   : RING && 3 * SLOT_U4 * 16 * (NP == 1 ? 2 : 1) <= 160 * 1024 ? 3 : 0;
  constexpr bool DA = NS > 0;
  constexpr int OPS_U4 = DA ? NS * SLOT_U4 : OP_U4;
  __shared__ uint4 smem[OPS_U4 > EP_U4 ? OPS_U4 : EP_U4];   // operands, then epilogue images

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Stride-2 input gradients (phase groups of 4 / 2 / 2 / 1 taps, contiguous in the tile
  // space) skip the XCD remap: it would hand each XCD the tiles of one or two groups (the
  // 4-tap group's XCDs then run 1.8x the average), while block order deals every group
  // evenly over the 8 XCDs and starts the longest tiles first.
  const int wgid = a.phase ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_n = tile % a.n_tiles;
  const int tile_mg = tile / a.n_tiles;
  int gi = 0;
#pragma unroll
  for (int g = 1; g < MAX_GROUPS; ++g)
    if (g < a.ngroups && tile_mg >= a.grp[g].tiles_begin) gi = g;
  const Group& G = a.grp[gi];
  const int tile_m = tile_mg - G.tiles_begin;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int M = G.M;
  const int k_begin = split * a.k_per_split;
  const int k_end = min(G.K, k_begin + a.k_per_split);
  const int nchunks = k_end > k_begin ? (k_end - k_begin + BKH - 1) / BKH : 0;
  const rsrc_t ra_src = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rb_src = make_rsrc(a.B, a.b_bytes);

  // ---------------- A rows (conv_gemm_bf16's geometry) --------------------------------------
  const int oct = wave & 3, rgrp = wave >> 2;
  const int src_h = (MODE == MODE_DGRAD) ? a.ho : a.h;
  const int src_w = (MODE == MODE_DGRAD) ? a.wo : a.w;
  int a_off[A_SL];
  uint64_t a_msk[A_SL];
#pragma unroll
  for (int i = 0; i < A_SL; ++i) {
    const int m = m0 + 64 * (rgrp + RG * i) + lane;
    const bool okm = m < M;
    const int mm = okm ? m : 0;
    int b, yb, xb;
    if (MODE == MODE_FWD) {
      const int hw = a.ho * a.wo;
      b = mm / hw;
      const int rem = mm - b * hw;
      const int oy = rem / a.wo, ox = rem - oy * a.wo;
      yb = oy * a.stride - a.pt;
      xb = ox * a.stride - a.pl;
    } else if (a.phase) {
      const int hw = G.hc * G.wc;
      b = mm / hw;
      const int rem = mm - b * hw;
      const int u = rem / G.wc, v = rem - u * G.wc;
      yb = (2 * u + G.ry + a.pt - G.r0) >> 1;
      xb = (2 * v + G.rx + a.pl - G.s0) >> 1;
    } else {
      const int hw = a.h * a.w;
      b = mm / hw;
      const int rem = mm - b * hw;
      const int iy = rem / a.w, ix = rem - iy * a.w;
      yb = iy + a.pt;
      xb = ix + a.pl;
    }
    a_off[i] = (int)(((int64_t)(b * src_h + yb) * src_w + xb) * a.lda * 4);
    uint64_t msk = 0;
    if (okm) {
      uint64_t colmask = 0;
      for (int ts = 0; ts < G.ns; ++ts) {
        const int sx = (MODE == MODE_FWD) ? xb + ts : xb - ts;
        if ((unsigned)sx < (unsigned)src_w) colmask |= (uint64_t)1 << ts;
      }
      int t = 0;
      for (int tr = 0; t < G.ntaps; ++tr, t += G.ns) {
        const int sy = (MODE == MODE_FWD) ? yb + tr : yb - tr;
        if ((unsigned)sy < (unsigned)src_h) msk |= colmask << t;
      }
      if (G.ntaps < 64) msk &= ((uint64_t)1 << G.ntaps) - 1;
    }
    a_msk[i] = msk;
  }
  // two wave-uniform tap walkers: channel quads 2 oct and 2 oct + 1 of the chunk
  int ks_t[2], ks_tr[2], ks_ts[2], ks_ci[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k0 = k_begin + oct * 8 + 4 * h;
    ks_t[h] = k0 / a.kc;
    ks_ci[h] = k0 - ks_t[h] * a.kc;
    ks_tr[h] = ks_t[h] / G.ns;
    ks_ts[h] = ks_t[h] - ks_tr[h] * G.ns;
  }
  const int sgn = MODE == MODE_FWD ? 1 : -1;
  const int tap_step = sgn * src_w * a.lda * 4;
  float4 ra[A_SL][2];
  auto load_a = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool tap_ok = ks_t[h] < G.ntaps;
      const int koff = ks_tr[h] * tap_step + sgn * ks_ts[h] * a.lda * 4 + ks_ci[h] * 4;
#pragma unroll
      for (int i = 0; i < A_SL; ++i) {
        const bool ok = tap_ok && ((a_msk[i] >> ks_t[h]) & 1);
        ra[i][h] = bload4(ra_src, ok ? (uint32_t)(a_off[i] + koff) : kOOB);
      }
    }
  };
  auto advance_a = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ks_ci[h] += BKH;
      while (ks_ci[h] >= a.kc) {
        ks_ci[h] -= a.kc;
        ++ks_t[h];
        if (++ks_ts[h] >= G.ns) {
          ks_ts[h] = 0;
          ++ks_tr[h];
        }
      }
    }
  };
  auto store_a = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_SL; ++i) {
      const int row = 64 * (rgrp + RG * i) + lane;
      uint4* img = smem + buf * A_U4 + row * 4 + (oct ^ x3_sw(row));
      if (NP == 1) {
        img[0] = pack_bf16x8(ra[i][0], ra[i][1]);
      } else {
        uint2 h0, m0v, l0, h1, m1, l1;
        split3x4(ra[i][0], h0, m0v, l0);
        split3x4(ra[i][1], h1, m1, l1);
        img[0] = make_uint4(h0.x, h0.y, h1.x, h1.y);
        img[(NP / 2) * BM * 4] = make_uint4(m0v.x, m0v.y, m1.x, m1.y);
        img[(NP - 1) * BM * 4] = make_uint4(l0.x, l0.y, l1.x, l1.y);
      }
    }
  };
  // ---------------- B (x3 weight planes [plane][n][k]) by LDS DMA ----------------------------
  uint32_t bd_off[BDW];
  int bd_lds[BDW];
#pragma unroll
  for (int k = 0; k < BDW; ++k) {
    const int g = wave + NW * k;
    const int p = g / (BN / 16), rbk = g % (BN / 16);
    const int n = rbk * 16 + (lane >> 2), o = (lane & 3) ^ x3_sw(lane >> 2);
    bd_off[k] = g < BDI && n0 + n < a.nb
                    ? (uint32_t)(((int64_t)p * a.b_plane + (int64_t)(n0 + n) * a.ldb + G.b_off +
                                  8 * o) * 2)
                    : kOOB;
    bd_lds[k] = g < BDI ? (p * BN + rbk * 16) * 4 : -1;
  }
  auto dma_b = [&](int buf, int bk) {
#pragma unroll
    for (int k = 0; k < BDW; ++k)
      if (BDI % NW == 0 || bd_lds[k] >= 0)
        dma16_to_lds(rb_src, smem + 2 * A_U4 + buf * B_U4 + bd_lds[k], bd_off[k], bk * 2);
  };

  // ---------------- main loop --------------------------------------------------------------
  f32x4 acc[SM][SN];
#pragma unroll
  for (int i = 0; i < SM; ++i)
#pragma unroll
    for (int j = 0; j < SN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
  const int wm0 = (wave / WAVES_N) * WM;
  const int wn0 = (wave % WAVES_N) * WN;
  const int l16 = lane & 15, lq = lane >> 4;
  const int frag = l16 * 4 + (lq ^ x3_sw(l16));   // rows 16-aligned + l16: swizzle of l16
  int b_k = k_begin;
  if constexpr (DA) {
    // this wave's DMA wave-instructions per chunk: 2 A_SL (A) + its share of B's
    const int nw = 2 * A_SL + (BDI % NW == 0 ? BDW : (BDI - wave + NW - 1) / NW);
    static_assert(2 * A_SL + BDW <= 7, "vm_wait covers 0..7");
    auto vm_wait = [](int n) {               // s_waitcnt vmcnt(n), n wave-uniform
      switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
      }
    };
    // chunk (walkers, bk) -> ring slot: lane L of the (octet, half, row group) instruction
    // brings row 64 (rgrp + RG i) + L's channel quad 2 oct + h (zeros where the tap is outside
    // the image or the row past M), so quad q of the chunk lands as BM contiguous rows
    auto issue = [&](int slot, int bk) {
      uint4* S = smem + slot * SLOT_U4;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool tap_ok = ks_t[h] < G.ntaps;
        const int koff = ks_tr[h] * tap_step + sgn * ks_ts[h] * a.lda * 4 + ks_ci[h] * 4;
#pragma unroll
        for (int i = 0; i < A_SL; ++i) {
          const bool ok = tap_ok && ((a_msk[i] >> ks_t[h]) & 1);
          dma16_to_lds(ra_src, S + (2 * oct + h) * BM + 64 * (rgrp + RG * i),
                       ok ? (uint32_t)(a_off[i] + koff) : kOOB, 0);
        }
      }
#pragma unroll
      for (int k = 0; k < BDW; ++k)
        if (BDI % NW == 0 || bd_lds[k] >= 0)
          dma16_to_lds(rb_src, S + AF_U4 + bd_lds[k], bd_off[k], bk * 2);
    };
    // per-lane LDS byte addresses of the fragment reads within a slot: A quad 2 lq of row
    // wm0 + l16 (+ BM rows for quad 2 lq + 1, + 16 rows per fragment), B as frag above
    const uint32_t smem_lds = lds_off(smem);
    const uint32_t a_rd = (uint32_t)(((2 * lq) * BM + wm0 + l16) * 16);
    const uint32_t b_rd = (uint32_t)((AF_U4 + wn0 * 4 + frag) * 16);
    if (nchunks > 0) issue(0, b_k);
    if (NS == 3 && nchunks > 1) {
      advance_a();
      b_k += BKH;
      issue(1, b_k);
    }
    for (int c = 0; c < nchunks; ++c) {
      vm_wait(NS == 3 && c + 1 < nchunks ? nw : 0);   // this wave's part of chunk c landed
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();          // every wave's part landed; slot (c + NS - 1) % NS,
      asm volatile("" ::: "memory");         // read in step c - 1, is free
      if (c + NS - 1 < nchunks) {
        advance_a();
        b_k += BKH;
        issue((c + NS - 1) % NS, b_k);
      }
      // The fragment reads are inline asm: an LDS load with a memory operand makes hipcc wait
      // vmcnt(0) -- the ring's in-flight DMAs -- before it.  One lgkmcnt(0) retires them.
      const uint32_t sb = smem_lds + (uint32_t)((c % NS) * SLOT_U4 * 16);
      uint4 ar[SM][2], br[NP][SN];
#pragma unroll
      for (int i = 0; i < SM; ++i) {
        ar[i][0] = ds_read16(sb + a_rd + 256 * i);
        ar[i][1] = ds_read16(sb + a_rd + 256 * i + BM * 16);
      }
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int j = 0; j < SN; ++j) br[p][j] = ds_read16(sb + b_rd + p * BN * 64 + j * 1024);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 av[NP][SM], bv[NP][SN];
#pragma unroll
      for (int i = 0; i < SM; ++i) {
        const float4 x0 = __builtin_bit_cast(float4, ar[i][0]);
        const float4 x1 = __builtin_bit_cast(float4, ar[i][1]);
        if constexpr (NP == 1) {
          av[0][i] = __builtin_bit_cast(bf16x8, pack_bf16x8(x0, x1));
        } else {
          uint2 h0, m0v, l0, h1, m1, l1;
          split3x4(x0, h0, m0v, l0);
          split3x4(x1, h1, m1, l1);
          av[0][i] = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
          av[NP / 2][i] = __builtin_bit_cast(bf16x8, make_uint4(m0v.x, m0v.y, m1.x, m1.y));
          av[NP - 1][i] = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
        }
      }
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int j = 0; j < SN; ++j) bv[p][j] = __builtin_bit_cast(bf16x8, br[p][j]);
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SN; ++j) {
          f32x4 x = acc[i][j];
          if (NP == 3) {
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP - 1][i], bv[0][j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[NP - 1][j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP / 2][i], bv[NP / 2][j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP / 2][i], bv[0][j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[NP / 2][j], x, 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], x, 0, 0, 0);
        }
    }
    __syncthreads();              // every wave's last ring reads done: LDS -> epilogue images
  } else {
  if (nchunks > 0) {
    load_a();
    dma_b(0, b_k);
    store_a(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) {
      advance_a();
      b_k += BKH;
      load_a();
      dma_b(buf ^ 1, b_k);
    }
    const uint4* As = smem + buf * A_U4;
    const uint4* Bs = smem + 2 * A_U4 + buf * B_U4;
    bf16x8 av[NP][SM], bv[NP][SN];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
      for (int i = 0; i < SM; ++i)
        av[p][i] = __builtin_bit_cast(bf16x8, As[p * BM * 4 + (wm0 + 16 * i) * 4 + frag]);
#pragma unroll
      for (int j = 0; j < SN; ++j)
        bv[p][j] = __builtin_bit_cast(bf16x8, Bs[p * BN * 4 + (wn0 + 16 * j) * 4 + frag]);
    }
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j) {
        f32x4 x = acc[i][j];
        if (NP == 3) {
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP - 1][i], bv[0][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[NP - 1][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP / 2][i], bv[NP / 2][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP / 2][i], bv[0][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[NP / 2][j], x, 0, 0, 0);
        }
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], x, 0, 0, 0);
      }
    if (more) store_a(buf ^ 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // own B DMA landed
    __syncthreads();
  }
  }

  // ---------------- epilogue ----------------------------------------------------------------
  const int row_base = G.tiles_begin * BM;
  float* S = a.slab + (int64_t)split * a.split_stride;
  if (a.vec_ep) {
    // the wave's WM x WN block through a private LDS image, back as float4 rows
    float* E = reinterpret_cast<float*>(smem) + wave * WM * WN;
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) E[(16 * i + 4 * lq + r) * WN + 16 * j + l16] = acc[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr int LPR = WN / 4, RPI = 64 / LPR;
    const int c4 = lane % LPR, rr = lane / LPR;
    const int n = n0 + wn0 + 4 * c4;
    if (a.splits > 1) {
#pragma unroll
      for (int q = 0; q < WM / RPI; ++q) {
        const int ml = q * RPI + rr;
        const int m = m0 + wm0 + ml;
        const float4 v = *reinterpret_cast<const float4*>(&E[ml * WN + 4 * c4]);
        if (m >= M || n >= a.N) continue;
        *reinterpret_cast<float4*>(&S[(int64_t)(row_base + m) * a.slab_ld + n]) = v;
      }
      return;
    }
    // rows in groups of GR through epilogue_rows4c: each group's residual / activation-source
    // quads loaded before its first store (row by row, every load sat behind the row's guard
    // and waited: WM / RPI serial memory round trips per wave)
    if constexpr (!EPC_BATCH) {        // the round-2 form, for A/B builds
#pragma unroll
      for (int q = 0; q < WM / RPI; ++q) {
        const int ml = q * RPI + rr;
        const int m = m0 + wm0 + ml;
        const float4 v = *reinterpret_cast<const float4*>(&E[ml * WN + 4 * c4]);
        if (m >= M || n >= a.N) continue;
        epilogue_store4<MODE>(a, 0, out_row(a, G, m), n, v);
      }
      return;
    }
    constexpr int NQ = WM / RPI, GR = NQ % 4 == 0 ? 4 : NQ % 2 == 0 ? 2 : 1;
    const bool bnp = MODE == MODE_DGRAD && a.bnp != nullptr;
    // input gradient with the BN partial sums of the layer whose output is act_src (one K
    // slice, host-checked): the lane's column quad over its rows (dgrad_rows4c_bnp), then over
    // the lanes of the quad (shuffles) and the WAVES_M waves of the column block in wave order
    // (LDS): one partial row per output tile (tile_mg, over the phase groups) and channel
    float4 bt = make_float4(0.f, 0.f, 0.f, 0.f), ig = bt, bsb = bt, bsg = bt;
    if (bnp && n < a.N) {
      bt = *reinterpret_cast<const float4*>(&a.bnp_b[n]);
      const float4 gm = *reinterpret_cast<const float4*>(&a.bnp_g[n]);
      ig = make_float4(1.f / gm.x, 1.f / gm.y, 1.f / gm.z, 1.f / gm.w);
    }
#pragma unroll
    for (int q0 = 0; q0 < NQ; q0 += GR) {
      float4 v[GR];
      int64_t row[GR];
      unsigned ok = 0;
#pragma unroll
      for (int g = 0; g < GR; ++g) {
        const int ml = (q0 + g) * RPI + rr;
        const int m = m0 + wm0 + ml;
        v[g] = *reinterpret_cast<const float4*>(&E[ml * WN + 4 * c4]);
        row[g] = out_row(a, G, min(m, M - 1));           // clamped: the loads stay in range
        ok |= (m < M && n < a.N ? 1u : 0u) << g;
      }
      if (bnp) {                         // (row by row: GR rows of three operand quads raised
#pragma unroll                                // the kernel's VGPRs past the two-workgroup budget)
        for (int g = 0; g < GR; ++g)
          dgrad_rows4c_bnp<1>(a, &row[g], (ok >> g) & 1u, n, min(n, a.N - 4), &v[g], bt, ig, bsb, bsg);
      } else
        epilogue_rows4c<MODE, GR>(a, 0, row, ok, n, min(n, a.N - 4), v);
    }
    if (MODE == MODE_DGRAD && bnp) {
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) {
        bsb.x += __shfl_xor(bsb.x, o, 64), bsb.y += __shfl_xor(bsb.y, o, 64);
        bsb.z += __shfl_xor(bsb.z, o, 64), bsb.w += __shfl_xor(bsb.w, o, 64);
        bsg.x += __shfl_xor(bsg.x, o, 64), bsg.y += __shfl_xor(bsg.y, o, 64);
        bsg.z += __shfl_xor(bsg.z, o, 64), bsg.w += __shfl_xor(bsg.w, o, 64);
      }
      __syncthreads();                    // every wave's E image reads are done
      float4* red = reinterpret_cast<float4*>(smem);   // [2][WAVES_M][BN / 4]
      const int wmi = wave / WAVES_N;
      if (rr == 0) {
        red[wmi * (BN / 4) + wn0 / 4 + c4] = bsb;
        red[(WAVES_M + wmi) * (BN / 4) + wn0 / 4 + c4] = bsg;
      }
      __syncthreads();
      if (tid < BN / 4 && n0 + 4 * tid < a.N) {
        float4 sb = red[tid], sg = red[WAVES_M * (BN / 4) + tid];
        for (int w2 = 1; w2 < WAVES_M; ++w2) {
          add4(sb, red[w2 * (BN / 4) + tid]);
          add4(sg, red[(WAVES_M + w2) * (BN / 4) + tid]);
        }
        float* prow = a.bnp + (int64_t)tile_mg * 2 * a.N + n0 + 4 * tid;
        *reinterpret_cast<float4*>(prow) = sb;
        *reinterpret_cast<float4*>(prow + a.N) = sg;
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < SN; ++j) {
    const int n = n0 + wn0 + 16 * j + l16;
    if (n >= a.N) continue;
    float bias = 0.f, scale = 1.f, shift = 0.f;
    if (a.splits == 1) column_params<MODE>(a, n, bias, scale, shift);
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm0 + 16 * i + 4 * lq + r;
        if (m >= M) continue;
        if (a.splits > 1) {
          S[(int64_t)(row_base + m) * a.slab_ld + n] = acc[i][j][r];
        } else {
          const int64_t row = out_row(a, G, m);
          epilogue_store<MODE>(a, row, n, acc[i][j][r], bias, scale, shift,
                               epilogue_aux<MODE>(a, row, n));
        }
      }
  }
}

// Weight gradient on bf16 MFMA: C[m=(tap,ci)][n=co] = sum_{k=output pixel} x[pix(k,tap)][ci] *
// dy[k][co], both operands rounded to bf16 while staged, fp32 accumulation into the split-K
// slabs (reduced by wgrad_reduce_kernel, as the f32 path).  The MFMA operands need 8
// consecutive pixels per lane, while NHWC keeps channels contiguous: each staging slot loads
// a 4-channel x 8-pixel block (8 float4, coalesced across the lanes of a pixel) and writes
// it transposed as 4 rows of 8 bf16 (ds_write_b128) into the same [row][k] images the
// fwd/dgrad kernel reads.  Chunk = 32 pixels; slots = BM + BN (4 rows x 8 pixels each).
// The bias gradient (column sums of dy) is accumulated in fp32 from the staged values.
template <int BM, int BN, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(256, 2) void conv_wgrad_bf16(GemmArgs a) {
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  constexpr int NSLOT = BM + BN;
  constexpr int SPT = (NSLOT + 255) / 256;
  __shared__ uint4 As[2][BM * SROW16];
  __shared__ uint4 Bs[2][BN * SROW16];
  __shared__ float csum[4][BN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_n = tile % a.n_tiles;
  const int tile_m = tile / a.n_tiles;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int M = a.M;
  const int k_begin = split * a.k_per_split;
  const int k_end = min(a.K, k_begin + a.k_per_split);
  const int nchunks = k_end > k_begin ? (k_end - k_begin + BKH - 1) / BKH : 0;
  const rsrc_t rx = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rd = make_rsrc(a.B, a.b_bytes);
  const bool do_colsum = a.colsum && tile_m == 0;

  // ---- per-slot fixed state
  bool s_isa[SPT], s_ok[SPT];
  int s_row[SPT], s_oc[SPT], s_col[SPT];          // LDS row, k-octet, channel offset
  int s_r[SPT], s_s[SPT];                         // A: tap
  int s_b[SPT], s_oy[SPT], s_ox[SPT];             // first pixel of the slot's octet
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int sl = tid + 256 * j;
    const bool live = sl < NSLOT;
    const bool isa = sl < BM;
    const int q = isa ? sl : sl - BM;
    const int nq = isa ? BM / 4 : BN / 4;
    const int rq = q % nq, oc = q / nq;
    s_isa[j] = isa;
    s_row[j] = 4 * rq;
    s_oc[j] = live ? oc : -1;
    if (isa) {
      const int m = m0 + 4 * rq;
      s_ok[j] = live && m < M;
      const int mm = m < M ? m : 0;
      const int tap = mm / a.kc;
      s_col[j] = mm - tap * a.kc;
      s_r[j] = tap / a.kw;
      s_s[j] = tap - s_r[j] * a.kw;
    } else {
      const int n = n0 + 4 * rq;
      s_ok[j] = live && n < a.nb;
      s_col[j] = n;
      s_r[j] = s_s[j] = 0;
    }
    const int k = k_begin + 8 * oc;
    const int hw = a.ho * a.wo;
    const int kk = k < a.K ? k : 0;
    s_b[j] = kk / hw;
    const int rem = kk - s_b[j] * hw;
    s_oy[j] = rem / a.wo;
    s_ox[j] = rem - s_oy[j] * a.wo;
  }
  float4 stg[SPT][8];
  float4 colacc = make_float4(0.f, 0.f, 0.f, 0.f);
  int kc0 = k_begin;   // first pixel of the current chunk

  auto load = [&]() {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      int b = s_b[j], oy = s_oy[j], ox = s_ox[j];
      const int kbase = kc0 + 8 * s_oc[j];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool okk = s_ok[j] && s_oc[j] >= 0 && kbase + e < k_end;
        uint32_t off = kOOB;
        if (s_isa[j]) {
          const int sy = oy * a.stride - a.pt + s_r[j], sx = ox * a.stride - a.pl + s_s[j];
          if (okk && (unsigned)sy < (unsigned)a.h && (unsigned)sx < (unsigned)a.w)
            off = (uint32_t)((((b * a.h + sy) * a.w + sx) * a.lda + s_col[j]) * 4);
          stg[j][e] = bload4(rx, off);
        } else {
          if (okk) off = (uint32_t)(((kbase + e) * a.ldb + s_col[j]) * 4);
          stg[j][e] = bload4(rd, off);
        }
        if (++ox >= a.wo) {
          ox = 0;
          if (++oy >= a.ho) {
            oy = 0;
            ++b;
          }
        }
      }
    }
  };
  auto advance = [&]() {
    kc0 += BKH;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      s_ox[j] += BKH;
      while (s_ox[j] >= a.wo) {
        s_ox[j] -= a.wo;
        if (++s_oy[j] >= a.ho) {
          s_oy[j] = 0;
          ++s_b[j];
        }
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (s_oc[j] < 0) continue;
      float4 t[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = stg[j][e];
      // rows (channel c of the quad) of 8 pixels each
      const uint4 r0 = pack_bf16x8(make_float4(t[0].x, t[1].x, t[2].x, t[3].x),
                                   make_float4(t[4].x, t[5].x, t[6].x, t[7].x));
      const uint4 r1 = pack_bf16x8(make_float4(t[0].y, t[1].y, t[2].y, t[3].y),
                                   make_float4(t[4].y, t[5].y, t[6].y, t[7].y));
      const uint4 r2 = pack_bf16x8(make_float4(t[0].z, t[1].z, t[2].z, t[3].z),
                                   make_float4(t[4].z, t[5].z, t[6].z, t[7].z));
      const uint4 r3 = pack_bf16x8(make_float4(t[0].w, t[1].w, t[2].w, t[3].w),
                                   make_float4(t[4].w, t[5].w, t[6].w, t[7].w));
      uint4* img = s_isa[j] ? As[buf] : Bs[buf];
      const int base = s_row[j] * SROW16 + s_oc[j];
      img[base] = r0;
      img[base + SROW16] = r1;
      img[base + 2 * SROW16] = r2;
      img[base + 3 * SROW16] = r3;
      if (!s_isa[j] && do_colsum) {
#pragma unroll
        for (int e = 0; e < 8; ++e) add4(colacc, t[e]);
      }
    }
  };

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
    load();
    store(0);
  }
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) {
      advance();
      load();
    }
#pragma unroll
    for (int st = 0; st < BKH / 16; ++st) {
      bf16x8 av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        av[i] = __builtin_bit_cast(bf16x8, As[buf][(wm0 + 32 * i + lrow) * SROW16 + 2 * st + lk]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bv[j] = __builtin_bit_cast(bf16x8, Bs[buf][(wn0 + 32 * j + lrow) * SROW16 + 2 * st + lk]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }

  // ---- raw partial sums into this K slice's slab (+ bias column sums in row M)
  float* S = a.slab + (int64_t)split * a.split_stride;
  if (do_colsum) {
    // B-slot threads hold 4 columns x their k-octet; 4 octets per column quad
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (!s_isa[j] && s_oc[j] >= 0) {
        const int cq = s_row[j];
        csum[s_oc[j]][cq] = colacc.x;
        csum[s_oc[j]][cq + 1] = colacc.y;
        csum[s_oc[j]][cq + 2] = colacc.z;
        csum[s_oc[j]][cq + 3] = colacc.w;
      }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.N)
      S[(int64_t)M * a.slab_ld + n0 + tid] = csum[0][tid] + csum[1][tid] + csum[2][tid] + csum[3][tid];
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + 32 * j + lrow;
    if (n >= a.N) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (m < M) S[(int64_t)m * a.slab_ld + n] = acc[i][j][r];
      }
  }
}

// ---- bf16 weight gradient, 3x3 stride 1: all 9 taps from one staged halo ---------------
// dW[r][s][ci][co] = sum_p x(p + (r, s) - pad)[ci] . dy(p)[co].  A workgroup owns CIB input x
// COB output channels for ALL 9 taps (wave = 32 ci x 32 co x 9 taps = 9 accumulators) and
// walks 8 x 16 output-pixel tiles of its K slice: per tile it stages dy [co][128 px] once and
// the x halo (10 rows x 18 px) once, as three copies shifted by s = 0, 1, 2 pixels so every
// tap's A fragment (8 consecutive pixels of one channel) is an aligned 16-byte LDS read.
// Against the implicit GEMM (each tap a separate GEMM row block re-reading x and dy through
// L2) this cuts global traffic per MFMA by ~3.5x.  Both LDS images are double-buffered, one
// barrier per tile; the fp32 -> bf16 rounding and the [pixel][ch] -> [ch][pixel] transpose
// happen in the staging registers.  XOR swizzles keep the ds_read_b128 fragments
// conflict-free: x rows (s, hy, ci) of 2 octets swap the octets of ci & 8; dy rows of 16
// octets XOR the octet with co & 15.  K slice = a range of pixel tiles (a.K tiles in all).
// Output: the same split-K slabs as conv_wgrad_bf16 (rows tap * kc + ci, bias row M).
// PF = 1 (of_set_tuning key 17, default): the fragments are software-pipelined.  A tap row's
// fragment (x row kk + r, shift s) serves the three output rows kk = row - r, so a tile needs
// 10 x 3 distinct A reads, not 8 x 9: rows are read two output rows ahead of their first use,
// and the tile's 8 B fragments at its start (PF = 0 read 9 A and 1 B fragment per output row
// right before their MFMAs, the B one behind a full lgkmcnt(0) wait).
template <int WAVES_CI, int WAVES_CO, int PF = 1>
__global__ __launch_bounds__(256, 1) void conv_wgrad_tile_bf16(GemmArgs a) {
  constexpr int CIB = 32 * WAVES_CI, COB = 32 * WAVES_CO, KS = 3, HH = TT_H + KS - 1;
  static_assert(WAVES_CI * WAVES_CO == 4 && COB >= 64, "4 waves, COB >= 64");
  static_assert(TT_H == 8 && TT_W == 16, "tile = 8 rows x 16 px");
  constexpr int XQ = HH * (CIB / 4) * 2, XS = (XQ + 255) / 256;   // (hy, ci quad, half)
  constexpr int DQ = 16 * (COB / 4), DS = DQ / 256;               // (octet, co quad)
  static_assert(DQ % 256 == 0, "dy items");
  constexpr int NG = 256 / (COB / 4);                              // colsum groups
  __shared__ uint4 Xs[2][KS * HH * CIB * 2];
  __shared__ uint4 Ds[2][COB * 16];
  __shared__ float csum[NG][COB];

  // LDS swizzles (conflict-free for both the transposing ds_write_b128 stores, 8 lanes =
  // 8 channel quads / co quads, and the MFMA fragment ds_read_b128 reads, 16-lane groups;
  // checked exhaustively offline): x row of channel ci -> xrow(ci), its two 16-byte
  // pixel octets swapped when bit 4 of ci is set; dy row co: octet o -> o ^ dsw(co).
  auto xrow = [](int ci) { return ci ^ ((ci >> 2) & 2); };
  auto xoct = [](int ci) { return (ci >> 4) & 1; };
  auto dsw = [](int co) { return ((co & 15) ^ (((co >> 2) & 7) << 1)) & 15; };
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_co = tile % a.n_tiles;
  const int tile_ci = tile / a.n_tiles;
  const int ci0 = tile_ci * CIB, co0 = tile_co * COB;
  const int t_begin = split * a.k_per_split;
  const int t_end = min(a.K, t_begin + a.k_per_split);
  const int steps = max(0, t_end - t_begin);
  const int tiles_x = (a.wo + TT_W - 1) / TT_W, tiles_y = (a.ho + TT_H - 1) / TT_H;
  const rsrc_t rx = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rd = make_rsrc(a.B, a.b_bytes);
  const bool do_colsum = a.colsum && tile_ci == 0;

  // x items: channel quad fastest (coalesced 16-B lanes of one pixel)
  const int xcq = tid % (CIB / 4);
  const bool xc_ok = ci0 + 4 * xcq < a.kc;
  // dy items: co quad fixed per thread across its DS items
  const int dcq = tid % (COB / 4);
  const bool dc_ok = co0 + 4 * dcq < a.nb;

  float4 xv[XS][10];
  float4 dv[DS][8];
  float4 colacc = make_float4(0.f, 0.f, 0.f, 0.f);

  auto load = [&](int t) {
    const int b = t / (tiles_x * tiles_y);
    const int trem = t - b * tiles_x * tiles_y;
    const int oy0 = (trem / tiles_x) * TT_H, ox0 = (trem % tiles_x) * TT_W;
#pragma unroll
    for (int j = 0; j < XS; ++j) {
      const int q = tid + 256 * j;
      const int half = (q / (CIB / 4)) & 1, hy = q / (CIB / 2);
      const int iy = oy0 - a.pt + hy;
      const bool rok = q < XQ && xc_ok && (unsigned)iy < (unsigned)a.h;
      const int ix0 = ox0 - a.pl + 8 * half;
      const int base = ((b * a.h + iy) * a.w + ix0) * a.lda + ci0 + 4 * xcq;
#pragma unroll
      for (int e = 0; e < 10; ++e) {
        const bool ok = rok && (unsigned)(ix0 + e) < (unsigned)a.w;
        xv[j][e] = bload4(rx, ok ? (uint32_t)((base + e * a.lda) * 4) : kOOB);
      }
    }
#pragma unroll
    for (int j = 0; j < DS; ++j) {
      const int o = (tid + 256 * j) / (COB / 4);
      const int oy = oy0 + (o >> 1), ox = ox0 + 8 * (o & 1);
      const bool rok = dc_ok && oy < a.ho;
      const int base = ((b * a.ho + oy) * a.wo + ox) * a.ldb + co0 + 4 * dcq;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = rok && ox + e < a.wo;
        dv[j][e] = bload4(rd, ok ? (uint32_t)((base + e * a.ldb) * 4) : kOOB);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < XS; ++j) {
      const int q = tid + 256 * j;
      if (q < XQ) {
        const int half = (q / (CIB / 4)) & 1, hy = q / (CIB / 2);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const float4* v = &xv[j][s];
          const uint4 r0 = pack_bf16x8(make_float4(v[0].x, v[1].x, v[2].x, v[3].x),
                                       make_float4(v[4].x, v[5].x, v[6].x, v[7].x));
          const uint4 r1 = pack_bf16x8(make_float4(v[0].y, v[1].y, v[2].y, v[3].y),
                                       make_float4(v[4].y, v[5].y, v[6].y, v[7].y));
          const uint4 r2 = pack_bf16x8(make_float4(v[0].z, v[1].z, v[2].z, v[3].z),
                                       make_float4(v[4].z, v[5].z, v[6].z, v[7].z));
          const uint4 r3 = pack_bf16x8(make_float4(v[0].w, v[1].w, v[2].w, v[3].w),
                                       make_float4(v[4].w, v[5].w, v[6].w, v[7].w));
          const int ci = 4 * xcq;
          uint4* blk = &Xs[buf][(s * HH + hy) * CIB * 2];
          blk[xrow(ci) * 2 + (half ^ xoct(ci))] = r0;
          blk[xrow(ci + 1) * 2 + (half ^ xoct(ci + 1))] = r1;
          blk[xrow(ci + 2) * 2 + (half ^ xoct(ci + 2))] = r2;
          blk[xrow(ci + 3) * 2 + (half ^ xoct(ci + 3))] = r3;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < DS; ++j) {
      const int o = (tid + 256 * j) / (COB / 4);
      const float4* v = dv[j];
      const uint4 r0 = pack_bf16x8(make_float4(v[0].x, v[1].x, v[2].x, v[3].x),
                                   make_float4(v[4].x, v[5].x, v[6].x, v[7].x));
      const uint4 r1 = pack_bf16x8(make_float4(v[0].y, v[1].y, v[2].y, v[3].y),
                                   make_float4(v[4].y, v[5].y, v[6].y, v[7].y));
      const uint4 r2 = pack_bf16x8(make_float4(v[0].z, v[1].z, v[2].z, v[3].z),
                                   make_float4(v[4].z, v[5].z, v[6].z, v[7].z));
      const uint4 r3 = pack_bf16x8(make_float4(v[0].w, v[1].w, v[2].w, v[3].w),
                                   make_float4(v[4].w, v[5].w, v[6].w, v[7].w));
      const int co = 4 * dcq;
      Ds[buf][(co + 0) * 16 + (o ^ dsw(co + 0))] = r0;
      Ds[buf][(co + 1) * 16 + (o ^ dsw(co + 1))] = r1;
      Ds[buf][(co + 2) * 16 + (o ^ dsw(co + 2))] = r2;
      Ds[buf][(co + 3) * 16 + (o ^ dsw(co + 3))] = r3;
      if (do_colsum) {
#pragma unroll
        for (int e = 0; e < 8; ++e) add4(colacc, v[e]);
      }
    }
  };

  f32x16 acc[KS * KS];
#pragma unroll
  for (int t = 0; t < KS * KS; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const int wci0 = (wave / WAVES_CO) * 32;
  const int wco0 = (wave % WAVES_CO) * 32;
  const int lrow = lane & 31, lk = lane >> 5;
  const int a_base = xrow(wci0 + lrow) * 2 + (lk ^ xoct(wci0 + lrow));
  const int b_base = (wco0 + lrow) * 16;
  const int b_sw = dsw(wco0 + lrow);

  if (steps > 0) {
    load(t_begin);
    store(0);
  }
  __syncthreads();
  for (int i = 0; i < steps; ++i) {
    const int buf = i & 1;
    const bool more = i + 1 < steps;
    if (more) load(t_begin + i + 1);
    if (PF) {
      auto afrag = [&](int row, int s) {
        return __builtin_bit_cast(bf16x8, Xs[buf][(s * HH + row) * CIB * 2 + a_base]);
      };
      auto bfrag = [&](int kk) {
        return __builtin_bit_cast(bf16x8, Ds[buf][b_base + ((2 * kk + lk) ^ b_sw)]);
      };
      bf16x8 bvs[TT_H], af[HH][KS];
      bvs[0] = bfrag(0);
#pragma unroll
      for (int row = 0; row < KS + 1; ++row)
#pragma unroll
        for (int s = 0; s < KS; ++s) af[row][s] = afrag(row, s);
      // the scheduler would otherwise sink every read to its first MFMA (one B read behind a
      // full lgkmcnt(0) wait per output row): sched_barrier fences keep the reads of output
      // row kk + 1's B and of x row kk + 4 ahead of row kk's 9 MFMAs
#pragma unroll
      for (int kk = 0; kk < TT_H; ++kk) {
        if (kk + 1 < TT_H) bvs[kk + 1] = bfrag(kk + 1);
        if (kk + KS + 1 < HH) {                   // x row kk + 4: first used at kk + 2
#pragma unroll
          for (int s = 0; s < KS; ++s) af[kk + KS + 1][s] = afrag(kk + KS + 1, s);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < KS; ++r)
#pragma unroll
          for (int s = 0; s < KS; ++s)
            acc[r * KS + s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kk + r][s], bvs[kk],
                                                                      acc[r * KS + s], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < TT_H; ++kk) {
        const bf16x8 bv = __builtin_bit_cast(bf16x8, Ds[buf][b_base + ((2 * kk + lk) ^ b_sw)]);
#pragma unroll
        for (int r = 0; r < KS; ++r)
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const bf16x8 av = __builtin_bit_cast(
                bf16x8, Xs[buf][(s * HH + kk + r) * CIB * 2 + a_base]);
            acc[r * KS + s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[r * KS + s], 0, 0, 0);
          }
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }

  // ---- raw partial sums into this K slice's slab (+ bias column sums in row M)
  float* S = a.slab + (int64_t)split * a.split_stride;
  if (do_colsum) {
    if (DS > 0) {
      const int g = tid / (COB / 4);
      csum[g][4 * dcq] = colacc.x;
      csum[g][4 * dcq + 1] = colacc.y;
      csum[g][4 * dcq + 2] = colacc.z;
      csum[g][4 * dcq + 3] = colacc.w;
    }
    __syncthreads();
    if (tid < COB && co0 + tid < a.N) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < NG; ++g) v += csum[g][tid];
      S[(int64_t)a.M * a.slab_ld + co0 + tid] = v;
    }
  }
  const int n = co0 + wco0 + lrow;
  if (n < a.N) {
#pragma unroll
    for (int t = 0; t < KS * KS; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = ci0 + wci0 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (ci < a.kc) S[((int64_t)t * a.kc + ci) * a.slab_ld + n] = acc[t][r];
      }
  }
}

// ---- fp32 weight gradient on bf16 MFMA by the three-term split, 3x3 stride 1 ------------
// dW[r][s][ci][co] = sum_p x(p + (r, s) - pad)[ci] . dy(p)[co] with both operands split
// exactly into hi + mid + lo bf16 terms and the six products of conv_tile_x3.  A workgroup
// (12 waves) owns CIB = 32 input x COB = 128 output channels for all 9 taps (wave = 32 ci x
// 32 co x the 3 taps of one kernel row: 48 accumulator registers, so three waves fit per
// SIMD) and walks XH x 16 output-pixel tiles of its K slice (XH = 8; 4 for the 64-channel
// input blocks, whose halo is twice as wide).  The x halo ((XH + 2) rows x 18 px) is staged once
// per tile as three split planes x three copies shifted by
// s = 0, 1, 2 pixels (aligned 16-byte A fragments, the swizzles of conv_wgrad_tile_bf16);
// it is single-buffered (92 / 110 KB) and register-staged one tile ahead.  dy never enters LDS:
// a lane loads its B fragment (8 pixels of one channel, coalesced across the 32 channels of
// a pixel) straight from L2 one k-step ahead and splits it in registers (the three kernel-row
// waves of a channel block read the same dy lines).  Output: the split-K slabs of the other wgrad kernels.
// conv_wgrad_tile_x3 pixel tiles: XH rows x 16 px (8 rows where the halo fits LDS)
int wgx3_rows(int cfg) { return cfg == 2 || cfg == 3 ? 4 : 8; }

__device__ __forceinline__ void split3x8(const float* v, bf16x8& h, bf16x8& m, bf16x8& l) {
  uint2 h0, m0, l0, h1, m1, l1;
  split3x4(make_float4(v[0], v[1], v[2], v[3]), h0, m0, l0);
  split3x4(make_float4(v[4], v[5], v[6], v[7]), h1, m1, l1);
  h = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
  m = __builtin_bit_cast(bf16x8, make_uint4(m0.x, m0.y, m1.x, m1.y));
  l = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
}

// ---- the stem's weight gradient (7x7 stride 2, 4 padded input channels, 64 outputs) on the
// split-bf16 MFMA.  dW[(r, s, ci)][co] = sum over output pixels p of
// x[2 py + r - pt][2 px + s - pl][ci] * dz[p][co]: GEMM M = (r, s, ci) over the 147 real rows
// (10 M tiles of 16), N = 64, K = output pixels.  The implicit GEMM gathers 49 taps x 16 bytes
// per pixel from global memory for every K step; here a workgroup owns 4 x 32-pixel output
// tiles: the tile's input halo (13 rows x 69 pixels x 4 channels) goes to LDS once, fp32,
// split by column parity ([row][ci][parity][col / 2]) so that kernel column s of 8 consecutive
// output pixels is 8 consecutive floats at a per-lane offset (each lane gathers its own A row
// with ds_read_b32, so the rows need no (r, s, ci) padding); it is prefetched one tile ahead
// into a second buffer.  Each 32-pixel output row is one K chunk whose dz (32 px x 64 co) is
// loaded two chunks ahead, cut into hi / mid / lo bf16 planes in B-fragment order ([plane]
// [k octet][co], conflict-free ds_read_b128) and double-buffered.  Wave w (5 waves) owns M
// tiles 2w, 2w + 1 x 4 N tiles, six v_mfma_f32_16x16x32_bf16 per fragment pair (rows 147-159
// compute discarded values).  Workgroups (three per CU) are persistent over a contiguous range
// of a.k_per_split tiles (a.K tiles in all) and write one split-K slab each (with a.colsum the
// bias column sums in slab row 196), reduced by wgrad_reduce_kernel.  NP = 1 is the bf16 path:
// the halo rows and dz rounded to bf16 (round to nearest even, as conv_wgrad_bf16 rounds its
// operands), one MFMA per fragment pair.
constexpr int SW_TH = 4, SW_TW = 32, SW_HH = 2 * SW_TH + 5, SW_HX = 2 * SW_TW + 5, SW_HC = 36;
constexpr int SW_HP = SW_HH * 4 * 2 * SW_HC;             // floats per halo buffer
constexpr int SW_NW = 5, SW_NT = 64 * SW_NW;
constexpr int SW_HQ = (SW_HH * SW_HX + SW_NT - 1) / SW_NT; // halo pixels per thread
constexpr int SW_WGS_PER_CU = 3;

// FUSED (round 5): the stem's backward in one kernel.  conv1 -> layer1_bn -> ReLU feeds out0 and
// the max-pool (model.py:12-17); dz = t * s with t = relu'(y) (g + the pooled gradient at the
// first maximum of each 2 x 2 window) and s = gamma / sqrt(var + eps) -- misc.hip's
// maxpool_bn_act_bwd_partial math -- is formed while each dz chunk is staged, from y (this row
// and its window partner row), g and the pooled gradient, so dz (the encoder's largest tensor)
// is never written and read back.  The BN sums ride along: slab rows 196 (sum t) and 197
// (sum t zhat, zhat = (y - beta) / gamma where y > 0) instead of the bias column sums.
template <int NP, bool FUSED = false>
__global__ __launch_bounds__(SW_NT, 3) void conv_wgrad_stem_x3(GemmArgs a) {
  constexpr int NT = SW_NT;
  static_assert(NP == 3 || NP == 1, "three split planes (fp32) or one (bf16)");
  __shared__ float Hs[2][SW_HP];                       // 2 x 14.6 KB
  __shared__ uint4 Ds[2][NP * 4 * 64];                 // 2 x 12 KB (4 KB for NP = 1)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int split = xcd_remap(blockIdx.x, gridDim.x);
  const int t_begin = split * a.k_per_split;
  const int t_end = min(a.K, t_begin + a.k_per_split);
  const int ntiles = max(0, t_end - t_begin);
  const int nchunks = ntiles * SW_TH;
  const int tiles_x = (a.wo + SW_TW - 1) / SW_TW, tiles_y = (a.ho + SW_TH - 1) / SW_TH;
  const rsrc_t rx = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rd = make_rsrc(a.B, a.b_bytes);
  auto tile_of = [&](int t, int& b, int& oy0, int& ox0) {
    b = t / (tiles_x * tiles_y);
    const int rem = t - b * tiles_x * tiles_y;
    oy0 = (rem / tiles_x) * SW_TH;
    ox0 = (rem % tiles_x) * SW_TW;
  };

  // ---- dz (waves 0-3): thread (co, k octet) loads 8 consecutive pixels of one channel (each
  // load instruction reads 64 channels of 4 pixels: 4 x 64-byte segments); two chunks in flight
  const int d_co = tid & 63, d_kg = (tid >> 6) & 3;
  const bool d_on = tid < 256 && d_co < a.N;
  const uint32_t d_step = (uint32_t)a.ldb * 4;        // bytes between consecutive pixels
  float dv[2][8], csum = 0.f;
  // FUSED: raw inputs of two chunks in flight (y of the row and of its window partner, g, the
  // four pooled gradients of the octet), the BN scale / shift of this lane's channel, sums
  float fy[FUSED ? 2 : 1][8], fp[FUSED ? 2 : 1][8], fg[FUSED ? 2 : 1][8], fd[FUSED ? 2 : 1][4];
  float f_sc = 0.f, f_bt = 0.f, f_ig = 0.f, f_st = 0.f, f_stz = 0.f;
  const rsrc_t ry = make_rsrc(FUSED ? a.st_y : a.B, FUSED ? a.b_bytes : 0);
  const rsrc_t rg = make_rsrc(FUSED && a.st_g ? a.st_g : a.B, FUSED && a.st_g ? a.b_bytes : 0);
  const rsrc_t rp = make_rsrc(FUSED ? a.st_dyp : a.B, FUSED ? a.b_bytes / 4 : 0);
  if constexpr (FUSED) {
    if (d_on) {
      const float gm = a.bn_g[d_co];
      f_sc = gm * rsqrtf(a.bn_v[d_co] + a.bn_eps);
      f_bt = a.bn_b[d_co];
      f_ig = 1.f / gm;
    }
  }
  auto load_dz = [&](int c, float* v, int set) {
    int b, oy0, ox0;
    tile_of(t_begin + c / SW_TH, b, oy0, ox0);
    const int oy = oy0 + c % SW_TH, px0 = ox0 + 8 * d_kg;
    const int lim = d_on && oy < a.ho ? a.wo - px0 : 0;   // pixels of this octet in the row
    const uint32_t base = (uint32_t)((((int64_t)b * a.ho + oy) * a.wo + px0) * a.ldb + d_co) * 4;
    if constexpr (FUSED) {
      // (even ho, wo and 4 x 32 tiles: the partner row oy ^ 1 and the octet's 4 windows are
      // inside the image whenever the row is)
      const uint32_t pbase = (uint32_t)((((int64_t)b * a.ho + (oy ^ 1)) * a.wo + px0) * a.ldb + d_co) * 4;
      const int pw = a.wo / 2;
      const uint32_t dbase =
          (uint32_t)((((int64_t)b * (a.ho / 2) + (oy >> 1)) * pw + (px0 >> 1)) * a.ldb + d_co) * 4;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        fy[set][e] = bload1(ry, e < lim ? base + e * d_step : kOOB);
        fp[set][e] = bload1(ry, e < lim ? pbase + e * d_step : kOOB);
        fg[set][e] = bload1(rg, e < lim ? base + e * d_step : kOOB);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) fd[set][e] = bload1(rp, 2 * e < lim ? dbase + e * d_step : kOOB);
      (void)v;
      return;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bload1(rd, e < lim ? base + e * d_step : kOOB);
  };
  // FUSED: dz of the chunk from its raw inputs; `odd`: the row is the odd row of its windows
  auto form_dz = [&](int set, bool odd, float* v) {
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      // window corners k = 2 (row parity) + (column parity), first maximum, strict >
      float wy[4];
      wy[odd ? 2 : 0] = fy[set][2 * e2];
      wy[odd ? 3 : 1] = fy[set][2 * e2 + 1];
      wy[odd ? 0 : 2] = fp[set][2 * e2];
      wy[odd ? 1 : 3] = fp[set][2 * e2 + 1];
      int bk = 0;
      float mx = wy[0];
#pragma unroll
      for (int k = 1; k < 4; ++k)
        if (wy[k] > mx) bk = k, mx = wy[k];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = (odd ? 2 : 0) + u;
        const float yk = fy[set][2 * e2 + u];
        const float t = yk > 0.f ? fg[set][2 * e2 + u] + (k == bk ? fd[set][e2] : 0.f) : 0.f;
        v[2 * e2 + u] = t * f_sc;
        f_st += t;
        f_stz += t * ((yk - f_bt) * f_ig);
      }
    }
  };
  auto store_dz = [&](int buf, const float* v) {
    if (tid >= 256) return;
    if (NP == 1) {
      Ds[buf][d_kg * 64 + d_co] = pack_bf16x8(make_float4(v[0], v[1], v[2], v[3]),
                                             make_float4(v[4], v[5], v[6], v[7]));
    } else {
      bf16x8 h, m, l;
      split3x8(v, h, m, l);
      Ds[buf][(0 * 4 + d_kg) * 64 + d_co] = __builtin_bit_cast(uint4, h);
      Ds[buf][((NP / 2) * 4 + d_kg) * 64 + d_co] = __builtin_bit_cast(uint4, m);
      Ds[buf][((NP - 1) * 4 + d_kg) * 64 + d_co] = __builtin_bit_cast(uint4, l);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) csum += v[e];
  };
  // ---- input halo ([row][ci][parity][col / 2] fp32), loaded one tile ahead
  float4 hv[SW_HQ];
  auto load_halo = [&](int t) {
    int b, oy0, ox0;
    tile_of(t, b, oy0, ox0);
    const int iy0 = 2 * oy0 - a.pt, ix0 = 2 * ox0 - a.pl;
#pragma unroll
    for (int k = 0; k < SW_HQ; ++k) {
      const int q = tid + NT * k;
      const int hy = q / SW_HX, hx = q - hy * SW_HX;
      const int iy = iy0 + hy, ix = ix0 + hx;
      const bool ok = q < SW_HH * SW_HX && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
      hv[k] = bload4(rx, ok ? (uint32_t)((((int64_t)b * a.h + iy) * a.w + ix) * a.lda * 4) : kOOB);
    }
  };
  auto store_halo = [&](int hb) {
#pragma unroll
    for (int k = 0; k < SW_HQ; ++k) {
      const int q = tid + NT * k;
      if (q >= SW_HH * SW_HX) continue;
      const int hy = q / SW_HX, hx = q - hy * SW_HX;
      float* dst = Hs[hb] + hy * 8 * SW_HC + (hx & 1) * SW_HC + (hx >> 1);
      dst[0] = hv[k].x;
      dst[2 * SW_HC] = hv[k].y;
      dst[4 * SW_HC] = hv[k].z;
      dst[6 * SW_HC] = hv[k].w;
    }
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
  // A row of this lane in M tile mt: m = 16 (2 wave + mt) + l16 = (tap = r * 7 + s) * 3 + ci
  const int l16 = lane & 15, kg = lane >> 4;
  int a_off[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int m = min(16 * (2 * wave + mt) + l16, 146);
    const int tap = m / 3, ci = m - 3 * tap, r = tap / 7, sc = tap - 7 * r;
    a_off[mt] = (r * 8 + ci * 2 + (sc & 1)) * SW_HC + 8 * kg + (sc >> 1);
  }

  if (nchunks > 0) {
    load_halo(t_begin);
    load_dz(0, dv[0], 0);
    if (nchunks > 1) load_dz(1, dv[1], 1);
    store_halo(0);
  }
  // chunk c uses dz register set c & 1 (static: the body is instantiated for both sets)
  auto chunk = [&](int c, float* dvc, int set) {
    const int j = c % SW_TH, tl = c / SW_TH;
    const int buf = c & 1;
    // The halo of tile tl + 1 is stored into the other buffer at j = 1: every wave passed this
    // chunk's barrier, so none still reads that buffer (tile tl - 1, last read at chunk c - 2).
    if (j == 0 && tl + 1 < ntiles) load_halo(t_begin + tl + 1);
    if constexpr (FUSED) {
      if (tid < 256) form_dz(set, (j & 1) != 0, dvc);   // tiles start at even rows
    }
    store_dz(buf, dvc);
    __syncthreads();                               // this chunk's dz (and its tile's halo)
    if (c + 2 < nchunks) load_dz(c + 2, dvc, set); // two chunks in flight
    if (j == 1 && tl + 1 < ntiles) store_halo((tl + 1) & 1);
    const float* hrow = Hs[tl & 1] + 2 * j * 8 * SW_HC;
    bf16x8 av[2][NP];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = hrow[a_off[mt] + e];
      if (NP == 1)
        av[mt][0] = __builtin_bit_cast(bf16x8, pack_bf16x8(make_float4(v[0], v[1], v[2], v[3]),
                                                           make_float4(v[4], v[5], v[6], v[7])));
      else
        split3x8(v, av[mt][0], av[mt][NP / 2], av[mt][NP - 1]);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      bf16x8 bv[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p)
        bv[p] = __builtin_bit_cast(bf16x8, Ds[buf][(p * 4 + kg) * 64 + nt * 16 + l16]);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        f32x4 x = acc[mt][nt];
        if (NP == 3) {
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[mt][NP - 1], bv[0], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[mt][0], bv[NP - 1], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[mt][NP / 2], bv[NP / 2], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[mt][NP / 2], bv[0], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[mt][0], bv[NP / 2], x, 0, 0, 0);
        }
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[mt][0], bv[0], x, 0, 0, 0);
      }
    }
  };
  for (int c = 0; c < nchunks; c += 2) {
    chunk(c, dv[0], 0);
    if (c + 1 < nchunks) chunk(c + 1, dv[1], 1);
  }

  // ---- this workgroup's slab: lane's value rr of (mt, nt) is row m = 16 (2 wave + mt) +
  // 4 kg + rr = tap * 3 + ci, column 16 nt + l16; slab row = tap * 4 + ci
  float* slab = a.slab + (int64_t)split * a.split_stride;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = 16 * (2 * wave + mt) + 4 * kg + rr;
      if (m >= 147) continue;
      const int tap = m / 3, ci = m - 3 * tap;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int co = nt * 16 + l16;
        if (co < a.N) slab[(int64_t)(tap * 4 + ci) * a.slab_ld + co] = acc[mt][nt][rr];
      }
    }
  if (FUSED) {                                     // BN sums (rows 196, 197), fixed order
    float* Cs = reinterpret_cast<float*>(&Ds[0][0]);
    __syncthreads();                               // every wave is done with Ds
    if (tid < 256) {
      Cs[d_kg * 64 + d_co] = f_st;
      Cs[256 + d_kg * 64 + d_co] = f_stz;
    }
    __syncthreads();
    if (tid < 128 && (tid & 63) < a.N) {
      const int o = (tid >> 6) * 256, cc = tid & 63;
      slab[(int64_t)(196 + (tid >> 6)) * a.slab_ld + cc] =
          (Cs[o + cc] + Cs[o + 64 + cc]) + (Cs[o + 128 + cc] + Cs[o + 192 + cc]);
    }
  } else if (a.colsum) {                           // bias: column sums of dz, fixed order
    float* Cs = reinterpret_cast<float*>(&Ds[0][0]);
    __syncthreads();                               // every wave is done with Ds
    if (tid < 256) Cs[d_kg * 64 + d_co] = csum;
    __syncthreads();
    if (tid < 64 && tid < a.N)
      slab[(int64_t)196 * a.slab_ld + tid] = (Cs[tid] + Cs[64 + tid]) + (Cs[128 + tid] + Cs[192 + tid]);
  }
}

// The fused stem backward's BN parameter gradients: per channel the slab rows 196 (sum t) and
// 197 (sum t zhat) of every split, in split order (four lane groups over contiguous quarters,
// then the quarters in order): dbeta (+)= sum t, dgamma (+)= sum t zhat, dbias (+)= s sum t.
__global__ __launch_bounds__(256) void stem_bn_final(const float* __restrict__ slab, int splits,
                                                     int64_t split_stride, int ld, int c,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ var, float eps,
                                                     float* __restrict__ dgamma,
                                                     float* __restrict__ dbeta,
                                                     float* __restrict__ dbias, int accum) {
  __shared__ float red[2][4][64];
  const int co = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int s0 = (int)((int64_t)g * splits / 4), s1 = (int)((int64_t)(g + 1) * splits / 4);
  float st = 0.f, stz = 0.f;
  if (co < c) {
    for (int sp = s0; sp < s1; ++sp) {
      st += slab[sp * split_stride + 196 * (int64_t)ld + co];
      stz += slab[sp * split_stride + 197 * (int64_t)ld + co];
    }
  }
  red[0][g][co] = st;
  red[1][g][co] = stz;
  __syncthreads();
  if (g != 0 || co >= c) return;
  st = (red[0][0][co] + red[0][1][co]) + (red[0][2][co] + red[0][3][co]);
  stz = (red[1][0][co] + red[1][1][co]) + (red[1][2][co] + red[1][3][co]);
  const float db = st * gamma[co] * rsqrtf(var[co] + eps);
  if (dbeta) dbeta[co] = accum ? dbeta[co] + st : st;
  if (dgamma) dgamma[co] = accum ? dgamma[co] + stz : stz;
  if (dbias) dbias[co] = accum ? dbias[co] + db : db;
}

template <int WAVES_CI, int WAVES_CO, int WAVES_R, int XH>
__global__ __launch_bounds__(64 * WAVES_CI * WAVES_CO * WAVES_R, 1) void conv_wgrad_tile_x3(GemmArgs a) {
  constexpr int NT = 64 * WAVES_CI * WAVES_CO * WAVES_R;
  static_assert(WAVES_R == 3, "one kernel row per wave group");
  constexpr int CIB = 32 * WAVES_CI, COB = 32 * WAVES_CO, KS = 3, HH = XH + KS - 1, NP = 3;
  constexpr int XQ = HH * KS * 2 * (CIB / 4), XS = (XQ + NT - 1) / NT;   // (hy, s, half, ci quad)
  constexpr int PL = KS * HH * CIB * 2;                              // uint4 per plane
  __shared__ uint4 Xs[NP * PL];

  auto xrow = [](int ci) { return ci ^ ((ci >> 2) & 2); };
  auto xoct = [](int ci) { return (ci >> 4) & 1; };
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_co = tile % a.n_tiles;
  const int tile_ci = tile / a.n_tiles;
  const int ci0 = tile_ci * CIB, co0 = tile_co * COB;
  const int t_begin = split * a.k_per_split;
  const int t_end = min(a.K, t_begin + a.k_per_split);
  const int steps = max(0, t_end - t_begin);
  const int tiles_x = (a.wo + TT_W - 1) / TT_W, tiles_y = (a.ho + XH - 1) / XH;
  const rsrc_t rx = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rd = make_rsrc(a.B, a.b_bytes);
  const int wr = wave / (WAVES_CI * WAVES_CO);            // this wave's kernel row
  const int wci0 = ((wave / WAVES_CO) % WAVES_CI) * 32;
  const int wco0 = (wave % WAVES_CO) * 32;
  const int lrow = lane & 31, lk = lane >> 5;
  const bool do_colsum = a.colsum && tile_ci == 0 && wci0 == 0 && wr == 0;

  // ---- x halo slots (channel quad fastest: coalesced 16-B lanes of one pixel)
  const int xcq = tid % (CIB / 4);
  const bool xc_ok = ci0 + 4 * xcq < a.kc;
  // slot q: channel quad (fastest: coalesced), pixel octet half, shift s, halo row hy; it
  // loads the 8 pixels its shifted copy needs and writes 4 channel rows x 3 planes
  float4 xv[XS][8];
  auto load_x = [&](int t) {
    const int b = t / (tiles_x * tiles_y);
    const int trem = t - b * tiles_x * tiles_y;
    const int oy0 = (trem / tiles_x) * XH, ox0 = (trem % tiles_x) * TT_W;
    const int iy0 = oy0 - a.pt, ix00 = ox0 - a.pl;
#pragma unroll
    for (int j = 0; j < XS; ++j) {
      const int q = tid + NT * j;
      const int r2 = q / (CIB / 4);
      const int half = r2 & 1, s = (r2 >> 1) % KS, hy = (r2 >> 1) / KS;
      const int iy = iy0 + hy;
      const bool rok = q < XQ && xc_ok && (unsigned)iy < (unsigned)a.h;
      const int ix0 = ix00 + 8 * half + s;
      const int base = ((b * a.h + iy) * a.w + ix0) * a.lda + ci0 + 4 * xcq;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = rok && (unsigned)(ix0 + e) < (unsigned)a.w;
        xv[j][e] = bload4(rx, ok ? (uint32_t)((base + e * a.lda) * 4) : kOOB);
      }
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int j = 0; j < XS; ++j) {
      const int q = tid + NT * j;
      if (q < XQ) {
        const int r2 = q / (CIB / 4);
        const int half = r2 & 1, s = (r2 >> 1) % KS, hy = (r2 >> 1) / KS;
        const int ci = 4 * xcq;
        uint4* blk = &Xs[(s * HH + hy) * CIB * 2];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float v8[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v8[e] = (&xv[j][e].x)[c];
          bf16x8 h, m, l;
          split3x8(v8, h, m, l);
          const int idx = xrow(ci + c) * 2 + (half ^ xoct(ci + c));
          blk[idx] = __builtin_bit_cast(uint4, h);
          blk[PL + idx] = __builtin_bit_cast(uint4, m);
          blk[2 * PL + idx] = __builtin_bit_cast(uint4, l);
        }
      }
    }
  };
  // ---- dy fragment of this lane: output channel co, pixels 8 lk .. 8 lk + 7 of tile row kk
  const int co = co0 + wco0 + lrow;
  const bool co_ok = co < a.nb;
  // Interior dy rows (all 16 pixels and the whole channel block in range) take fixed per-lane
  // offsets plus a uniform scalar offset: no per-load address math or bounds tests.
  const uint32_t dy_lane = (uint32_t)((8 * lk * a.ldb + co) * 4);
  const bool dy_co_full = co0 + COB <= a.nb;
  auto load_dy = [&](float (&dv)[8], int t, int kk) {
    const int b = t / (tiles_x * tiles_y);
    const int trem = t - b * tiles_x * tiles_y;
    const int oy = (trem / tiles_x) * XH + kk, ox0 = (trem % tiles_x) * TT_W;
    if (dy_co_full && oy < a.ho && ox0 + TT_W <= a.wo) {
      const int so = ((b * a.ho + oy) * a.wo + ox0) * a.ldb * 4;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        dv[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              rd, dy_lane + e * a.ldb * 4, so, 0));
      return;
    }
    const int ox = ox0 + 8 * lk;
    const bool rok = co_ok && oy < a.ho;
    const int base = ((b * a.ho + oy) * a.wo + ox) * a.ldb + co;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool ok = rok && ox + e < a.wo;
      dv[e] = bload1(rd, ok ? (uint32_t)((base + e * a.ldb) * 4) : kOOB);
    }
  };

  f32x16 acc[KS];                       // taps (wr, s), s = 0..2
#pragma unroll
  for (int t = 0; t < KS; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const int a_base = xrow(wci0 + lrow) * 2 + (lk ^ xoct(wci0 + lrow));
  float colacc = 0.f;
  float dcur[8], dnext[8];

  if (steps > 0) {
    load_x(t_begin);
    load_dy(dcur, t_begin, 0);
    store_x();
  }
  __syncthreads();
  for (int i = 0; i < steps; ++i) {
    const int t = t_begin + i;
    const bool more = i + 1 < steps;
    if (more) load_x(t + 1);
#pragma unroll
    for (int kk = 0; kk < XH; ++kk) {
      if (kk + 1 < XH) load_dy(dnext, t, kk + 1);
      else if (more) load_dy(dnext, t + 1, 0);
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 bh, bm, bl;
      split3x8(dcur, bh, bm, bl);
      if (do_colsum) {
#pragma unroll
        for (int e = 0; e < 8; ++e) colacc += dcur[e];
      }
      // A fragments one tap ahead of the MFMAs (bounded register footprint)
      bf16x8 fa[2][NP];
      auto load_a = [&](bf16x8 (&f)[NP], int s) {
        const int xa = (s * HH + kk + wr) * CIB * 2 + a_base;
#pragma unroll
        for (int p = 0; p < NP; ++p) f[p] = __builtin_bit_cast(bf16x8, Xs[p * PL + xa]);
      };
      load_a(fa[0], 0);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
          if (s + 1 < KS) load_a(fa[(s + 1) & 1], s + 1);
          __builtin_amdgcn_sched_barrier(0);
          const bf16x8 ah = fa[s & 1][0], am = fa[s & 1][1], al = fa[s & 1][2];
          f32x16 x = acc[s];
          x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, x, 0, 0, 0);
          acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, x, 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) dcur[e] = dnext[e];
    }
    __syncthreads();              // every wave is done with this tile's halo
    if (more) store_x();
    __syncthreads();
  }

  // ---- raw partial sums into this K slice's slab (+ bias column sums in row M)
  float* S = a.slab + (int64_t)split * a.split_stride;
  if (do_colsum) {
    const float v = colacc + __shfl_xor(colacc, 32);
    if (lk == 0 && co < a.N) S[(int64_t)a.M * a.slab_ld + co] = v;
  }
  if (co < a.N) {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = ci0 + wci0 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (ci < a.kc) S[((int64_t)(wr * KS + s) * a.kc + ci) * a.slab_ld + co] = acc[s][r];
      }
  }
}

// ---- conv_wgrad_tile_x3b: the same weight gradient with all 9 taps per wave ---------------
// Wave = 16 MI ci x 16 NJ co x 9 taps on v_mfma_f32_16x16x32_bf16 (MI NJ = 2: 18 accumulator
// tiles, 72 registers): one 32-pixel k-step (two tile rows of 16 px) takes one dy fragment per
// 16-column block (8 pixels of one channel per lane, from L2, split in registers) and feeds it
// to 9 taps x MI row blocks x 6 products: with MI = 2 a loaded and split dy value serves 108
// MFMAs and no other wave loads it (the 3-tap form: 18, three waves splitting the same value).
// Workgroup = WAVES_CI x WAVES_CO waves over CIB = 16 MI WAVES_CI input x COB = 16 NJ WAVES_CO
// output channels; the x halo ((XH + 2) rows x 18 px) is staged once
// per XH x 16 tile as three split planes x three pixel-shifted copies, single-buffered and
// register-staged one tile ahead.  LDS row block (plane, s, hy): 8-channel groups of
// 256 bytes, (ci, octet) in slot (2 (ci & 7) + octet) ^ 2 ((ci >> 3) & 3): the 16x16x32
// A-fragment reads (16 consecutive channels x 2 octets x 2 rows) and the staging stores (8
// lanes = 8 channel quads) are both conflict-free.  Output: the split-K slabs (+ bias row).
__device__ __forceinline__ int wgx3b_slot(int ci, int oct) {
  return (ci >> 3) * 16 + ((2 * (ci & 7) + oct) ^ (((ci >> 3) & 3) << 1));
}

// The body is shared with the bf16 weight gradient (NP = 1: x and dy rounded to bf16 RNE, one
// plane, one MFMA per fragment pair); NP = 3 is the fp32 split.
template <int WAVES_CI, int WAVES_CO, int XH, int MI, int NP>
__device__ __forceinline__ void wgrad_x3b_body(const GemmArgs& a) {
  constexpr int NJ = 2 / MI;
  static_assert(MI * NJ == 2, "18 accumulator tiles per wave");
  static_assert(NP == 1 || NP == 3, "planes");
  constexpr int NT = 64 * WAVES_CI * WAVES_CO;
  constexpr int CIB = 16 * MI * WAVES_CI, COB = 16 * NJ * WAVES_CO, KS = 3, HH = XH + KS - 1;
  static_assert(XH % 2 == 0 && CIB % 32 == 0, "k-steps of 2 tile rows; 8-channel slot groups");
  constexpr int XQ = HH * KS * 2 * (CIB / 4), XS = (XQ + NT - 1) / NT;   // (hy, s, half, ci quad)
  constexpr int RB = CIB * 2;                      // uint4 per (plane, s, hy) row block
  constexpr int PL = KS * HH * RB;                 // uint4 per plane
  static_assert(NT / 64 * 512 * 4 <= NP * PL * 16, "epilogue images fit LDS");
  __shared__ uint4 Xs[NP * PL];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_co = tile % a.n_tiles;
  const int tile_ci = tile / a.n_tiles;
  const int ci0 = tile_ci * CIB, co0 = tile_co * COB;
  const int t_begin = split * a.k_per_split;
  const int t_end = min(a.K, t_begin + a.k_per_split);
  const int steps = max(0, t_end - t_begin);
  const int tiles_x = (a.wo + TT_W - 1) / TT_W, tiles_y = (a.ho + XH - 1) / XH;
  const rsrc_t rx = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rd = make_rsrc(a.B, a.b_bytes);
  const int wci0 = (wave / WAVES_CO) * 16 * MI;
  const int wco0 = (wave % WAVES_CO) * 16 * NJ;
  const int l16 = lane & 15, lq = lane >> 4;

  // ---- x halo slots (channel quad fastest: coalesced 16-byte lanes of one pixel)
  const int xcq = tid % (CIB / 4);
  const bool xc_ok = ci0 + 4 * xcq < a.kc;
  float4 xv[XS][8];
  auto load_x = [&](int t) {
    const int b = t / (tiles_x * tiles_y);
    const int trem = t - b * tiles_x * tiles_y;
    const int oy0 = (trem / tiles_x) * XH, ox0 = (trem % tiles_x) * TT_W;
    const int iy0 = oy0 - a.pt, ix00 = ox0 - a.pl;
#pragma unroll
    for (int j = 0; j < XS; ++j) {
      const int q = tid + NT * j;
      const int r2 = q / (CIB / 4);
      const int half = r2 & 1, s = (r2 >> 1) % KS, hy = (r2 >> 1) / KS;
      const int iy = iy0 + hy;
      const bool rok = q < XQ && xc_ok && (unsigned)iy < (unsigned)a.h;
      const int ix0 = ix00 + 8 * half + s;
      const int base = ((b * a.h + iy) * a.w + ix0) * a.lda + ci0 + 4 * xcq;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = rok && (unsigned)(ix0 + e) < (unsigned)a.w;
        xv[j][e] = bload4(rx, ok ? (uint32_t)((base + e * a.lda) * 4) : kOOB);
      }
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int j = 0; j < XS; ++j) {
      const int q = tid + NT * j;
      if (XQ % NT == 0 || q < XQ) {
        const int r2 = q / (CIB / 4);
        const int half = r2 & 1, s = (r2 >> 1) % KS, hy = (r2 >> 1) / KS;
        uint4* blk = &Xs[(s * HH + hy) * RB];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float v8[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v8[e] = (&xv[j][e].x)[c];
          const int idx = wgx3b_slot(4 * xcq + c, half);
          if constexpr (NP == 1) {
            blk[idx] = pack_bf16x8(make_float4(v8[0], v8[1], v8[2], v8[3]),
                                   make_float4(v8[4], v8[5], v8[6], v8[7]));
          } else {
            bf16x8 h, m, l;
            split3x8(v8, h, m, l);
            blk[idx] = __builtin_bit_cast(uint4, h);
            blk[PL + idx] = __builtin_bit_cast(uint4, m);
            blk[2 * PL + idx] = __builtin_bit_cast(uint4, l);
          }
        }
      }
    }
  };
  // ---- dy fragments: column blocks j < NJ (co = co0 + wco0 + 16 j + l16), pixels
  // 8 (lq & 1) .. + 7 of tile row 2 kk + (lq >> 1)
  int co[NJ];
  bool co_ok[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    co[j] = co0 + wco0 + 16 * j + l16;
    co_ok[j] = co[j] < a.nb;
  }
  const int prow = lq >> 1, pcol = 8 * (lq & 1);
  // Interior dy rows (the whole 16-pixel row and channel block in range) take fixed per-lane
  // offsets plus a uniform scalar offset: no per-load address math or bounds tests.
  const bool dy_co_full = co0 + COB <= a.nb;
  const uint32_t dy_lane = (uint32_t)(((prow * a.wo + pcol) * a.ldb + co0 + wco0 + l16) * 4);
  auto load_dy = [&](float (&dv)[NJ][8], int t, int kk) {
    const int b = t / (tiles_x * tiles_y);
    const int trem = t - b * tiles_x * tiles_y;
    const int oyr = (trem / tiles_x) * XH + 2 * kk, ox0 = (trem % tiles_x) * TT_W;
    if (dy_co_full && oyr + 1 < a.ho && ox0 + TT_W <= a.wo) {
      const int so = ((b * a.ho + oyr) * a.wo + ox0) * a.ldb * 4;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          dv[j][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                   rd, dy_lane + (e * a.ldb + 16 * j) * 4, so, 0));
      return;
    }
    const int oy = oyr + prow, ox = ox0 + pcol;
    const bool rok = oy < a.ho;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int base = ((b * a.ho + oy) * a.wo + ox) * a.ldb + co[j];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = rok && co_ok[j] && ox + e < a.wo;
        dv[j][e] = bload1(rd, ok ? (uint32_t)((base + e * a.ldb) * 4) : kOOB);
      }
    }
  };

  f32x4 acc[KS * KS][MI][NJ];
#pragma unroll
  for (int t = 0; t < KS * KS; ++t)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][i][j][r] = 0.f;
  // A fragment of tap (r, s) at k-step kk, row block i: row block (s, 2 kk + prow + r), this
  // lane's slot for channel wci0 + 16 i + l16
  int a_lane[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) a_lane[i] = prow * RB + wgx3b_slot(wci0 + 16 * i + l16, lq & 1);
  const bool do_colsum = a.colsum && tile_ci == 0 && wci0 == 0;
  float colacc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) colacc[j] = 0.f;
  float dcur[NJ][8], dnext[NJ][8];

  if (steps > 0) {
    load_x(t_begin);
    load_dy(dcur, t_begin, 0);
    store_x();
  }
  __syncthreads();
  for (int i = 0; i < steps; ++i) {
    const int t = t_begin + i;
    const bool more = i + 1 < steps;
    if (more) load_x(t + 1);
#pragma unroll
    for (int kk = 0; kk < XH / 2; ++kk) {
      if (kk + 1 < XH / 2) load_dy(dnext, t, kk + 1);
      else if (more) load_dy(dnext, t + 1, 0);
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 bh[NJ], bm[NJ], bl[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (NP == 1)
          bh[j] = __builtin_bit_cast(bf16x8, pack_bf16x8(make_float4(dcur[j][0], dcur[j][1], dcur[j][2], dcur[j][3]),
                                                         make_float4(dcur[j][4], dcur[j][5], dcur[j][6], dcur[j][7])));
        else
          split3x8(dcur[j], bh[j], bm[j], bl[j]);
      }
      if (do_colsum) {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) colacc[j] += dcur[j][e];
      }
      // A fragments one tap ahead of the MFMAs (bounded register footprint)
      bf16x8 fa[2][MI][NP];
      auto load_a = [&](bf16x8 (&f)[MI][NP], int tap) {
        const int r = tap / KS, s = tap % KS;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int xa = (s * HH + 2 * kk + r) * RB + a_lane[i];
#pragma unroll
          for (int p = 0; p < NP; ++p) f[i][p] = __builtin_bit_cast(bf16x8, Xs[p * PL + xa]);
        }
      };
      load_a(fa[0], 0);
#pragma unroll
      for (int tap = 0; tap < KS * KS; ++tap) {
        if (tap + 1 < KS * KS) load_a(fa[(tap + 1) & 1], tap + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          if constexpr (NP == 1) {
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              acc[tap][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[tap & 1][i][0], bh[j],
                                                                       acc[tap][i][j], 0, 0, 0);
            continue;
          } else {
          const bf16x8 ah = fa[tap & 1][i][0], am = fa[tap & 1][i][1], al = fa[tap & 1][i][2];
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            f32x4 x = acc[tap][i][j];
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm[j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh[j], x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm[j], x, 0, 0, 0);
            acc[tap][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j], x, 0, 0, 0);
          }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) dcur[j][e] = dnext[j][e];
    }
    __syncthreads();              // every wave is done with this tile's halo
    if (more) store_x();
    __syncthreads();
  }

  // ---- raw partial sums into this K slice's slab (+ bias column sums in row M)
  float* S = a.slab + (int64_t)split * a.split_stride;
  if (do_colsum) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float v = colacc[j] + __shfl_xor(colacc[j], 16);
      v += __shfl_xor(v, 32);
      if (lq == 0 && co[j] < a.N) S[(int64_t)a.M * a.slab_ld + co[j]] = v;
    }
  }
  // (16 MI) x (16 NJ) blocks per tap through a private 2 KB LDS image (the loop's last barrier
  // freed the halo), back as float4 rows of 4 NJ column quads: slab rows tap * kc + ci
  constexpr int EW = 16 * NJ, LPR = 4 * NJ, RPI = 64 / LPR;
  float* E = reinterpret_cast<float*>(Xs) + wave * 512;
  const int c4 = lane % LPR, rr = lane / LPR;
  const bool vec = a.vec_ep;
#pragma unroll
  for (int tap = 0; tap < KS * KS; ++tap) {
    if (vec) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) E[(16 * i + 4 * lq + r) * EW + 16 * j + l16] = acc[tap][i][j][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int q = 0; q < 16 * MI / RPI; ++q) {
        const int row = RPI * q + rr;
        const int ci = ci0 + wci0 + row, n = co0 + wco0 + 4 * c4;
        const float4 v = *reinterpret_cast<const float4*>(&E[row * EW + 4 * c4]);
        if (ci < a.kc && n < a.N)
          *reinterpret_cast<float4*>(&S[((int64_t)tap * a.kc + ci) * a.slab_ld + n]) = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ci = ci0 + wci0 + 16 * i + 4 * lq + r;
            if (ci < a.kc && co[j] < a.N)
              S[((int64_t)tap * a.kc + ci) * a.slab_ld + co[j]] = acc[tap][i][j][r];
          }
    }
  }
}

template <int WAVES_CI, int WAVES_CO, int XH, int MI = 1>
__global__ __launch_bounds__(64 * WAVES_CI * WAVES_CO, 1) void conv_wgrad_tile_x3b(GemmArgs a) {
  wgrad_x3b_body<WAVES_CI, WAVES_CO, XH, MI, 3>(a);
}

// bf16 (configs 3-5) 3x3 stride-1 weight gradient on the 9-tap structure, one plane.
template <int WAVES_CI, int WAVES_CO, int XH>
__global__ __launch_bounds__(64 * WAVES_CI * WAVES_CO, 1) void conv_wgrad_tile_b16(GemmArgs a) {
  wgrad_x3b_body<WAVES_CI, WAVES_CO, XH, 1, 1>(a);
}

// ---- fp32 weight gradient on the split-bf16 MFMA: implicit GEMM (other shapes) ------------
// C[m = (tap, ci)][n = co] = sum over output pixels k of x(pix(k, tap))[ci] . dy(k)[co] for
// the stem, the stride-2 block convs and the projections: conv_wgrad_bf16's staging (slots of
// 4 channels x 8 pixels, coalesced across the channel quads of a pixel, written transposed as
// [channel row][pixel octet] images) with every value cut into the hi / mid / lo bf16 planes
// and six v_mfma_f32_16x16x32_bf16 per fragment pair.  LDS rows are four octets; octet o of
// row r sits in slot o ^ [0, 2, 3, 1][(r >> 2) & 3], which keeps the 16x16x32 fragment reads
// conflict-free and the staging stores (8 lanes = rows 4 apart) at 2-way.  Double-buffered,
// one barrier per 32-pixel chunk; split-K slabs + the bias column sums, as the other wgrads.
__device__ __forceinline__ int wx3_sw(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

// NP = 1: the bf16 weight gradient of the same shapes (one plane, one MFMA per fragment pair,
// operands rounded to bf16 as conv_wgrad_bf16 rounds them).
template <int BM, int BN, int WAVES_M, int WAVES_N, int NP = 3>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N, NP == 1 ? 2 : 1) void conv_wgrad_x3(GemmArgs a) {
  static_assert(NP == 3 || NP == 1, "three split planes (fp32) or one (bf16)");
  constexpr int NT = 64 * WAVES_M * WAVES_N, NW = NT / 64;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, SM = WM / 16, SN = WN / 16;
  static_assert(SM >= 1 && SN >= 1 && WM % 16 == 0 && WN % 16 == 0, "tile");
  constexpr int NSLOT = BM + BN, SPT = (NSLOT + NT - 1) / NT;
  constexpr int A_U4 = NP * BM * 4, B_U4 = NP * BN * 4;
  constexpr int OP_U4 = 2 * (A_U4 + B_U4), EP_U4 = NW * WM * WN * 4 / 16;
  static_assert(4 * BN * 4 <= OP_U4 * 16, "column-sum image fits LDS");
  __shared__ uint4 smem[OP_U4 > EP_U4 ? OP_U4 : EP_U4];   // operands, then epilogue images

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_n = tile % a.n_tiles;
  const int tile_m = tile / a.n_tiles;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int M = a.M;
  const int k_begin = split * a.k_per_split;
  const int k_end = min(a.K, k_begin + a.k_per_split);
  const int nchunks = k_end > k_begin ? (k_end - k_begin + BKH - 1) / BKH : 0;
  const rsrc_t rx = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rd = make_rsrc(a.B, a.b_bytes);
  const bool do_colsum = a.colsum && tile_m == 0;

  // ---- per-slot fixed state (slot = channel quad x pixel octet of the 32-pixel chunk)
  bool s_isa[SPT], s_ok[SPT];
  int s_row[SPT], s_oc[SPT], s_col[SPT], s_r[SPT], s_s[SPT];
  int s_b[SPT], s_oy[SPT], s_ox[SPT];
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int sl = tid + NT * j;
    const bool live = sl < NSLOT;
    const bool isa = sl < BM;
    const int q = isa ? sl : sl - BM;
    const int nq = isa ? BM / 4 : BN / 4;
    const int rq = q % nq, oc = q / nq;
    s_isa[j] = isa;
    s_row[j] = 4 * rq;
    s_oc[j] = live ? oc : -1;
    if (isa) {
      const int m = m0 + 4 * rq;
      s_ok[j] = live && m < M;
      const int mm = m < M ? m : 0;
      const int tap = mm / a.kc;
      s_col[j] = mm - tap * a.kc;
      s_r[j] = tap / a.kw;
      s_s[j] = tap - s_r[j] * a.kw;
    } else {
      const int n = n0 + 4 * rq;
      s_ok[j] = live && n < a.nb;
      s_col[j] = n;
      s_r[j] = s_s[j] = 0;
    }
    const int k = k_begin + 8 * oc;
    const int hw = a.ho * a.wo;
    const int kk = k < a.K ? k : 0;
    s_b[j] = kk / hw;
    const int rem = kk - s_b[j] * hw;
    s_oy[j] = rem / a.wo;
    s_ox[j] = rem - s_oy[j] * a.wo;
  }
  float4 stg[SPT][8];
  float4 colacc = make_float4(0.f, 0.f, 0.f, 0.f);
  int kc0 = k_begin;
  auto load = [&]() {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      int b = s_b[j], oy = s_oy[j], ox = s_ox[j];
      const int kbase = kc0 + 8 * s_oc[j];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool okk = s_ok[j] && s_oc[j] >= 0 && kbase + e < k_end;
        uint32_t off = kOOB;
        if (s_isa[j]) {
          const int sy = oy * a.stride - a.pt + s_r[j], sx = ox * a.stride - a.pl + s_s[j];
          if (okk && (unsigned)sy < (unsigned)a.h && (unsigned)sx < (unsigned)a.w)
            off = (uint32_t)((((b * a.h + sy) * a.w + sx) * a.lda + s_col[j]) * 4);
          stg[j][e] = bload4(rx, off);
        } else {
          if (okk) off = (uint32_t)(((kbase + e) * a.ldb + s_col[j]) * 4);
          stg[j][e] = bload4(rd, off);
        }
        if (++ox >= a.wo) {
          ox = 0;
          if (++oy >= a.ho) {
            oy = 0;
            ++b;
          }
        }
      }
    }
  };
  auto advance = [&]() {
    kc0 += BKH;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      s_ox[j] += BKH;
      while (s_ox[j] >= a.wo) {
        s_ox[j] -= a.wo;
        if (++s_oy[j] >= a.ho) {
          s_oy[j] = 0;
          ++s_b[j];
        }
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (s_oc[j] < 0) continue;
      const int rows = s_isa[j] ? BM : BN;
      uint4* img = smem + (s_isa[j] ? buf * A_U4 : 2 * A_U4 + buf * B_U4);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float v8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v8[e] = (&stg[j][e].x)[c];
        const int row = s_row[j] + c;
        const int idx = row * 4 + (s_oc[j] ^ wx3_sw(row));
        if (NP == 1) {
          img[idx] = pack_bf16x8(make_float4(v8[0], v8[1], v8[2], v8[3]),
                                 make_float4(v8[4], v8[5], v8[6], v8[7]));
        } else {
          bf16x8 h, m, l;
          split3x8(v8, h, m, l);
          img[idx] = __builtin_bit_cast(uint4, h);
          img[(NP / 2) * rows * 4 + idx] = __builtin_bit_cast(uint4, m);
          img[(NP - 1) * rows * 4 + idx] = __builtin_bit_cast(uint4, l);
        }
      }
      if (!s_isa[j] && do_colsum) {
#pragma unroll
        for (int e = 0; e < 8; ++e) add4(colacc, stg[j][e]);
      }
    }
  };

  f32x4 acc[SM][SN];
#pragma unroll
  for (int i = 0; i < SM; ++i)
#pragma unroll
    for (int j = 0; j < SN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
  const int wm0 = (wave / WAVES_N) * WM;
  const int wn0 = (wave % WAVES_N) * WN;
  const int l16 = lane & 15, lq = lane >> 4;
  const int frag = l16 * 4 + (lq ^ wx3_sw(l16));   // rows 16-aligned + l16

  if (nchunks > 0) {
    load();
    store(0);
  }
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) {
      advance();
      load();
    }
    const uint4* As = smem + buf * A_U4;
    const uint4* Bs = smem + 2 * A_U4 + buf * B_U4;
    bf16x8 av[NP][SM], bv[NP][SN];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
      for (int i = 0; i < SM; ++i)
        av[p][i] = __builtin_bit_cast(bf16x8, As[p * BM * 4 + (wm0 + 16 * i) * 4 + frag]);
#pragma unroll
      for (int j = 0; j < SN; ++j)
        bv[p][j] = __builtin_bit_cast(bf16x8, Bs[p * BN * 4 + (wn0 + 16 * j) * 4 + frag]);
    }
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j) {
        f32x4 x = acc[i][j];
        if (NP == 3) {
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP - 1][i], bv[0][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[NP - 1][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP / 2][i], bv[NP / 2][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[NP / 2][i], bv[0][j], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[NP / 2][j], x, 0, 0, 0);
        }
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], x, 0, 0, 0);
      }
    if (more) store(buf ^ 1);
    __syncthreads();
  }

  // ---- raw partial sums into this K slice's slab (+ bias column sums in row M)
  float* S = a.slab + (int64_t)split * a.split_stride;
  if (do_colsum) {
    // B-slot threads hold 4 columns x their pixel octet: 4 octets per column quad, summed in a
    // fixed order (the loop's last barrier freed the images)
    float* csum = reinterpret_cast<float*>(smem);      // [4 octets][BN]
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (!s_isa[j] && s_oc[j] >= 0) {
        const int cq = s_row[j];
        csum[s_oc[j] * BN + cq] = colacc.x;
        csum[s_oc[j] * BN + cq + 1] = colacc.y;
        csum[s_oc[j] * BN + cq + 2] = colacc.z;
        csum[s_oc[j] * BN + cq + 3] = colacc.w;
      }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.N)
      S[(int64_t)M * a.slab_ld + n0 + tid] =
          csum[tid] + csum[BN + tid] + csum[2 * BN + tid] + csum[3 * BN + tid];
    __syncthreads();
  }
  if (a.vec_ep) {
    float* E = reinterpret_cast<float*>(smem) + wave * WM * WN;
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) E[(16 * i + 4 * lq + r) * WN + 16 * j + l16] = acc[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr int LPR = WN / 4, RPI = 64 / LPR;
    const int c4 = lane % LPR, rr = lane / LPR;
    const int n = n0 + wn0 + 4 * c4;
#pragma unroll
    for (int q = 0; q < WM / RPI; ++q) {
      const int ml = q * RPI + rr, m = m0 + wm0 + ml;
      const float4 v = *reinterpret_cast<const float4*>(&E[ml * WN + 4 * c4]);
      if (m < M && n < a.N) *reinterpret_cast<float4*>(&S[(int64_t)m * a.slab_ld + n]) = v;
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < SN; ++j) {
    const int n = n0 + wn0 + 16 * j + l16;
    if (n >= a.N) continue;
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm0 + 16 * i + 4 * lq + r;
        if (m < M) S[(int64_t)m * a.slab_ld + n] = acc[i][j][r];
      }
  }
}

// ---- fp32 weight gradient, 3x3 stride 1: all 9 taps from one staged halo ----------------
// dW[r][s][ci][co] = sum_p x(p + (r, s) - pad)[ci] . dy(p)[co] on v_mfma_f32_32x32x2_f32, the
// fp32 counterpart of conv_wgrad_tile_bf16: a workgroup owns CIB x COB channels for all 9
// taps (wave = 32 ci x 32 co x 9 accumulators) and walks 8 x 16 output-pixel tiles; per tile
// it stages the x halo (10 x 18 px x CIB, pixel-major as in HBM) and dy (128 px x COB) once,
// and every tap reads its A fragments from the halo at a shifted pixel.  fp32 fragments are
// single dwords, so a shift needs no aligned copies: lanes 0-31 read 32 consecutive channels
// of one pixel, lanes 32-63 of the next (conflict-free ds_read_b32).  One LDS image, register
// prefetch of the next tile during the MFMAs.  Output: the split-K slabs of the GEMM path.
template <int WAVES_CI, int WAVES_CO>
__global__ __launch_bounds__(256, 1) void conv_wgrad_tile_f32(GemmArgs a) {
  constexpr int CIB = 32 * WAVES_CI, COB = 32 * WAVES_CO, KS = 3;
  constexpr int HH = TT_H + KS - 1, HW = TT_W + KS - 1, HP = HH * HW;
  static_assert(WAVES_CI * WAVES_CO == 4 && COB >= 64, "4 waves, COB >= 64");
  constexpr int XQ = HP * (CIB / 4), XS = (XQ + 255) / 256;      // (halo px, ci quad)
  constexpr int DQ = TT_H * TT_W * (COB / 4), DS = DQ / 256;     // (px, co quad)
  static_assert(DQ % 256 == 0, "dy items");
  constexpr int NG = 256 / (COB / 4);
  __shared__ float4 Xs4[HP * CIB / 4];
  __shared__ float4 Ds4[TT_H * TT_W * COB / 4];
  __shared__ float csum[NG][COB];
  const float* Xs = reinterpret_cast<const float*>(Xs4);
  const float* Dsf = reinterpret_cast<const float*>(Ds4);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_co = tile % a.n_tiles;
  const int tile_ci = tile / a.n_tiles;
  const int ci0 = tile_ci * CIB, co0 = tile_co * COB;
  const int t_begin = split * a.k_per_split;
  const int t_end = min(a.K, t_begin + a.k_per_split);
  const int steps = max(0, t_end - t_begin);
  const int tiles_x = (a.wo + TT_W - 1) / TT_W, tiles_y = (a.ho + TT_H - 1) / TT_H;
  const rsrc_t rx = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rd = make_rsrc(a.B, a.b_bytes);
  const bool do_colsum = a.colsum && tile_ci == 0;
  const int xcq = tid % (CIB / 4);
  const bool xc_ok = ci0 + 4 * xcq < a.kc;
  const int dcq = tid % (COB / 4);
  const bool dc_ok = co0 + 4 * dcq < a.nb;

  float4 xv[XS], dv[DS];
  float4 colacc = make_float4(0.f, 0.f, 0.f, 0.f);
  auto load = [&](int t) {
    const int b = t / (tiles_x * tiles_y);
    const int trem = t - b * tiles_x * tiles_y;
    const int oy0 = (trem / tiles_x) * TT_H, ox0 = (trem % tiles_x) * TT_W;
#pragma unroll
    for (int j = 0; j < XS; ++j) {
      const int q = tid + 256 * j;
      const int hp = q / (CIB / 4);
      const int iy = oy0 - a.pt + hp / HW, ix = ox0 - a.pl + hp % HW;
      const bool ok = q < XQ && xc_ok && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
      xv[j] = bload4(rx, ok ? (uint32_t)((((b * a.h + iy) * a.w + ix) * a.lda + ci0 + 4 * xcq) * 4)
                            : kOOB);
    }
#pragma unroll
    for (int j = 0; j < DS; ++j) {
      const int px = (tid + 256 * j) / (COB / 4);
      const int oy = oy0 + px / TT_W, ox = ox0 + px % TT_W;
      const bool ok = dc_ok && oy < a.ho && ox < a.wo;
      dv[j] = bload4(rd, ok ? (uint32_t)((((b * a.ho + oy) * a.wo + ox) * a.ldb + co0 + 4 * dcq) * 4)
                            : kOOB);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < XS; ++j) {
      const int q = tid + 256 * j;
      if (q < XQ) Xs4[q] = xv[j];          // [halo px][CIB] with quads contiguous
    }
#pragma unroll
    for (int j = 0; j < DS; ++j) {
      Ds4[tid + 256 * j] = dv[j];           // [px][COB]
      if (do_colsum) add4(colacc, dv[j]);
    }
  };

  f32x16 acc[KS * KS];
#pragma unroll
  for (int t = 0; t < KS * KS; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const int wci0 = (wave / WAVES_CO) * 32;
  const int wco0 = (wave % WAVES_CO) * 32;
  const int lrow = lane & 31, lk = lane >> 5;

  if (steps > 0) {
    load(t_begin);
    store();
  }
  __syncthreads();
  for (int i = 0; i < steps; ++i) {
    const bool more = i + 1 < steps;
    if (more) load(t_begin + i + 1);
#pragma unroll 2
    for (int k2 = 0; k2 < TT_H * TT_W / 2; ++k2) {
      const int p = 2 * k2 + lk;                        // this lane's pixel of the pair
      const float bv = Dsf[p * COB + wco0 + lrow];
      const float* xa = Xs + ((p / TT_W) * HW + p % TT_W) * CIB + wci0 + lrow;
#pragma unroll
      for (int r = 0; r < KS; ++r)
#pragma unroll
        for (int s = 0; s < KS; ++s)
          acc[r * KS + s] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[(r * HW + s) * CIB], bv,
                                                                 acc[r * KS + s], 0, 0, 0);
    }
    if (more) {
      __syncthreads();
      store();
    }
    __syncthreads();
  }

  float* S = a.slab + (int64_t)split * a.split_stride;
  if (do_colsum) {
    const int g = tid / (COB / 4);
    csum[g][4 * dcq] = colacc.x;
    csum[g][4 * dcq + 1] = colacc.y;
    csum[g][4 * dcq + 2] = colacc.z;
    csum[g][4 * dcq + 3] = colacc.w;
    __syncthreads();
    if (tid < COB && co0 + tid < a.N) {
      float v = 0.f;
#pragma unroll
      for (int g2 = 0; g2 < NG; ++g2) v += csum[g2][tid];
      S[(int64_t)a.M * a.slab_ld + co0 + tid] = v;
    }
  }
  const int n = co0 + wco0 + lrow;
  if (n < a.N) {
#pragma unroll
    for (int t = 0; t < KS * KS; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = ci0 + wci0 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (ci < a.kc) S[((int64_t)t * a.kc + ci) * a.slab_ld + n] = acc[t][r];
      }
  }
}

// Split-K epilogue for fwd/dgrad: sum the K slices' slabs, then the fused epilogue.
// Workgroup = 32 items x 8 split lanes; item = (slab row, 4 columns); the 8 lanes each sum
// every 8th slice (many independent loads in flight), then a fixed-order LDS reduction.
constexpr int EP_ITEMS = 32, EP_LANES = 8;
// sum over z = z0, z0 + EP_LANES, ... < zend of src[z * stride .. + 3], in that order, with
// four loads in flight (the split-K reductions are latency-bound at one load per step)
__device__ __forceinline__ float4 strided_sum4(const float* src, int z0, int zend, int64_t stride) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int z = z0;
  for (; z + 3 * EP_LANES < zend; z += 4 * EP_LANES) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      v[u] = *reinterpret_cast<const float4*>(src + (int64_t)(z + u * EP_LANES) * stride);
#pragma unroll
    for (int u = 0; u < 4; ++u) add4(acc, v[u]);
  }
  for (; z < zend; z += EP_LANES) add4(acc, *reinterpret_cast<const float4*>(src + (int64_t)z * stride));
  return acc;
}

template <int MODE>
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(GemmArgs a) {
  __shared__ float4 red[EP_LANES][EP_ITEMS];
  const int it = threadIdx.x % EP_ITEMS, sl = threadIdx.x / EP_ITEMS;
  const int nq = (a.N + 3) / 4;
  const int64_t rows = (int64_t)(a.tiles_total / a.n_tiles) * a.bm;
  const int64_t item = (int64_t)blockIdx.x * EP_ITEMS + it;
  const bool live = item < rows * nq;
  const int q = live ? (int)(item % nq) : 0;
  const int64_t srow = live ? item / nq : 0;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    acc = strided_sum4(a.slab + srow * a.slab_ld + 4 * q, sl, a.splits, a.split_stride);
  }
  red[sl][it] = acc;
  __syncthreads();
  if (sl != 0 || !live) return;
  for (int k = 1; k < EP_LANES; ++k) add4(acc, red[k][it]);
  const int tm = (int)(srow / a.bm);
  int gi = 0;
  for (int g = 1; g < a.ngroups; ++g)
    if (tm >= a.grp[g].tiles_begin) gi = g;
  const Group& G = a.grp[gi];
  const int m = (int)(srow - (int64_t)G.tiles_begin * a.bm);
  if (m >= G.M) return;
  const int64_t row = out_row(a, G, m);
  const float v[4] = {acc.x, acc.y, acc.z, acc.w};
  EpAux aux[4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
    aux[e] = 4 * q + e < a.N ? epilogue_aux<MODE>(a, row, 4 * q + e) : EpAux{0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int n = 4 * q + e;
    if (n >= a.N) break;
    float bias, scale, shift;
    column_params<MODE>(a, n, bias, scale, shift);
    epilogue_store<MODE>(a, row, n, v[e], bias, scale, shift, aux[e]);
  }
}

// Split-K epilogue for a few slices over many rows (the common case: 2-6 slices of a layer
// whose tile grid half-fills the chip).  One (slab row, 4 columns) item per thread in a
// grid-stride loop; the slices are summed in order with four loads in flight, then the fused
// epilogue runs on all four columns.  VEC: every row-major operand takes 16-byte accesses
// (host-checked alignment and leading dimensions).  The 8-lane kernel above is kept for many
// slices over few rows, where one thread per item would serialise the slice loads.
__device__ __forceinline__ float4 ld4(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}

template <int MODE, bool VEC>
__global__ __launch_bounds__(256) void splitk_epilogue_flat(GemmArgs a) {
  const int nq = (a.N + 3) / 4;
  const int64_t items = (int64_t)(a.tiles_total / a.n_tiles) * a.bm * nq;
  const int64_t ss = a.split_stride;
  for (int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; item < items;
       item += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(item % nq);
    const int64_t srow = item / nq;
    const int tm = (int)(srow / a.bm);
    int gi = 0;
    for (int g = 1; g < a.ngroups; ++g)
      if (tm >= a.grp[g].tiles_begin) gi = g;
    const Group& G = a.grp[gi];
    const int m = (int)(srow - (int64_t)G.tiles_begin * a.bm);
    if (m >= G.M) continue;
    const float* src = a.slab + srow * a.slab_ld + 4 * q;
    float4 acc = ld4(src);
    int z = 1;
    for (; z + 4 <= a.splits; z += 4) {
      const float4 p0 = ld4(src + z * ss), p1 = ld4(src + (z + 1) * ss);
      const float4 p2 = ld4(src + (z + 2) * ss), p3 = ld4(src + (z + 3) * ss);
      add4(acc, p0);
      add4(acc, p1);
      add4(acc, p2);
      add4(acc, p3);
    }
    for (; z < a.splits; ++z) add4(acc, ld4(src + z * ss));
    const int64_t row = out_row(a, G, m);
    float v[4] = {acc.x, acc.y, acc.z, acc.w};
    const int n0 = 4 * q;
    if (VEC) {
      float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f), r4 = s4;
      if (MODE == MODE_FWD && a.res) s4 = ld4(a.res + row * a.ldr + n0);
      if (MODE == MODE_DGRAD) {
        s4 = a.act_src ? ld4(a.act_src + row * a.ld_act + n0) : make_float4(1.f, 1.f, 1.f, 1.f);
        if (a.res) r4 = ld4(a.res + row * a.ldr + n0);
      }
      const float s[4] = {s4.x, s4.y, s4.z, s4.w}, r[4] = {r4.x, r4.y, r4.z, r4.w};
      float zv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float bias, scale, shift;
        column_params<MODE>(a, n0 + e, bias, scale, shift);
        if (MODE == MODE_FWD) {
          v[e] += bias;
          zv[e] = v[e];
          if (a.bn_g) v[e] = v[e] * scale + shift;
          v[e] = act_fwd(v[e] + s[e], a.act, a.alpha);
        } else {
          v[e] = dgrad_ep(a, v[e], s[e], r[e]);
        }
      }
      if (MODE == MODE_FWD && a.z)
        *reinterpret_cast<float4*>(a.z + row * a.ldz + n0) = make_float4(zv[0], zv[1], zv[2], zv[3]);
      *reinterpret_cast<float4*>(a.C + row * a.ldc + n0) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      EpAux aux[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        aux[e] = n0 + e < a.N ? epilogue_aux<MODE>(a, row, n0 + e) : EpAux{0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + e;
        if (n >= a.N) break;
        float bias, scale, shift;
        column_params<MODE>(a, n, bias, scale, shift);
        epilogue_store<MODE>(a, row, n, v[e], bias, scale, shift, aux[e]);
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

// Input-gradient weights: rows (group tap t, co) group after group, each group's block
// padded to BK rows; columns ci.  Wd[row][ci] = W[r][s][ci][co].
struct PackGroups {
  int ngroups;
  int dt;
  int r0[MAX_GROUPS], s0[MAX_GROUPS], ns[MAX_GROUPS], ntaps[MAX_GROUPS];
  int64_t row_begin[MAX_GROUPS + 1];     // f32 packing: group row blocks padded to BK
  int64_t row_begin16[MAX_GROUPS + 1];   // bf16 packing: group k blocks padded to BKH
};

__global__ void pack_bwd_kernel(const float* __restrict__ w, PackGroups pg, int kw, int cin,
                                int cout, int cout_p, int nd, float* __restrict__ out) {
  const int64_t total = pg.row_begin[pg.ngroups] * nd;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = idx / nd;
    const int n = (int)(idx - row * nd);
    int g = 0;
    for (int q = 1; q < pg.ngroups; ++q)
      if (row >= pg.row_begin[q]) g = q;
    const int k = (int)(row - pg.row_begin[g]);
    const int t = k / cout_p, co = k - t * cout_p;
    float v = 0.f;
    if (t < pg.ntaps[g] && co < cout && n < cin) {
      const int r = pg.r0[g] + pg.dt * (t / pg.ns[g]);
      const int s = pg.s0[g] + pg.dt * (t % pg.ns[g]);
      v = w[((int64_t)(r * kw + s) * cin + n) * cout + co];
    }
    out[idx] = v;
  }
}

// All convs of a model packed in one launch from a device-resident table.
struct PackEntry {
  const float* w;
  float* wf;               // f32 packing; bf16 packing: __bf16 buffers
  float* wd;
  int taps, kw, cin, cout, cin_p, cout_p, kf, nf, nd;
  int bf16;                // 1: transposed bf16 images [n][k] (conv_gemm_bf16); 2: the
                           // three split planes of those images (conv_tile_x3)
  int kf16;
  int64_t kd16;
  int64_t work_begin;      // cumulative elements (fwd then bwd; bf16: bwd only) before this entry
  int tile_begin;          // bf16: cumulative forward-image tiles (pack_fwd16_tile) before it
  const float* bn_g;       // non-NULL: the input-gradient image is scaled per output channel
  const float* bn_v;       // by gamma / sqrt(var + eps) (inference BN folded into the dgrad)
  float bn_eps;
  PackGroups pg;
};

__device__ __forceinline__ float bn_fold(const PackEntry& E, int co) {
  return E.bn_g ? E.bn_g[co] * rsqrtf(E.bn_v[co] + E.bn_eps) : 1.f;
}

struct PackTableHeader {
  int nconv;
  int ntiles16;            // forward-image tiles of the bf16 entries (pack_fwd16_tile)
  int64_t total;           // elements of pack_elem's part
};

// bf16 image element k (mode 1: RNE), or its three split terms in planes `plane` apart (mode 2,
// conv_tile_x3).
__device__ __forceinline__ void put16(int mode, float* base, int64_t k, int64_t plane, float v) {
  __bf16* o = reinterpret_cast<__bf16*>(base);
  if (mode == 1) {
    o[k] = (__bf16)v;
    return;
  }
  const uint32_t hb = __float_as_uint(v) & 0xffff0000u;
  const float r = v - __uint_as_float(hb);
  const uint32_t mb = __float_as_uint(r) & 0xffff0000u;
  const uint32_t lb = __float_as_uint(r - __uint_as_float(mb));
  o[k] = __builtin_bit_cast(__bf16, (uint16_t)(hb >> 16));
  o[k + plane] = __builtin_bit_cast(__bf16, (uint16_t)(mb >> 16));
  o[k + 2 * plane] = __builtin_bit_cast(__bf16, (uint16_t)(lb >> 16));
}

// One packed element of entry E (f32: fwd rows [k][n] then bwd rows; bf16: transposed).
// k < 2^31 (entry-local; the host checks): 32-bit index arithmetic.
__device__ void pack_elem(const PackEntry& E, int k) {
  if (E.bf16) {
    const int nfwd16 = E.cout_p * E.kf16;
    if (k < nfwd16) {                       // W16_f[n][tap*cin_p + ci]
      const int n = k / E.kf16, kk = k - n * E.kf16;
      const int tap = kk / E.cin_p, ci = kk - tap * E.cin_p;
      float v = 0.f;
      if (tap < E.taps && ci < E.cin && n < E.cout)
        v = E.w[(tap * E.cin + ci) * E.cout + n];
      put16(E.bf16, E.wf, k, nfwd16, v);
    } else {                                // W16_d[ci][group k block: t*cout_p + co]
      k -= nfwd16;
      const int kd16 = (int)E.kd16;
      const int ci = k / kd16;
      const int kc = k - ci * kd16;
      const PackGroups& pg = E.pg;
      int g = 0;
      for (int q = 1; q < pg.ngroups; ++q)
        if (kc >= pg.row_begin16[q]) g = q;
      const int kk = kc - (int)pg.row_begin16[g];
      const int t = kk / E.cout_p, co = kk - t * E.cout_p;
      float v = 0.f;
      if (t < pg.ntaps[g] && co < E.cout && ci < E.cin) {
        const int r = pg.r0[g] + pg.dt * (t / pg.ns[g]);
        const int ss = pg.s0[g] + pg.dt * (t % pg.ns[g]);
        v = E.w[((r * E.kw + ss) * E.cin + ci) * E.cout + co] * bn_fold(E, co);
      }
      put16(E.bf16, E.wd, k, E.kd16 * E.nd, v);
    }
    return;
  }
  const int nfwd = E.kf * E.nf;
  if (k < nfwd) {
    const int kk = k / E.nf, nn = k - kk * E.nf;
    const int tap = kk / E.cin_p, ci = kk - tap * E.cin_p;
    float v = 0.f;
    if (tap < E.taps && ci < E.cin && nn < E.cout)
      v = E.w[(tap * E.cin + ci) * E.cout + nn];
    E.wf[k] = v;
  } else {
    k -= nfwd;
    const int row = k / E.nd;
    const int nn = k - row * E.nd;
    const PackGroups& pg = E.pg;
    int g = 0;
    for (int q = 1; q < pg.ngroups; ++q)
      if (row >= pg.row_begin[q]) g = q;
    const int kk = row - (int)pg.row_begin[g];
    const int t = kk / E.cout_p, co = kk - t * E.cout_p;
    float v = 0.f;
    if (t < pg.ntaps[g] && co < E.cout && nn < E.cin) {
      const int r = pg.r0[g] + pg.dt * (t / pg.ns[g]);
      const int ss = pg.s0[g] + pg.dt * (t % pg.ns[g]);
      v = E.w[((r * E.kw + ss) * E.cin + nn) * E.cout + co] * bn_fold(E, co);
    }
    E.wd[k] = v;
  }
}

// The bf16 / split forward images W16_f[n][tap * cin_p + ci] of the table's bf16 entries, by
// 32 (n) x 64 (K) tiles through LDS: the HWIO source is read along n (its contiguous axis) and
// the image written along K.  (Element by element in image order, every lane of a wave read a
// different source line: consecutive K are cout floats apart.)
constexpr int PK_TN = 32, PK_TK = 64;
__device__ void pack_fwd16_tile(const PackEntry& E, int t, float (*tile)[PK_TN + 1]) {
  const int ntk = (E.kf16 + PK_TK - 1) / PK_TK;
  const int tn = t / ntk, tk = t - tn * ntk;
  const int n0 = tn * PK_TN, k0 = tk * PK_TK;
  const int ln = threadIdx.x & (PK_TN - 1), lk = threadIdx.x / PK_TN;    // 8 K rows a pass
#pragma unroll
  for (int p = 0; p < PK_TK / 8; ++p) {
    const int kk = k0 + 8 * p + lk, n = n0 + ln;
    const int tap = kk / E.cin_p, ci = kk - tap * E.cin_p;
    float v = 0.f;
    if (tap < E.taps && ci < E.cin && n < E.cout) v = E.w[(tap * E.cin + ci) * E.cout + n];
    tile[8 * p + lk][ln] = v;
  }
  __syncthreads();
  const int wk = threadIdx.x & (PK_TK - 1), wn = threadIdx.x / PK_TK;   // 4 n rows a pass
  const int64_t plane = (int64_t)E.cout_p * E.kf16;
#pragma unroll
  for (int p = 0; p < PK_TN / 4; ++p) {
    const int n = n0 + 4 * p + wn, kk = k0 + wk;
    if (n < E.cout_p && kk < E.kf16)
      put16(E.bf16, E.wf, (int64_t)n * E.kf16 + kk, plane, tile[wk][4 * p + wn]);
  }
  __syncthreads();                          // the tile is rewritten by the next iteration
}

// Workgroups [0, b1): PACK_PT x 256 consecutive elements each (lane-strided: coalesced
// stores); the entry of its first element is found once and advanced at entry boundaries (no
// per-element search of the table).  The entry is read in place: a register copy of PackEntry
// (dynamically indexed group arrays) lands in scratch.  bf16 entries' element range is their
// input-gradient image only; workgroups [b1, grid) walk the forward-image tiles
// (pack_fwd16_tile), grid-stride.
constexpr int PACK_PT = 8;
__global__ __launch_bounds__(256) void pack_many_kernel(const char* __restrict__ table, int b1) {
  const PackTableHeader* h = reinterpret_cast<const PackTableHeader*>(table);
  const PackEntry* e = reinterpret_cast<const PackEntry*>(table + sizeof(PackTableHeader));
  const int n = h->nconv;
  if ((int)blockIdx.x >= b1) {
    __shared__ float tile[PK_TK][PK_TN + 1];
    const int nt = h->ntiles16;
    for (int t = (int)blockIdx.x - b1; t < nt; t += (int)gridDim.x - b1) {
      int lo = 0, hi = n - 1;                 // the last entry with tile_begin <= t (entries
      while (lo < hi) {                       // without tiles share the next one's begin)
        const int mid = (lo + hi + 1) >> 1;
        if (e[mid].tile_begin <= t) lo = mid; else hi = mid - 1;
      }
      pack_fwd16_tile(e[lo], t - e[lo].tile_begin, tile);
    }
    return;
  }
  const int64_t total = h->total;
  const int64_t base = (int64_t)blockIdx.x * 256 * PACK_PT;
  if (base >= total) return;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (e[mid].work_begin <= base) lo = mid; else hi = mid - 1;
  }
  int cur = lo;
  int64_t next = cur + 1 < n ? e[cur + 1].work_begin : total;
  for (int u = 0; u < PACK_PT; ++u) {
    const int64_t idx = base + u * 256 + threadIdx.x;
    if (idx >= total) break;
    while (idx >= next) {
      ++cur;
      next = cur + 1 < n ? e[cur + 1].work_begin : total;
    }
    const PackEntry& E = e[cur];                        // entry fields: cached global loads
    pack_elem(E, (int)(idx - E.work_begin) + (E.bf16 ? E.cout_p * E.kf16 : 0));
  }
}

__global__ void pack_one_kernel(PackEntry E, int64_t total) {
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x)
    pack_elem(E, (int)idx);
}

// dw[tap][ci][co] (HWIO) = sum_z slab[z][tap*kc + ci][co]; optional db[co] = sum_z slab[z][M][co].
// Workgroup = 256 / LANES items x LANES split lanes, item = (output row, 4 columns); each lane
// sums every LANES-th slab with eight loads in flight, then a fixed-order LDS reduction over
// the lanes.  LANES = 32 for many slabs (the 9-tap weight gradients write one slab per
// workgroup: 256 of them for the encoder's 64-channel layers): more workgroups and fewer
// serial loads per lane, so the pass keeps its bandwidth when it shares the chip.
template <int LANES>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws,
                                                           int splits, int64_t split_stride,
                                                           int taps, int kc, int cin, int cout,
                                                           int ldc, float* __restrict__ dw,
                                                           float* __restrict__ db, int accum,
                                                           const float* __restrict__ bn_g,
                                                           const float* __restrict__ bn_v,
                                                           float bn_eps) {
  constexpr int ITEMS = 256 / LANES;
  __shared__ float4 red[LANES][ITEMS];
  const int it = threadIdx.x % ITEMS, sl = threadIdx.x / ITEMS;
  const int cq = (cout + 3) / 4;
  const int rows = taps * cin + (db ? 1 : 0);
  const int64_t item = (int64_t)blockIdx.x * ITEMS + it;
  const bool live = item < (int64_t)rows * cq;
  const int q = live ? (int)(item % cq) : 0;
  const int row = live ? (int)(item / cq) : 0;
  const bool is_bias = row == taps * cin;
  int64_t m;
  if (is_bias) {
    m = (int64_t)taps * kc;
  } else {
    const int tap = row / cin, ci = row - tap * cin;
    m = (int64_t)tap * kc + ci;
  }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    const float* src = ws + m * ldc + 4 * q;
    int z = sl;
    for (; z + 7 * LANES < splits; z += 8 * LANES) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = *reinterpret_cast<const float4*>(src + (int64_t)(z + u * LANES) * split_stride);
#pragma unroll
      for (int u = 0; u < 8; ++u) add4(acc, v[u]);
    }
    for (; z < splits; z += LANES)
      add4(acc, *reinterpret_cast<const float4*>(src + (int64_t)z * split_stride));
  }
  red[sl][it] = acc;
  __syncthreads();
  if (sl != 0 || !live) return;
  for (int k = 1; k < LANES; ++k) add4(acc, red[k][it]);
  float v[4] = {acc.x, acc.y, acc.z, acc.w};
  float* dst = is_bias ? db + 4 * q : dw + (int64_t)row * cout + 4 * q;
  const int nv = min(4, cout - 4 * q);
  if (bn_g)                       // dL/dz = t * gamma / sqrt(var + eps), folded per column
    for (int e = 0; e < nv; ++e) v[e] *= bn_g[4 * q + e] * rsqrtf(bn_v[4 * q + e] + bn_eps);
  for (int e = 0; e < nv; ++e) dst[e] = accum ? dst[e] + v[e] : v[e];
}

// launch with the lane count by the number of slabs
#ifndef WGR_ABL
#define WGR_ABL 0      // 1: skip the reduce (timing ablation, WRONG results; tools/ab_build.sh)
#endif
static int g_wgr_lanes = 0;   // of_set_tuning key 29: wgrad_reduce lanes (launch_wgrad_reduce)
void launch_wgrad_reduce(hipStream_t s, const float* ws, int splits, int64_t split_stride,
                         int taps, int kc, int cin, int cout, int ldc, float* dw, float* db,
                         int accum, const float* bn_g, const float* bn_v, float bn_eps) {
  if (WGR_ABL) return;
  const int64_t items = ((int64_t)taps * cin + (db ? 1 : 0)) * cdiv(cout, 4);
  // lanes: about 8 slab loads in flight per lane (key 29 = 1: the round-4 rule, 32 lanes from
  // 64 slabs up -- two loads a lane at 64 slabs)
  // (key 29 = 2: about 32 loads a lane, 3: about 64, 4: about 8)
  const int per = g_wgr_lanes == 2 ? 32 : g_wgr_lanes == 3 ? 64 : g_wgr_lanes == 4 ? 8 : 16;
  int lanes = 1;
  while (lanes < 32 && lanes * per < splits) lanes *= 2;
  if (g_wgr_lanes == 1) lanes = splits >= 64 ? 32 : 8;
  if (lanes == 32)
    hipLaunchKernelGGL(wgrad_reduce_kernel<32>, dim3(cdiv(items, 8)), dim3(256), 0, s, ws, splits,
                       split_stride, taps, kc, cin, cout, ldc, dw, db, accum, bn_g, bn_v, bn_eps);
  else if (lanes == 16)
    hipLaunchKernelGGL(wgrad_reduce_kernel<16>, dim3(cdiv(items, 16)), dim3(256), 0, s, ws, splits,
                       split_stride, taps, kc, cin, cout, ldc, dw, db, accum, bn_g, bn_v, bn_eps);
  else if (lanes == 8)
    hipLaunchKernelGGL(wgrad_reduce_kernel<8>, dim3(cdiv(items, 32)), dim3(256), 0, s, ws, splits,
                       split_stride, taps, kc, cin, cout, ldc, dw, db, accum, bn_g, bn_v, bn_eps);
  else if (lanes == 4)
    hipLaunchKernelGGL(wgrad_reduce_kernel<4>, dim3(cdiv(items, 64)), dim3(256), 0, s, ws, splits,
                       split_stride, taps, kc, cin, cout, ldc, dw, db, accum, bn_g, bn_v, bn_eps);
  else if (lanes == 2)
    hipLaunchKernelGGL(wgrad_reduce_kernel<2>, dim3(cdiv(items, 128)), dim3(256), 0, s, ws, splits,
                       split_stride, taps, kc, cin, cout, ldc, dw, db, accum, bn_g, bn_v, bn_eps);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<1>, dim3(cdiv(items, 256)), dim3(256), 0, s, ws, splits,
                       split_stride, taps, kc, cin, cout, ldc, dw, db, accum, bn_g, bn_v, bn_eps);
}

// ------------------------------------------------------------------------------ dispatch --
namespace {

struct Geo {
  int taps, cin_p, cout_p, kf, nf, nd;
  bool phase;            // dgrad as stride-2 phase groups
  PackGroups pg;
  int64_t kd;            // packed bwd rows
  int kf16;              // bf16: fwd K (padded to BKH) = row length of W16_f [cout_p][kf16]
  int64_t kd16;          // bf16: dgrad K over all groups = row length of W16_d [cin_p][kd16]
};

Geo geo(const of_conv_desc* d) {
  Geo g{};
  g.taps = d->kh * d->kw;
  g.cin_p = d->cin_p;
  g.cout_p = (int)round_up(d->cout, 4);
  g.kf = (int)round_up((int64_t)g.taps * g.cin_p, BK);
  g.nf = g.cout_p;
  g.nd = g.cin_p;
  g.phase = d->stride == 2;
  PackGroups& pg = g.pg;
  pg.row_begin[0] = 0;
  pg.row_begin16[0] = 0;
  if (g.phase) {
    pg.ngroups = 4;
    pg.dt = 2;
    for (int c = 0; c < 4; ++c) {
      const int qy = c >> 1, qx = c & 1;
      const int nr = std::max(0, (d->kh - qy + 1) / 2), ns = std::max(0, (d->kw - qx + 1) / 2);
      pg.r0[c] = qy;
      pg.s0[c] = qx;
      pg.ns[c] = std::max(ns, 1);
      pg.ntaps[c] = nr * ns;
      pg.row_begin[c + 1] = pg.row_begin[c] + round_up((int64_t)pg.ntaps[c] * g.cout_p, BK);
      pg.row_begin16[c + 1] =
          pg.row_begin16[c] + round_up((int64_t)pg.ntaps[c] * g.cout_p, BKH);
    }
  } else {
    pg.ngroups = 1;
    pg.dt = 1;
    pg.r0[0] = pg.s0[0] = 0;
    pg.ns[0] = d->kw;
    pg.ntaps[0] = g.taps;
    pg.row_begin[1] = round_up((int64_t)g.taps * g.cout_p, BK);
    pg.row_begin16[1] = round_up((int64_t)g.taps * g.cout_p, BKH);
  }
  g.kd = pg.row_begin[pg.ngroups];
  g.kf16 = (int)round_up((int64_t)g.taps * g.cin_p, BKH);
  g.kd16 = pg.row_begin16[pg.ngroups];
  return g;
}

int validate(const of_conv_desc* d) {
  OF_CHECK_ARG(d != nullptr, "conv desc is NULL");
  OF_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->cin > 0 && d->cout > 0, "conv dims");
  OF_CHECK_ARG(d->cin_p >= d->cin && d->cin_p % 4 == 0, "cin_p must be >= cin, multiple of 4");
  OF_CHECK_ARG(d->kh > 0 && d->kw > 0 && d->stride > 0, "conv kernel/stride");
  OF_CHECK_ARG(d->ho > 0 && d->wo > 0, "conv output dims");
  OF_CHECK_ARG(d->kh * d->kw <= 64, "conv: at most 64 taps (tap bitmasks)");
  return OF_OK;
}

// Tile configuration by GEMM N: (BM, BN).  Narrow N gets taller M tiles so every wave still
// owns >= 2 MFMA accumulators and the per-chunk staging cost is amortised.
// (A 256x128 tile -- 4x2 MFMA tiles per wave, 2 waves/SIMD -- measured 5-10 % slower on
// dgrad/wgrad and spills on fwd; 128x128 with 4 waves/SIMD is kept.)
int pick_bn(int N) { return N > 96 ? 128 : N > 64 ? 96 : N > 32 ? 64 : 32; }
int pick_bm(int N) { return N > 64 ? 128 : 256; }

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
  a.dt = 1;
  a.splits = 1;
  return a;
}

void single_group(GemmArgs& a, const of_conv_desc* d, int M, int K) {
  a.ngroups = 1;
  a.bm = pick_bm(a.N);
  Group& g = a.grp[0];
  g = Group{};
  g.m_tiles = (int)cdiv(M, a.bm);
  g.M = M;
  g.ns = d->kw;
  g.ntaps = d->kh * d->kw;
  g.K = K;
  a.n_tiles = (int)cdiv(a.N, pick_bn(a.N));
  a.tiles_total = g.m_tiles * a.n_tiles;
}

// fwd/dgrad split-K: split when the tile grid cannot fill the chip.  Target: g_split_wgs
// workgroups per CU (of_set_tuning key 1), slices of at least g_split_min_chunks chunks (key 2).
static int g_split_wgs = 4;
static int g_split_min_chunks = 12;
void plan_splits(GemmArgs& a, int kmax, int bk = BK) {
  a.splits = 1;
  a.k_per_split = (int)round_up(kmax, bk);
  if (a.tiles_total >= 2 * device_cus()) return;
  const int nchunks = (int)cdiv(kmax, bk);
  int s = std::max(1, (g_split_wgs * device_cus()) / a.tiles_total);
  s = std::min(s, std::max(1, nchunks / (bk == BK ? g_split_min_chunks : g_split_min_chunks / 2)));
  if (s <= 1) return;
  a.k_per_split = (int)round_up(cdiv(kmax, s), bk);
  a.splits = (int)cdiv(kmax, a.k_per_split);
}

int64_t slab_rows(const GemmArgs& a) { return (int64_t)(a.tiles_total / a.n_tiles) * a.bm; }

size_t fd_workspace(const GemmArgs& a) {
  if (a.splits <= 1) return 0;
  return (size_t)a.splits * slab_rows(a) * round_up(a.N, 4) * sizeof(float);
}

// Attach the split-K slab; without (enough) workspace fall back to one K slice.
void attach_slab(GemmArgs& a, void* ws, size_t ws_bytes, int bk = BK) {
  if (a.splits > 1 && ws && ws_bytes >= fd_workspace(a)) {
    a.slab = static_cast<float*>(ws);
    a.slab_ld = (int)round_up(a.N, 4);
    a.split_stride = slab_rows(a) * a.slab_ld;
    return;
  }
  int kmax = 0;
  for (int g = 0; g < a.ngroups; ++g) kmax = std::max(kmax, a.grp[g].K);
  a.splits = 1;
  a.k_per_split = (int)round_up(kmax, bk);
}

// bf16: K in units of k padded to BKH, B = W16_f [cout_p rows][kf16] (row length ldb).
GemmArgs fwd_args(const of_conv_desc* d, const Geo& g, bool bf16 = false) {
  GemmArgs a = base_args(d);
  a.kc = g.cin_p;
  a.N = d->cout;
  a.M = d->n * d->ho * d->wo;
  const int K = bf16 ? g.kf16 : g.kf;
  single_group(a, d, a.M, K);
  plan_splits(a, K, bf16 ? BKH : BK);
  a.ldb = bf16 ? g.kf16 : g.nf;
  a.nb = bf16 ? d->cout : g.nf;
  return a;
}

// skip_empty: the output already holds the added gradient (in-place accumulation, dx == add),
// so the stride-2 phase groups that no tap reaches (3 of 4 for a 1x1 stride-2 projection)
// launch no tiles at all instead of rewriting dx = add.  Splits stay as planned for the
// full grid, so the slab fits of_conv2d_dgrad_workspace().
GemmArgs dgrad_args(const of_conv_desc* d, const Geo& g, bool bf16 = false,
                    bool skip_empty = false) {
  GemmArgs a = base_args(d);
  a.kc = g.cout_p;
  a.N = g.cin_p;
  a.ldb = bf16 ? (int)g.kd16 : g.nd;
  a.nb = g.nd;
  int kmax = 0;
  if (g.phase) {
    a.phase = 1;
    a.dt = 2;
    a.ngroups = 4;
    a.bm = pick_bm(a.N);
    a.n_tiles = (int)cdiv(a.N, pick_bn(a.N));
    int tiles = 0;
    for (int c = 0; c < 4; ++c) {
      Group& G = a.grp[c];
      G = Group{};
      const int qy = c >> 1, qx = c & 1;
      // input rows iy with (iy + pt) % 2 == qy  ->  iy = 2u + ry
      G.ry = (((qy - d->pad_top) % 2) + 2) % 2;
      G.rx = (((qx - d->pad_left) % 2) + 2) % 2;
      G.hc = std::max(0, (d->h - G.ry + 1) / 2);
      G.wc = std::max(0, (d->w - G.rx + 1) / 2);
      G.M = d->n * G.hc * G.wc;
      G.m_tiles = (int)cdiv(G.M, a.bm);
      G.tiles_begin = tiles;
      tiles += G.m_tiles;
      G.r0 = g.pg.r0[c];
      G.s0 = g.pg.s0[c];
      G.ns = g.pg.ns[c];
      G.ntaps = g.pg.ntaps[c];
      const int64_t* rb = bf16 ? g.pg.row_begin16 : g.pg.row_begin;
      G.K = (int)(rb[c + 1] - rb[c]);
      G.b_off = rb[c];
      kmax = std::max(kmax, G.K);
    }
    a.tiles_total = tiles * a.n_tiles;
    a.M = d->n * d->h * d->w;
  } else {
    a.M = d->n * d->h * d->w;
    kmax = (int)(bf16 ? g.kd16 : g.kd);
    single_group(a, d, a.M, kmax);
  }
  plan_splits(a, kmax, bf16 ? BKH : BK);
  if (skip_empty && a.phase) {
    int tiles = 0;
    for (int c = 0; c < 4; ++c) {
      Group& G = a.grp[c];
      if (G.ntaps == 0) G.m_tiles = 0;
      G.tiles_begin = tiles;
      tiles += G.m_tiles;
    }
    a.tiles_total = tiles * a.n_tiles;
  }
  return a;
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// The tile kernels' 4-column epilogue (epilogue_store4) needs whole float4 columns and
// 16-byte aligned rows in every tensor it touches.
static int g_vec_ep = 1;   // of_set_tuning key 3 (0: per-element epilogue, for A/B and tests)
// of_set_tuning key 4: conv_wgrad_tile_x3b for Cout % 128 == 0 (1, default), for every
// x3 weight gradient (2), or never (0: the 3-tap form).  Measured per layer (same box): the
// 9-tap form +6-11 % on the Cout = 128 layers, even on Cout 96 / 64, -6 % on Cout 32.
static int g_wgx3b = 1;
// of_set_tuning key 5: conv_wgrad_tile_x3b wave shape, 16 MI ci x 32 / MI co (MI = 1 or 2).
// MI = 2 halves the dy loads and splits per MFMA and measured the same (dec3.c1 0.516 vs
// 0.517 ms): the split VALU is not what bounds the kernel.
static int g_wgx3b_mi = 1;
// of_set_tuning key 33: at least this many K tiles per split-K slice of the 9-tap weight
// gradients (conv_wgrad_tile_x3b / _b16).  Every slice writes a 9 x cin x cout fp32 slab that
// wgrad_reduce_kernel reads back: with one slice per CU the slabs are a fixed ~38 MB per launch
// whatever the layer's size.  2 (default): fp32 B=8 650.1 / 646.9 -> 655.4 / 655.0 pairs/s, bf16
// B=32 1803.0 / 1813.7 -> 1814.2 / 1816.2 at 4 (one box, gpurun_out/ab33); 4: +0.4 %, 8: -0.7 %.
static int g_wgx3_min_tiles = 2;
// of_set_tuning key 11: the 32 x 64 channel-block weight gradient (cfg 4) for Cout 64 layers
// whose Cin is not a multiple of 64 (1, default) or the 64 x 64 blocks (0).
static int g_wgx3_c4 = 1;
// of_set_tuning key 6: the other shapes' fp32 weight gradient on the split-bf16 implicit GEMM
// (conv_wgrad_x3, 1) or on the fp32 MFMA GEMM (0).
static int g_wgx3_gemm = 1;
// of_set_tuning key 12: bf16 3x3 stride-1 fwd / dgrad on conv_tile_b16 (1) or on the round-1
// conv_tile_bf16 (0, default).  key 13: the weight gradient on conv_wgrad_tile_b16 (1) or
// conv_wgrad_tile_bf16 (0, default).  Measured (bf16 B=32 bench, one box): the split kernels'
// structure with one plane is not faster for bf16 -- 1280 pairs/s with both against 1381 --
// fwd even (564 vs 578 TFLOP/s at 8 x 32 x 128), dgrad BN 128 4 x 32 +8 %, weight gradient
// 427 vs 449 TFLOP/s (Cout 128), 167 vs 364 (Cout 32): with one MFMA per fragment pair the
// per-tap staging and barriers of that structure are no longer hidden.
static int g_wgrad_b16 = 0;
bool vec_ep_ok(const GemmArgs& a) {
  if (!g_vec_ep || a.N % 4) return false;
  if (a.slab && !(a.slab_ld % 4 == 0 && a.split_stride % 4 == 0 && al16(a.slab))) return false;
  if (a.splits > 1) return a.slab != nullptr;
  auto ok = [](const float* p, int ld) { return !p || (ld % 4 == 0 && al16(p)); };
  return ok(a.C, a.ldc) && ok(a.res, a.ldr) && ok(a.z, a.ldz) && ok(a.act_src, a.ld_act);
}

// fwd/dgrad split-K epilogue: the flat kernel unless many slices meet few rows.
template <int MODE>
int launch_splitk_epilogue(const GemmArgs& a, hipStream_t s) {
  const int64_t items = slab_rows(a) * cdiv(a.N, 4);
  if (a.splits > 8 && items < 65536) {
    hipLaunchKernelGGL(splitk_epilogue_kernel<MODE>, dim3(cdiv(items, EP_ITEMS)), dim3(256), 0,
                       s, a);
    return check_launch("conv_splitk_epilogue");
  }
  bool vec = a.N % 4 == 0 && a.ldc % 4 == 0 && al16(a.C);
  if (a.res) vec = vec && a.ldr % 4 == 0 && al16(a.res);
  if (MODE == MODE_FWD && a.z) vec = vec && a.ldz % 4 == 0 && al16(a.z);
  if (MODE == MODE_DGRAD && a.act_src) vec = vec && a.ld_act % 4 == 0 && al16(a.act_src);
  const dim3 grid((unsigned)std::min<int64_t>(cdiv(items, 256), 8 * device_cus()));
  if (vec) hipLaunchKernelGGL((splitk_epilogue_flat<MODE, true>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((splitk_epilogue_flat<MODE, false>), grid, dim3(256), 0, s, a);
  return check_launch("conv_splitk_epilogue");
}

// Timing kinds: mode * 8 + tile config (0: 128x128, 1: 128x96, 2: 256x64, 3: 256x32) -- one
// per conv_gemm_f32 template instance.
template <int MODE>
int launch_gemm(const GemmArgs& a, hipStream_t s, double flops) {
  const int bn = pick_bn(a.N);
  dim3 grid(a.tiles_total * a.splits), block(256);
  const int cfg = bn == 128 ? 0 : bn == 96 ? 1 : bn == 64 ? 2 : 3;
  if (timing_on()) timing_begin(s);
  if (cfg == 0) hipLaunchKernelGGL((conv_gemm_f32<128, 128, 2, 2, MODE>), grid, block, 0, s, a);
  else if (cfg == 1) hipLaunchKernelGGL((conv_gemm_f32<128, 96, 4, 1, MODE>), grid, block, 0, s, a);
  else if (cfg == 2) hipLaunchKernelGGL((conv_gemm_f32<256, 64, 4, 1, MODE>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((conv_gemm_f32<256, 32, 4, 1, MODE>), grid, block, 0, s, a);
  if (timing_on()) timing_end(s, MODE * 8 + cfg, flops);
  int st = check_launch("conv_gemm_f32");
  if (st || MODE == MODE_WGRAD || a.splits == 1) return st;
  return launch_splitk_epilogue<MODE>(a, s);
}

// bf16 instances: timing kinds 64 + mode * 8 + tile config.
template <int MODE>
int launch_gemm_bf16(const GemmArgs& a, hipStream_t s, double flops) {
  const int bn = pick_bn(a.N);
  dim3 grid(a.tiles_total * a.splits), block(256);
  const int cfg = bn == 128 ? 0 : bn == 96 ? 1 : bn == 64 ? 2 : 3;
  if (timing_on()) timing_begin(s);
  if (cfg == 0) hipLaunchKernelGGL((conv_gemm_bf16<128, 128, 2, 2, MODE>), grid, block, 0, s, a);
  else if (cfg == 1) hipLaunchKernelGGL((conv_gemm_bf16<128, 96, 4, 1, MODE>), grid, block, 0, s, a);
  else if (cfg == 2) hipLaunchKernelGGL((conv_gemm_bf16<256, 64, 4, 1, MODE>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((conv_gemm_bf16<256, 32, 4, 1, MODE>), grid, block, 0, s, a);
  if (timing_on()) timing_end(s, 64 + MODE * 8 + cfg, flops);
  int st = check_launch("conv_gemm_bf16");
  if (st || a.splits == 1) return st;
  return launch_splitk_epilogue<MODE>(a, s);
}

// bf16 3x3 stride-1 fwd / dgrad: halo-tiled kernel (conv_tile_bf16).
bool tile_ok(const of_conv_desc* d) { return d->kh == 3 && d->kw == 3 && d->stride == 1; }

// conv_tile_x3 with BN = 128 or 96 takes X3_TH0 x 32 output tiles (twice the MFMAs per staged
// B tap) when that still leaves >= 4 workgroups per CU, else 4 x 32.
bool x3_tall(int n, int oh, int ow, int N) {
  const int bn = pick_bn(N);
  return (bn == 128 || bn == 96) && (int64_t)n * cdiv(oh, X3_TH0) * cdiv(ow, TF_W) >= 4 * device_cus();
}

// conv_tile_x3 BN = 128 with 4 x 32 tiles: unsplit grids of >= X3_NB1_MIN tiles take the
// single-buffered 4-wave form (two workgroups per CU: enc.l3 142 -> 154, dec2 dgrad 170 ->
// 185 TFLOP/s); split grids keep the 8-wave double-buffered one (the 4-wave
// form measured dec1 134 -> 108, enc.l4 159 -> 143).  x3_nb1_candidate() only sizes the
// K-split cost model (two slots per CU); the launch takes the 4-wave form when the final
// plan is also unsplit (x3_nb1).
constexpr int X3_NB1_MIN = 384;
bool x3_nb1_candidate(const GemmArgs& a, bool tall) {
  return !tall && a.bn_tile == 0 && pick_bn(a.N) == 128 && a.tiles_total >= X3_NB1_MIN;
}
bool x3_nb1(const GemmArgs& a) {
  return a.bm != X3_TH0 * TF_W && a.splits == 1 && x3_nb1_candidate(a, false);
}

// conv_tile_ws: bf16 layers whose N tile is 128 or 96, forward and input gradient
// (of_set_tuning key 12 = 2) or forward only (key 12 = 3).
static int g_tile_b16 = 0;
bool ws_ok(const of_conv_desc* d, int mode) {
  const int N = mode == MODE_FWD ? d->cout : d->cin_p;
  return (g_tile_b16 == 2 || (g_tile_b16 == 3 && mode == MODE_FWD)) && pick_bn(N) >= 96;
}

// of_set_tuning keys 25 / 26: the K-split cost models' slab-pass term, in tenths of a chunk per
// slice and tile round, of the halo-tile kernels (tile_args) and of conv_gemm_x3 (gemm_x3_plan).
static int g_x3t_ep = 5;
static int g_x3g_ep = 5;
static int g_x3_small_bn = 1200;
// of_set_tuning key 36: the fp32 split 3x3 form for 64-column N tiles.  0: conv_tile_x3<64, 4,
// 2, MODE, 4> (8 waves of 32 px x 32 columns: 2 MFMAs per fragment read, LDS-read-bound);
// 1: the 4-wave single-buffered 8 x 32 form (64 px x 64 columns per wave: 4 MFMAs per read, as
// the BN = 128 8 x 32 form) on grids that stay large enough, else 0; 2: <64, 4, 1, MODE, 4, 1>
// (32 px x 64 columns: 2.67); 3: <64, 2, 2, MODE, 4, 1> (64 px x 32 columns: 2.67).
static int g_x3_bn64 = 0;
// of_set_tuning key 39: timing ablation -- the split 3x3 input gradients without their act'
// source reads (RESULTS ARE WRONG: the derivative taken as 1; A/B timing only; default 0)
static int g_abl_noact = 0;
GemmArgs tile_args(const of_conv_desc* d, const Geo& g, int mode, bool x3 = false,
                   bool b16 = false, bool ws = false) {
  GemmArgs a = base_args(d);
  const bool fwd = mode == MODE_FWD;
  a.kc = fwd ? g.cin_p : g.cout_p;
  a.N = fwd ? d->cout : g.cin_p;
  a.nb = fwd ? d->cout : g.nd;
  a.ldb = fwd ? g.kf16 : (int)g.kd16;
  const int OH = fwd ? d->ho : d->h, OW = fwd ? d->wo : d->w;
  // of_set_tuning key 27: fp32 split layers whose BN = 128 grid of 4 x 32 tiles has fewer than
  // g_x3_small_bn workgroups run BN = 64 tiles instead (conv_tile_x3<64, ...>: 64 KB of LDS, two
  // workgroups per CU, twice the N tiles): the coarse levels' grids (enc.l4, dec0 / dec1 heads)
  // leave CUs idle at BN = 128 with one workgroup per CU.
  if (x3 && !b16 && !ws && g_x3_small_bn > 0 && pick_bn(a.N) == 128 &&
      (int64_t)d->n * cdiv(OH, TF_H) * cdiv(OW, TF_W) * cdiv(a.N, 128) < g_x3_small_bn)
    a.bn_tile = 64;
  // of_set_tuning key 36 = 1: fp32 split layers with N = 64 on the 4-wave 8 x 32 form
  // (conv_tile_x3<64, 4, 1, MODE, X3_TH0, 1>) where that grid keeps >= 4 workgroups per CU
  const bool tall64 = x3 && !b16 && !ws && !a.bn_tile && g_x3_bn64 == 1 && pick_bn(a.N) == 64 &&
                      (int64_t)d->n * cdiv(OH, X3_TH0) * cdiv(OW, TF_W) >= 4 * device_cus();
  // bf16: fwd only (8 x 32 tiles measured +5 % on dec3 fwd, -2 % on dgrad); conv_tile_ws: always
  const bool tall = tall64 ? true : a.bn_tile ? false : ws ? true
                  : x3 || b16 ? x3_tall(d->n, OH, OW, a.N)
                             : (fwd || g_tall16_dgrad) && pick_bn(a.N) == 128 &&
                                   x3_tall(d->n, OH, OW, a.N);
  const int th = tall ? X3_TH0 : TF_H;
  const int m_tiles = d->n * (int)cdiv(OH, th) * (int)cdiv(OW, TF_W);
  a.bm = th * TF_W;
  a.ngroups = 1;
  Group& G = a.grp[0];
  G = Group{};
  G.M = d->n * OH * OW;
  G.m_tiles = m_tiles;
  G.ns = 3;
  G.ntaps = 9;
  a.M = G.M;
  a.n_tiles = (int)cdiv(a.N, a.bn_tile ? a.bn_tile : pick_bn(a.N));
  a.tiles_total = m_tiles * a.n_tiles;
  a.K = (int)cdiv(a.kc, 32);                       // channel chunks
  G.K = a.K;
  a.splits = 1;
  a.k_per_split = a.K;
  if (x3 || b16 || ws) {
    // One workgroup per CU (conv_tile_b16: two): choose the K split with the least modelled time, in units of one
    // chunk (9 taps): rounds of 256 workgroups x (chunks per slice + 1 for prologue and
    // epilogue), plus 0.5 per slice and tile round for the slab write and epilogue pass.
    // (Measured: enc.l3 384 tiles unsplit, dec1 192 tiles unsplit, enc.l4 96 tiles in 2.)
    // (The single-buffered BN = 128 4 x 32 configuration, used from X3_NB1_MIN tiles, runs
    // two workgroups per CU.)
    const bool bn64 = x3 && !b16 && !ws && (a.bn_tile ? a.bn_tile : pick_bn(a.N)) == 64;
    const int slots = !ws && ((b16 && !tall) || x3_nb1_candidate(a, tall) || a.bn_tile == 64 ||
                              (g_x3_bn64 && bn64))
                          ? 2 * device_cus() : device_cus();
    int best = 1;
    double best_cost = 1e30;
    for (int sp = 1; sp <= std::min(8, a.K); ++sp) {
      const int per = (int)cdiv(a.K, sp);
      if (cdiv(a.K, per) != sp) continue;            // not a distinct slice count
      const int64_t w = (int64_t)a.tiles_total * sp;
      const double cost = (double)cdiv(w, slots) * (per + 1.0) +
                          (sp > 1 ? 0.1 * g_x3t_ep * sp * a.tiles_total / (double)slots : 0.0);
      if (cost < best_cost - 1e-9) {
        best_cost = cost;
        best = sp;
      }
    }
    a.k_per_split = (int)cdiv(a.K, best);
    a.splits = (int)cdiv(a.K, a.k_per_split);
  } else if (a.tiles_total < 2 * device_cus()) {
    int sp = std::max(1, (4 * device_cus()) / a.tiles_total);
    sp = std::min(sp, std::max(1, a.K / 2));       // >= 2 chunks (6 tap rows) per slice
    a.k_per_split = (int)cdiv(a.K, sp);
    a.splits = (int)cdiv(a.K, a.k_per_split);
  }
  return a;
}

template <int MODE>
int launch_tile_bf16(const GemmArgs& a, hipStream_t s, double flops) {
  const int bn = pick_bn(a.N);
  dim3 grid(a.tiles_total * a.splits), block(256);
  const bool tall = a.bm == X3_TH0 * TF_W;
  const int cfg = bn == 128 ? (tall ? 4 : 0) : bn == 96 ? 1 : bn == 64 ? 2 : 3;
  if (timing_on()) timing_begin(s);
  if (!g_tile16_pf) {
    if (cfg == 4) hipLaunchKernelGGL((conv_tile_bf16<128, 4, 2, MODE, X3_TH0, 0>), grid, dim3(512), 0, s, a);
    else if (cfg == 0) hipLaunchKernelGGL((conv_tile_bf16<128, 2, 2, MODE, OF_TF_H, 0>), grid, block, 0, s, a);
    else if (cfg == 1) hipLaunchKernelGGL((conv_tile_bf16<96, 4, 1, MODE, OF_TF_H, 0>), grid, block, 0, s, a);
    else if (cfg == 2) hipLaunchKernelGGL((conv_tile_bf16<64, 2, 2, MODE, OF_TF_H, 0>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv_tile_bf16<32, 4, 1, MODE, OF_TF_H, 0>), grid, block, 0, s, a);
  } else if (cfg == 4) hipLaunchKernelGGL((conv_tile_bf16<128, 4, 2, MODE, X3_TH0>), grid, dim3(512), 0, s, a);
  else if (cfg == 0) hipLaunchKernelGGL((conv_tile_bf16<128, 2, 2, MODE>), grid, block, 0, s, a);
  else if (cfg == 1) hipLaunchKernelGGL((conv_tile_bf16<96, 4, 1, MODE>), grid, block, 0, s, a);
  else if (cfg == 2) hipLaunchKernelGGL((conv_tile_bf16<64, 2, 2, MODE>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((conv_tile_bf16<32, 4, 1, MODE>), grid, block, 0, s, a);
  if (timing_on()) timing_end(s, 64 + 32 + MODE * 8 + cfg, flops);
  int st = check_launch("conv_tile_bf16");
  if (st || a.splits == 1) return st;
  return launch_splitk_epilogue<MODE>(a, s);
}

struct WgradPlan {
  int splits, k_per_split, M, ldc;
  int64_t split_stride;
};

// fp32 3x3 stride-1 fwd / dgrad on the split-bf16 kernel: timing kinds 128 + mode * 8 + cfg.
template <int MODE>
int launch_tile_x3(const GemmArgs& a, hipStream_t s, double flops) {
  const int bn = a.bn_tile ? a.bn_tile : pick_bn(a.N);
  dim3 grid(a.tiles_total * a.splits), block(256);
  const bool tall = a.bm == X3_TH0 * TF_W;
  const int cfg = bn == 128 ? (tall ? 0 : x3_nb1(a) ? 4 : 6)
                            : bn == 96 ? (tall ? 5 : 1)
                            : bn == 64 ? (tall || g_x3_bn64 >= 2 ? 7 : 2) : 3;
  if (timing_on()) timing_begin(s);
  if (cfg == 7) {                         // of_set_tuning key 36
    if (tall) hipLaunchKernelGGL((conv_tile_x3<64, 4, 1, MODE, X3_TH0, 1>), grid, block, 0, s, a);
    else if (g_x3_bn64 == 2) hipLaunchKernelGGL((conv_tile_x3<64, 4, 1, MODE, 4, 1>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv_tile_x3<64, 2, 2, MODE, 4, 1>), grid, block, 0, s, a);
  } else if (cfg == 0) hipLaunchKernelGGL((conv_tile_x3<128, 4, 2, MODE, X3_TH0>), grid, dim3(512), 0, s, a);
  else if (cfg == 4) hipLaunchKernelGGL((conv_tile_x3<128, 2, 2, MODE, 4, 1>), grid, block, 0, s, a);
  else if (cfg == 6) hipLaunchKernelGGL((conv_tile_x3<128, 2, 4, MODE, 4>), grid, dim3(512), 0, s, a);
  else if (cfg == 5) hipLaunchKernelGGL((conv_tile_x3<96, 4, 3, MODE, X3_TH0>), grid, dim3(768), 0, s, a);
  else if (cfg == 1) hipLaunchKernelGGL((conv_tile_x3<96, 2, 3, MODE, 4>), grid, dim3(384), 0, s, a);
  else if (cfg == 2) hipLaunchKernelGGL((conv_tile_x3<64, 4, 2, MODE, 4>), grid, dim3(512), 0, s, a);
  else hipLaunchKernelGGL((conv_tile_x3<32, 4, 1, MODE, 4>), grid, block, 0, s, a);
  if (timing_on()) timing_end(s, 128 + MODE * 8 + cfg, flops);
  int st = check_launch("conv_tile_x3");
  if (st || a.splits == 1) return st;
  return launch_splitk_epilogue<MODE>(a, s);
}

// bf16 3x3 stride-1 fwd / dgrad on conv_tile_b16: timing kinds 192 + mode * 8 + cfg (the
// conv_tile_x3 configurations; cfg 4, the single-buffered one, is not used).
template <int MODE>
int launch_tile_b16(const GemmArgs& a, hipStream_t s, double flops) {
  const int bn = pick_bn(a.N);
  dim3 grid(a.tiles_total * a.splits);
  const bool tall = a.bm == X3_TH0 * TF_W;
  const int cfg = bn == 128 ? (tall ? 0 : 6) : bn == 96 ? (tall ? 5 : 1) : bn == 64 ? 2 : 3;
  if (timing_on()) timing_begin(s);
  if (cfg == 0) hipLaunchKernelGGL((conv_tile_b16<128, 4, 2, MODE, X3_TH0>), grid, dim3(512), 0, s, a);
  else if (cfg == 6) hipLaunchKernelGGL((conv_tile_b16<128, 2, 4, MODE, 4>), grid, dim3(512), 0, s, a);
  else if (cfg == 5) hipLaunchKernelGGL((conv_tile_b16<96, 4, 3, MODE, X3_TH0>), grid, dim3(768), 0, s, a);
  else if (cfg == 1) hipLaunchKernelGGL((conv_tile_b16<96, 2, 3, MODE, 4>), grid, dim3(384), 0, s, a);
  else if (cfg == 2) hipLaunchKernelGGL((conv_tile_b16<64, 4, 2, MODE, 4>), grid, dim3(512), 0, s, a);
  else hipLaunchKernelGGL((conv_tile_b16<32, 4, 1, MODE, 4>), grid, dim3(256), 0, s, a);
  if (timing_on()) timing_end(s, 192 + MODE * 8 + cfg, flops);
  int st = check_launch("conv_tile_b16");
  if (st || a.splits == 1) return st;
  return launch_splitk_epilogue<MODE>(a, s);
}

// bf16 3x3 stride-1 fwd / dgrad on conv_tile_ws: timing kinds 224 + mode * 8 + cfg
// (0: BN 128, 1: BN 96; 8 x 32 output tiles, 4 compute + 4 staging waves).
template <int MODE>
int launch_tile_ws(const GemmArgs& a, hipStream_t s, double flops) {
  if (timing_on()) timing_begin(s);
  int st = launch_tile_ws_kernel(a, MODE, s);
  if (timing_on()) timing_end(s, 224 + MODE * 8 + (pick_bn(a.N) == 128 ? 0 : 1), flops);
  if (st || a.splits == 1) return st;
  return launch_splitk_epilogue<MODE>(a, s);
}

// fp32 implicit GEMM on the split-bf16 kernel (conv_gemm_x3, every non-3x3-stride-1 shape):
// BN 128 (8 waves of 32 x 64) for N > 64, else 256 x 64 tiles; one workgroup per CU, so K
// splits come from the cost model of tile_args (rounds of 256 workgroups x (chunks per slice
// + 1) + half a chunk per slice and tile round for the slab pass).  Timing kinds 160 + 8 mode
// + (0: 128 x 128, 1: 256 x 64).
void gemm_x3_plan(GemmArgs& a) {
  const int bm = a.N > 64 ? 128 : 256, bn = a.N > 64 ? 128 : 64;
  int tiles = 0, tiles_all = 0, kmax = 0;
  for (int g = 0; g < a.ngroups; ++g) {
    Group& G = a.grp[g];
    if (G.m_tiles) G.m_tiles = (int)cdiv(G.M, bm);   // (phase groups skipped in place stay 0)
    G.tiles_begin = tiles;
    tiles += G.m_tiles;
    tiles_all += (int)cdiv(G.M, bm);
    kmax = std::max(kmax, G.K);
  }
  a.bm = bm;
  a.n_tiles = (int)cdiv(a.N, bn);
  a.tiles_total = tiles * a.n_tiles;
  // the split is planned on the full grid, so of_conv2d_dgrad_x3_workspace() covers the
  // in-place form (fewer tiles, fewer slab rows) too
  const int64_t plan_tiles = (int64_t)tiles_all * a.n_tiles;
  const int chunks = (int)cdiv(kmax, BKH);
  int best = 1;
  double best_cost = 1e30;
  for (int sp = 1; sp <= std::min(8, chunks); ++sp) {
    const int per = (int)cdiv(chunks, sp);
    if (cdiv(chunks, per) != sp) continue;
    const int64_t w = plan_tiles * sp;
    const double cost = (double)cdiv(w, device_cus()) * (per + 1.0) +
                        (sp > 1 ? 0.1 * g_x3g_ep * sp * plan_tiles / (double)device_cus() : 0.0);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = sp;
    }
  }
  a.k_per_split = (int)cdiv(chunks, best) * BKH;
  a.splits = (int)cdiv(kmax, a.k_per_split);
}

// of_set_tuning key 30: conv_gemm_x3 on a DMA ring of 3 slots (1: one chunk in flight across
// each barrier, one workgroup per CU) or of 2 slots (2, default: two workgroups per CU where
// the LDS allows -- the fp32 128 x 128 form; the 256 x 64 form keeps 3 slots), or on the
// round-2..4 register-staged A with one chunk in flight (0).  Bitwise the same results.
// Measured (tools/conv_bench.py, one box): enc.l3.c0 fwd 81 / 84 / 71 us for 0 / 1 / 2,
// enc.l4.c0 fwd 69 / 72 / 60, dgrad 77 / 79 / 69; the bench step even (626-628 pairs/s).
static int g_gx3_ring = 2;
// (NP = 1, the bf16 form: timing kinds 240 + mode * 8 + cfg)
template <int MODE, int NP = 3>
int launch_gemm_x3(const GemmArgs& a, hipStream_t s, double flops) {
  const int cfg = a.N > 64 ? 0 : 1;
  dim3 grid(a.tiles_total * a.splits), block(512);
  if (timing_on()) timing_begin(s);
  if (g_gx3_ring == 1) {
    if (cfg == 0) hipLaunchKernelGGL((conv_gemm_x3<128, 128, 4, 2, MODE, NP, 3>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv_gemm_x3<256, 64, 8, 1, MODE, NP, 3>), grid, block, 0, s, a);
  } else if (g_gx3_ring == 2) {
    if (cfg == 0) hipLaunchKernelGGL((conv_gemm_x3<128, 128, 4, 2, MODE, NP, 2>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv_gemm_x3<256, 64, 8, 1, MODE, NP, 2>), grid, block, 0, s, a);
  } else {
    if (cfg == 0) hipLaunchKernelGGL((conv_gemm_x3<128, 128, 4, 2, MODE, NP, 0>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv_gemm_x3<256, 64, 8, 1, MODE, NP, 0>), grid, block, 0, s, a);
  }
  if (timing_on()) timing_end(s, (NP == 1 ? 240 : 160) + MODE * 8 + cfg, flops);
  int st = check_launch("conv_gemm_x3");
  if (st || a.splits == 1) return st;
  return launch_splitk_epilogue<MODE>(a, s);
}

// bf16 3x3 stride-1 wgrad on conv_wgrad_tile_bf16: block channel tiles (CIB x COB).
// bf16: every 3x3 stride-1 layer.  fp32 (MFMA-bound either way): where the implicit GEMM
// loses to its N = 64 tiles or to many small split-K slabs (measured, tools/conv_bench.py):
// Cout = 64, or Cout % 128 == 0 on up to 8 x 96 x 128 output pixels.
bool wgt_ok(const of_conv_desc* d, bool bf16) {
  if (!tile_ok(d)) return false;
  if (bf16) return true;
  const int64_t npix = (int64_t)d->n * d->ho * d->wo;
  return d->cout == 64 || (d->cout % 128 == 0 && npix <= 8 * 96 * 128);
}
int wgt_cfg(const of_conv_desc* d) { return d->cout > 64 ? 0 : 2; }   // <1,4> : <2,2>
void wgt_blocks(const of_conv_desc* d, int& cib, int& cob) {
  cib = wgt_cfg(d) == 0 ? 32 : 64;
  cob = wgt_cfg(d) == 0 ? 128 : 64;
}

// fp32 wgrad on conv_wgrad_tile_x3, 3x3 stride 1, by Cout: channel blocks (CIB x COB)
// 32 x 128 (cfg 0, Cout % 128 == 0), 32 x 96 (cfg 1, Cout 96), 64 x 64 (cfg 2, Cout 64),
// 64 x 32 (cfg 3, Cout 32), 32 x 64 (cfg 4: Cout 64 with Cin not a multiple of 64 -- the
// 96 -> 64 flow-head convs, whose second 64-channel input block was half empty; 9-tap form
// only); other layers keep the fp32 wgrad kernels.
int wgx3_cfg(const of_conv_desc* d) {
  if (!tile_ok(d)) return -1;
  if (d->cout == 64) return d->cin_p % 64 == 0 || !g_wgx3_c4 ? 2 : 4;
  return d->cout % 128 == 0 ? 0 : d->cout == 96 ? 1 : d->cout == 32 ? 3 : -1;
}
bool wgx3_ok(const of_conv_desc* d) { return wgx3_cfg(d) >= 0; }
void wgx3_blocks(const of_conv_desc* d, int& cib, int& cob) {
  const int c = wgx3_cfg(d);
  cib = c == 2 || c == 3 ? 64 : 32;
  cob = c == 0 ? 128 : c == 1 ? 96 : c == 2 || c == 4 ? 64 : 32;
}

// of_set_tuning key 14: the stem's fp32 weight gradient (3 input channels) on
// conv_wgrad_stem_x3 (1, default) or on the fp32 MFMA GEMM (0).
static int g_stem_wg = 1;
// (3 real input channels: the kernel's M rows are the 49 x 3 real (tap, ci) pairs)
bool stem_wg_ok(const of_conv_desc* d) { return g_stem_wg && stem_x3_ok(d) && d->cin == 3; }
int stem_wg_tiles(const of_conv_desc* d) {
  return d->n * (int)cdiv(d->ho, SW_TH) * (int)cdiv(d->wo, SW_TW);
}

// of_set_tuning key 10: fp32 / bf16 GEMM weight-gradient split-K target workgroups per CU.
static int g_wgrad_wgs = 4;
// of_set_tuning key 23: the split 3x3 kernels' direct epilogues (conv_dev.h), bit 0 the
// forward's (direct_fwd_f32), bit 1 the input gradient's (direct_dgrad_f32); a clear bit keeps
// the per-pass transposes.  Default 1: the input gradient's measured slower (per layer dec3.c1
// 0.506 -> 0.531 ms, c2 0.413 -> 0.426; fp32 step 651.8 -> 650.6 pairs/s, profiles/r4_late/step_ab.txt).
static int g_x3_direct = 1;
// of_set_tuning key 32: bf16 input gradients that carry BN partial sums
// (of_conv2d_dgrad_add_act_bnp) on conv_tile_b16, whose one-slice vectorised epilogue forms
// them (1), or declined (0, default: the caller's separate reduction pass, conv_tile_bf16).
// Measured (bf16 B = 32 bench, one box, two interleaved rounds): 1750.1 / 1750.9 pairs/s
// declined, 1721.6 / 1716.3 fused -- conv_tile_b16 loses more on these input gradients than
// the side-stream reductions cost.
static int g_bnp_b16 = 0;

// of_set_tuning key 16: which bf16 implicit GEMMs (stride-2 block convs, 1x1 projections; the
// stem when key 15 = 0) run on the one-plane conv_gemm_x3 / conv_wgrad_x3 forms instead of
// conv_gemm_bf16 / conv_wgrad_bf16: bit 0 forward, bit 1 input gradient, bit 2 weight
// gradient.  Default 6: measured per layer at bf16 B = 32 (tools/gpu_r3n.sh), the one-plane
// input and weight gradients are faster (0.77 -> 0.71, 0.46 -> 0.40 ms per step), the
// forward slower (0.31 -> 0.35 ms).
static int g_gemm_b16 = 6;
// of_set_tuning key 17: conv_wgrad_tile_bf16 with software-pipelined fragments (1, default)
// or the round-1 per-row reads (0).
static int g_wgt_pf = 1;
bool gemm_b16_wg(const of_conv_desc* d) {
  return (g_gemm_b16 & 4) && !narrow_ok(d) && !tile_ok(d) && !(stem_wg_ok(d) && g_stem_bf16);
}

WgradPlan wgrad_plan(const of_conv_desc* d, bool bf16 = false, bool x3 = false) {
  Geo g = geo(d);
  WgradPlan p;
  p.M = g.taps * g.cin_p;
  p.ldc = g.cout_p;
  p.split_stride = (int64_t)(p.M + 1) * p.ldc;   // + one row for the bias column sums
  if (stem_wg_ok(d) && (!bf16 || g_stem_bf16)) {
    // conv_wgrad_stem_x3: K = 4 x 32 output tiles, persistent workgroups (3 per CU)
    const int T = stem_wg_tiles(d);
    int splits = std::max(1, std::min(T, SW_WGS_PER_CU * device_cus()));
    p.k_per_split = (int)cdiv(T, splits);
    p.splits = (int)cdiv(T, p.k_per_split);
    return p;
  }
  if ((x3 || (bf16 && g_wgrad_b16)) && wgx3_ok(d)) {
    // K = 4 x 16 pixel tiles; one workgroup per CU, equal slices
    int cib, cob;
    wgx3_blocks(d, cib, cob);
    const int chan_tiles = (int)(cdiv(g.cin_p, cib) * cdiv(d->cout, cob));
    const int T = d->n * (int)cdiv(d->ho, wgx3_rows(wgx3_cfg(d))) * (int)cdiv(d->wo, TT_W);
    int splits = std::max(1, std::min(T, device_cus() / chan_tiles));
    splits = std::max(1, std::min(splits, T / g_wgx3_min_tiles));
    p.k_per_split = (int)cdiv(T, splits);
    p.splits = (int)cdiv(T, p.k_per_split);
    return p;
  }
  const bool g16 = bf16 && gemm_b16_wg(d);
  if ((x3 || g16) && !narrow_ok(d)) {
    // conv_wgrad_x3: 128 x (128 | 64) tiles, one workgroup per CU (two for the one-plane bf16
    // form); K = output pixels in 32-pixel chunks, split to fill the CUs with at least 8
    // chunks per slice
    const int K = d->n * d->ho * d->wo;
    const int tiles = (int)(cdiv(p.M, 128) * cdiv(d->cout, d->cout > 64 ? 128 : 64));
    int splits = std::max(1, (g16 ? 2 : 1) * device_cus() / tiles);
    splits = std::min(splits, (int)std::max<int64_t>(1, cdiv(K, 8 * BKH)));
    p.k_per_split = (int)round_up(cdiv(K, splits), BKH);
    p.splits = (int)cdiv(K, p.k_per_split);
    return p;
  }
  if (wgt_ok(d, bf16)) {
    // K = 8 x 16 pixel tiles; one workgroup per CU (LDS-bound occupancy), equal slices
    int cib, cob;
    wgt_blocks(d, cib, cob);
    const int chan_tiles = (int)(cdiv(g.cin_p, cib) * cdiv(d->cout, cob));
    const int T = d->n * (int)cdiv(d->ho, TT_H) * (int)cdiv(d->wo, TT_W);
    int splits = std::max(1, std::min(T, device_cus() / chan_tiles));
    p.k_per_split = (int)cdiv(T, splits);
    p.splits = (int)cdiv(T, p.k_per_split);
    return p;
  }
  const int bk = bf16 ? BKH : BK;
  const int K = d->n * d->ho * d->wo;
  const int tiles = (int)(cdiv(p.M, pick_bm(d->cout)) * cdiv(d->cout, pick_bn(d->cout)));
  // Fill up to g_wgrad_wgs (4) workgroups per CU without overshooting a multiple of the CU
  // count (an overshoot leaves a few CUs with one extra long-running workgroup: a tail).
  int splits = std::max(1, (g_wgrad_wgs * device_cus()) / tiles);
  splits = std::min(splits, (int)std::max<int64_t>(1, cdiv(K, 8 * bk)));
  p.k_per_split = (int)round_up(cdiv(K, splits), bk);
  p.splits = (int)cdiv(K, p.k_per_split);
  return p;
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
  return g.kd * g.nd;
}

int64_t of_conv_wfwd16_elems(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return -1;
  Geo g = geo(d);
  return (int64_t)g.cout_p * g.kf16;
}

int64_t of_conv_wbwd16_elems(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return -1;
  Geo g = geo(d);
  return g.kd16 * g.nd;
}

static PackEntry pack_entry(const of_conv_desc* d, const float* w, void* wf, void* wd,
                            int bf16) {
  const Geo g = geo(d);
  PackEntry E{};
  E.w = w;
  E.wf = static_cast<float*>(wf);
  E.wd = static_cast<float*>(wd);
  E.taps = g.taps;
  E.kw = d->kw;
  E.cin = d->cin;
  E.cout = d->cout;
  E.cin_p = g.cin_p;
  E.cout_p = g.cout_p;
  E.kf = g.kf;
  E.nf = g.nf;
  E.nd = g.nd;
  E.bf16 = bf16;
  E.kf16 = g.kf16;
  E.kd16 = g.kd16;
  E.pg = g.pg;
  return E;
}

static int64_t pack_work(const of_conv_desc* d, int bf16) {
  const Geo g = geo(d);
  return bf16 ? (int64_t)g.cout_p * g.kf16 + g.kd16 * g.nd : (int64_t)g.kf * g.nf + g.kd * g.nd;
}

// pack_many_kernel's shares of one entry: elements (bf16: the input-gradient image only) and
// forward-image tiles (bf16 only)
static int64_t pack_work_many(const of_conv_desc* d, int bf16) {
  const Geo g = geo(d);
  return bf16 ? g.kd16 * g.nd : (int64_t)g.kf * g.nf + g.kd * g.nd;
}
static int64_t pack_tiles16(const of_conv_desc* d, int bf16) {
  const Geo g = geo(d);
  return bf16 ? cdiv(g.cout_p, PK_TN) * cdiv(g.kf16, PK_TK) : 0;
}

int of_conv_pack_weights_bf16(const of_conv_desc* d, const float* w_hwio, void* w16_fwd,
                              void* w16_bwd, void* stream) {
  int st = validate(d);
  if (st) return st;
  OF_CHECK_ARG(w_hwio && w16_fwd && w16_bwd, "pack bf16: NULL pointer");
  const int64_t total = pack_work(d, 1);
  OF_CHECK_ARG(total < INT32_MAX, "pack: layer too large");
  const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 4096);
  hipLaunchKernelGGL(pack_one_kernel, dim3(blocks), dim3(256), 0, as_stream(stream),
                     pack_entry(d, w_hwio, w16_fwd, w16_bwd, 1), total);
  return check_launch("pack_bf16");
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
    const int64_t total = g.kd * g.nd;
    const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 4096);
    hipLaunchKernelGGL(pack_bwd_kernel, dim3(blocks), dim3(256), 0, s, w_hwio, g.pg, d->kw,
                       d->cin, d->cout, g.cout_p, g.nd, w_bwd);
    if ((st = check_launch("pack_bwd"))) return st;
  }
  return OF_OK;
}

int of_set_tuning(int key, int value) {
  if (key == 8 && value >= 0 && value <= 2) { g_stem_x3 = value; return OF_OK; }
  if (key == 7 && (value == 0 || value == 1)) { g_warp_win = value; return OF_OK; }
  if (key == 9 && value >= 0 && value <= 7) { g_corr_blk = value; return OF_OK; }
  if (key == 19 && (value == 0 || value == 1)) { g_corr_ty8 = value; return OF_OK; }
  if (key == 10 && value >= 1 && value <= 16) { g_wgrad_wgs = value; return OF_OK; }
  if (key == 11 && (value == 0 || value == 1)) { g_wgx3_c4 = value; return OF_OK; }
  if (key == 1 && value >= 1 && value <= 16) { g_split_wgs = value; return OF_OK; }
  if (key == 2 && value >= 2 && value <= 64) { g_split_min_chunks = value; return OF_OK; }
  if (key == 3 && (value == 0 || value == 1)) { g_vec_ep = value; return OF_OK; }
  if (key == 4 && value >= 0 && value <= 2) { g_wgx3b = value; return OF_OK; }
  if (key == 5 && (value == 1 || value == 2)) { g_wgx3b_mi = value; return OF_OK; }
  if (key == 6 && (value == 0 || value == 1)) { g_wgx3_gemm = value; return OF_OK; }
  if (key == 12 && value >= 0 && value <= 3) { g_tile_b16 = value; return OF_OK; }
  if (key == 13 && (value == 0 || value == 1)) { g_wgrad_b16 = value; return OF_OK; }
  if (key == 14 && (value == 0 || value == 1)) { g_stem_wg = value; return OF_OK; }
  if (key == 15 && (value == 0 || value == 1)) { g_stem_bf16 = value; return OF_OK; }
  if (key == 16 && value >= 0 && value <= 7) { g_gemm_b16 = value; return OF_OK; }
  if (key == 18 && (value == 0 || value == 1)) { g_tall16_dgrad = value; return OF_OK; }
  if (key == 17 && (value == 0 || value == 1)) { g_wgt_pf = value; return OF_OK; }
  if (key == 20 && (value == 0 || value == 1)) { g_tile16_pf = value; return OF_OK; }
  if (key == 21 && value >= 0 && value <= 3) { g_b16i_abl = value; return OF_OK; }
  if (key == 22 && (value == 0 || value == 1)) { g_b16i_direct = value; return OF_OK; }
  if (key == 23 && value >= 0 && value <= 3) { g_x3_direct = value; return OF_OK; }
  if (key == 24 && value >= 0 && value <= 2) { g_b16i_persist = value; return OF_OK; }
  if (key == 25 && value >= 0 && value <= 1000) { g_x3t_ep = value; return OF_OK; }
  if (key == 26 && value >= 0 && value <= 1000) { g_x3g_ep = value; return OF_OK; }
  if (key == 27 && value >= 0 && value <= 100000) { g_x3_small_bn = value; return OF_OK; }
  if (key == 28 && value >= 0 && value <= 64) { g_det_rmax = value; return OF_OK; }
  if (key == 29 && value >= 0 && value <= 4) { g_wgr_lanes = value; return OF_OK; }
  if (key == 30 && value >= 0 && value <= 2) { g_gx3_ring = value; return OF_OK; }
  if (key == 31 && value >= -1 && value <= 8) { g_stem_persist = value; return OF_OK; }
  if (key == 32 && (value == 0 || value == 1)) { g_bnp_b16 = value; return OF_OK; }
  if (key == 33 && value >= 1 && value <= 256) { g_wgx3_min_tiles = value; return OF_OK; }
  if (key == 34 && value >= 0 && value <= 2) { g_det_tile = value; return OF_OK; }
  if (key == 35 && (value == 0 || value == 1)) { g_det_tpre = value; return OF_OK; }
  if (key == 36 && value >= 0 && value <= 3) { g_x3_bn64 = value; return OF_OK; }
  if (key == 37 && value >= 0 && value <= 16) { g_det_fx_grid = value; return OF_OK; }
  if (key == 38 && value >= 0 && value <= 131072) { g_det_lds_probe = value; return OF_OK; }
  if (key == 39 && (value == 0 || value == 1)) { g_abl_noact = value; return OF_OK; }
  return fail(OF_EINVAL, "of_set_tuning: unknown key/value " + std::to_string(key));
}

size_t of_conv_pack_table_bytes(int nconv) {
  return sizeof(PackTableHeader) + (size_t)std::max(nconv, 0) * sizeof(PackEntry);
}

int of_conv_pack_table_ex(int nconv, const of_conv_desc* descs, const float* const* w_hwio,
                          void* const* w_fwd, void* const* w_bwd, const int* bf16,
                          void* host_table) {
  OF_CHECK_ARG(nconv > 0 && descs && w_hwio && w_fwd && w_bwd && host_table, "pack table: args");
  PackTableHeader* h = static_cast<PackTableHeader*>(host_table);
  PackEntry* e = reinterpret_cast<PackEntry*>(static_cast<char*>(host_table) +
                                              sizeof(PackTableHeader));
  int64_t work = 0, tiles = 0;
  for (int i = 0; i < nconv; ++i) {
    int st = validate(&descs[i]);
    if (st) return st;
    OF_CHECK_ARG(w_hwio[i] && w_fwd[i] && w_bwd[i], "pack table: NULL weight pointer");
    const int b16 = bf16 ? (bf16[i] == 2 ? 2 : bf16[i] != 0) : 0;   // 2: x3 planes
    e[i] = pack_entry(&descs[i], w_hwio[i], w_fwd[i], w_bwd[i], b16);
    e[i].work_begin = work;
    e[i].tile_begin = (int)tiles;
    OF_CHECK_ARG(pack_work(&descs[i], b16) < INT32_MAX, "pack table: layer too large");
    work += pack_work_many(&descs[i], b16);
    tiles += pack_tiles16(&descs[i], b16);
    OF_CHECK_ARG(tiles < INT32_MAX, "pack table: too many tiles");
  }
  h->nconv = nconv;
  h->ntiles16 = (int)tiles;
  h->total = work;
  return OF_OK;
}

int of_conv_pack_table(int nconv, const of_conv_desc* descs, const float* const* w_hwio,
                       float* const* w_fwd, float* const* w_bwd, void* host_table) {
  return of_conv_pack_table_ex(nconv, descs, w_hwio, reinterpret_cast<void* const*>(w_fwd),
                               reinterpret_cast<void* const*>(w_bwd), nullptr, host_table);
}

int of_conv_pack_many(const void* dev_table, int64_t total_work, void* stream) {
  OF_CHECK_ARG(dev_table && total_work > 0, "pack many: args");
  const int64_t blocks = cdiv(total_work, 256 * PACK_PT);
  OF_CHECK_ARG(blocks < INT32_MAX / 2, "pack many: too much work");
  // as many tile workgroups again (a bf16 entry's forward image is about the size of its
  // input-gradient image; they walk the header's tile count grid-stride, so any number serves)
  hipLaunchKernelGGL(pack_many_kernel, dim3((unsigned)(2 * blocks)), dim3(256), 0,
                     as_stream(stream), static_cast<const char*>(dev_table), (int)blocks);
  return check_launch("pack_many");
}

// Timing kind of the narrow (VALU) path; GEMM kinds are MODE * 8 + tile config (0..3).
constexpr int KIND_NARROW = 7;
constexpr int KIND_STEM_X3 = 184;   // conv_stem_x3 (bench.py kind_name)
constexpr int KIND_STEM_B16 = 186;  // conv_stem_x3<32, 1> (bf16); 187: conv_wgrad_stem_x3<1>

double conv_flops(const of_conv_desc* d) {
  return 2.0 * d->n * d->ho * d->wo * (double)d->cout * d->kh * d->kw * d->cin;
}

size_t of_conv2d_fwd_workspace(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return 0;
  return fd_workspace(fwd_args(d, geo(d)));
}

size_t of_conv2d_dgrad_workspace(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return 0;
  return fd_workspace(dgrad_args(d, geo(d)));
}

size_t of_conv2d_fwd_bf16_workspace(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return 0;
  if (tile_ok(d))
    return fd_workspace(tile_args(d, geo(d), MODE_FWD, false, g_tile_b16 == 1, ws_ok(d, MODE_FWD)));
  GemmArgs a = fwd_args(d, geo(d), true);
  if (g_gemm_b16 & 1) gemm_x3_plan(a);
  return std::max(fd_workspace(a), fd_workspace(fwd_args(d, geo(d), true)));
}

size_t of_conv2d_dgrad_bf16_workspace(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return 0;
  if (tile_ok(d))
    return fd_workspace(tile_args(d, geo(d), MODE_DGRAD, false, g_tile_b16 == 1,
                                  ws_ok(d, MODE_DGRAD)));
  GemmArgs a = dgrad_args(d, geo(d), true);
  if (g_gemm_b16 & 2) gemm_x3_plan(a);
  return std::max(fd_workspace(a), fd_workspace(dgrad_args(d, geo(d), true)));
}

int of_conv_path(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return -1;
  return narrow_ok(d) ? 1 : 0;
}

// prec: 0 fp32 MFMA, 1 bf16, 2 fp32 on the split-bf16 tile kernel (3x3 stride 1 only).
static int conv_fwd_impl(int prec, const of_conv_desc* d, const float* x, int ldx,
                         const void* w_fwd, const float* bias, const float* bn_gamma,
                         const float* bn_beta, const float* bn_mean, const float* bn_var,
                         float bn_eps, const float* residual, int ldr, int act, float alpha,
                         float* z, int ldz, float* y, int ldy, void* workspace, size_t ws_bytes,
                         void* stream, float* pool = nullptr) {
  int st = validate(d);
  if (st) return st;
  const bool bf16 = prec == 1, x3 = prec == 2;
  OF_CHECK_ARG(!x3 || !narrow_ok(d), "conv fwd x3: the Cout <= 4 layers take the fp32 kernels");
  OF_CHECK_ARG(x && w_fwd && y, "conv fwd: NULL pointer");
  OF_CHECK_ARG(ldx >= d->cin_p && ldx % 4 == 0, "conv fwd: ldx");
  OF_CHECK_ARG(ldy >= d->cout, "conv fwd: ldy");
  OF_CHECK_ARG(!bn_gamma || (bn_beta && bn_mean && bn_var), "conv fwd: incomplete BN params");
  OF_CHECK_ARG(!residual || ldr >= d->cout, "conv fwd: ldr");
  OF_CHECK_ARG(!z || ldz >= d->cout, "conv fwd: ldz");
  OF_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)w_fwd & 15) == 0,
               "conv fwd: x / w must be 16-byte aligned");
  if (!prec && narrow_ok(d) && !bn_gamma && !residual && !z) {   // 2-channel layers: VALU
    hipStream_t s = as_stream(stream);
    if (timing_on()) timing_begin(s);
    st = narrow_fwd(d, x, ldx, static_cast<const float*>(w_fwd), bias, act, alpha, y, ldy, s);
    if (timing_on()) timing_end(s, MODE_FWD * 8 + KIND_NARROW, conv_flops(d));
    return st;
  }
  Geo g = geo(d);
  const bool tile = (bf16 || x3) && tile_ok(d);
  const bool ws = tile && bf16 && ws_ok(d, MODE_FWD);
  const bool b16 = tile && bf16 && g_tile_b16 == 1;
  GemmArgs a = tile ? tile_args(d, g, MODE_FWD, x3, b16, ws) : fwd_args(d, g, bf16 || x3);
  bool stem = (x3 || (bf16 && g_stem_bf16)) && !tile && g_stem_x3 && stem_x3_ok(d);
  if (stem) {                            // conv_stem_x3: one workgroup per output tile, no split
    a.splits = 1;
    a.k_per_split = a.K;
    a.slab = nullptr;
  }
  a.C = y;   // (vec_ep_ok reads the output fields)
  a.ldc = ldy;
  a.res = residual;
  a.ldr = ldr;
  a.z = z;
  a.ldz = ldz;
  stem = stem && vec_ep_ok(a);
  const bool g16 = bf16 && !tile && !stem && (g_gemm_b16 & 1);   // conv_gemm_x3<..., 1>
  if ((x3 || g16) && !tile && !stem) gemm_x3_plan(a);
  if (!stem) attach_slab(a, workspace, ws_bytes, tile ? 1 : (bf16 || x3) ? BKH : BK);
  a.A = x;
  a.lda = ldx;
  a.a_bytes = (int64_t)d->n * d->h * d->w * ldx * 4;
  a.B = static_cast<const float*>(w_fwd);
  a.b_plane = (int64_t)g.cout_p * g.kf16;
  a.b_bytes = x3 ? 3 * a.b_plane * 2 : bf16 ? a.b_plane * 2 : (int64_t)g.kf * g.nf * 4;
  OF_CHECK_ARG(a.a_bytes < INT32_MAX && a.b_bytes < INT32_MAX,
               "conv fwd: tensors must be < 2 GiB (32-bit buffer offsets)");
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
  const double flops = 2.0 * d->n * d->ho * d->wo * (double)d->cout * g.taps * d->cin;
  a.vec_ep = vec_ep_ok(a);
  // split 3x3 forward, one K slice, fp32 output only: the direct epilogue (conv_dev.h)
  a.direct16 = x3 && tile && (g_x3_direct & 1) && a.splits == 1 && a.vec_ep && !residual && !z &&
               d->cout % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)y & 15) == 0;
  if (pool) {
    if (!stem || d->ho % 2 || d->wo % 2 || d->cout % 4)
      return fail(OF_EUNSUPPORTED, "conv fwd pool: only the stem kernel with an even output");
    OF_CHECK_ARG(((uintptr_t)pool & 15) == 0, "conv fwd pool: 16-byte alignment");
    a.pool_out = pool;
  }
  if (stem) {
    const int64_t tiles = (int64_t)d->n * cdiv(d->ho, ST_TH) * cdiv(d->wo, ST_TW);
    OF_CHECK_ARG(tiles < INT32_MAX, "conv stem: too many tiles");
    if (timing_on()) timing_begin(s);
    // persistent (of_set_tuning key 31 = workgroups per CU, default as many as the LDS holds:
    // 2 fp32 / 3 bf16 / 1 for the 64-channel form; 0: one tile per workgroup, the round-2..4
    // grid): B staged once per workgroup, the next tile's halo loaded during this tile's MFMAs
    const int groups = bf16 || g_stem_x3 != 2 ? 2 : 1;
    const int per_cu = g_stem_persist < 0 ? (bf16 ? 3 : g_stem_x3 == 2 ? 1 : 2) : g_stem_persist;
    const int64_t cap = per_cu > 0 ? (int64_t)per_cu * device_cus() : tiles * groups;
    const unsigned grid = (unsigned)(std::min(tiles * groups, cap) / groups * groups);
    if (bf16)
      hipLaunchKernelGGL((conv_stem_x3<32, 1>), dim3(grid), dim3(256), 0, s, a, (int)tiles);
    else if (g_stem_x3 == 2)
      hipLaunchKernelGGL(conv_stem_x3<64>, dim3(grid), dim3(512), 0, s, a, (int)tiles);
    else
      hipLaunchKernelGGL(conv_stem_x3<32>, dim3(grid), dim3(256), 0, s, a, (int)tiles);
    if (timing_on()) timing_end(s, bf16 ? KIND_STEM_B16 : KIND_STEM_X3, flops);
    return check_launch("conv_stem_x3");
  }
  st = x3     ? (tile ? launch_tile_x3<MODE_FWD>(a, s, flops) : launch_gemm_x3<MODE_FWD>(a, s, flops))
       : ws   ? launch_tile_ws<MODE_FWD>(a, s, flops)
       : b16  ? launch_tile_b16<MODE_FWD>(a, s, flops)
       : tile ? launch_tile_bf16<MODE_FWD>(a, s, flops)
       : g16  ? launch_gemm_x3<MODE_FWD, 1>(a, s, flops)
       : bf16 ? launch_gemm_bf16<MODE_FWD>(a, s, flops)
              : launch_gemm<MODE_FWD>(a, s, flops);
  return st;
}

int of_conv2d_fwd(const of_conv_desc* d, const float* x, int ldx, const float* w_fwd,
                  const float* bias, const float* bn_gamma, const float* bn_beta,
                  const float* bn_mean, const float* bn_var, float bn_eps,
                  const float* residual, int ldr, int act, float alpha, float* z, int ldz,
                  float* y, int ldy, void* workspace, size_t ws_bytes, void* stream) {
  return conv_fwd_impl(0, d, x, ldx, w_fwd, bias, bn_gamma, bn_beta, bn_mean, bn_var,
                       bn_eps, residual, ldr, act, alpha, z, ldz, y, ldy, workspace, ws_bytes,
                       stream);
}

int of_conv2d_fwd_pool(const of_conv_desc* d, int precision, const float* x, int ldx,
                       const void* w_fwd, const float* bias, const float* bn_gamma,
                       const float* bn_beta, const float* bn_mean, const float* bn_var,
                       float bn_eps, int act, float alpha, float* z, int ldz, float* y, int ldy,
                       float* pool, void* workspace, size_t ws_bytes, void* stream) {
  OF_CHECK_ARG(pool && (precision == 1 || precision == 2), "conv fwd pool: args");
  return conv_fwd_impl(precision, d, x, ldx, w_fwd, bias, bn_gamma, bn_beta, bn_mean, bn_var,
                       bn_eps, nullptr, 0, act, alpha, z, ldz, y, ldy, workspace, ws_bytes,
                       stream, pool);
}

int of_conv2d_fwd_bf16(const of_conv_desc* d, const float* x, int ldx, const void* w16_fwd,
                       const float* bias, const float* bn_gamma, const float* bn_beta,
                       const float* bn_mean, const float* bn_var, float bn_eps,
                       const float* residual, int ldr, int act, float alpha, float* z, int ldz,
                       float* y, int ldy, void* workspace, size_t ws_bytes, void* stream) {
  return conv_fwd_impl(1, d, x, ldx, w16_fwd, bias, bn_gamma, bn_beta, bn_mean, bn_var,
                       bn_eps, residual, ldr, act, alpha, z, ldz, y, ldy, workspace, ws_bytes,
                       stream);
}

// fused BN partial sums of an input gradient (of_conv2d_dgrad_add_act_bnp)
struct BnpArgs {
  const float* gamma; const float* beta; const float* res; int ld_res;
  float* part; size_t part_bytes; int* nblk;
};

static int conv_dgrad_impl(int prec, const of_conv_desc* d, const float* dy, int lddy,
                           const void* w_bwd, const float* act_src, int ld_act, int act,
                           float alpha, const float* add, int ld_add, float* dx, int lddx,
                           void* workspace, size_t ws_bytes, void* stream, int act_post = 0,
                           const BnpArgs* bnp = nullptr) {
  int st = validate(d);
  if (st) return st;
  Geo g = geo(d);
  const bool bf16 = prec == 1, x3 = prec == 2;
  OF_CHECK_ARG(!x3 || !narrow_ok(d), "conv dgrad x3: the Cout <= 4 layers take the fp32 kernels");
  OF_CHECK_ARG(dy && w_bwd && dx, "conv dgrad: NULL pointer");
  OF_CHECK_ARG(lddy >= g.cout_p && lddy % 4 == 0, "conv dgrad: lddy (>= round_up(cout,4))");
  OF_CHECK_ARG(lddx >= d->cin_p, "conv dgrad: lddx");
  OF_CHECK_ARG(!act_src || ld_act >= d->cin_p, "conv dgrad: ld_act");
  OF_CHECK_ARG(!add || ld_add >= d->cin_p, "conv dgrad: ld_add");
  OF_CHECK_ARG(((uintptr_t)dy & 15) == 0 && ((uintptr_t)w_bwd & 15) == 0,
               "conv dgrad: dy / w must be 16-byte aligned");
  OF_CHECK_ARG(d->stride == 1 || d->stride == 2, "conv dgrad: stride must be 1 or 2");
  if (!prec && narrow_ok(d)) {
    OF_CHECK_ARG(!add && !act_post, "conv dgrad: the Cout <= 4 kernels take no added gradient");
    hipStream_t s = as_stream(stream);
    if (timing_on()) timing_begin(s);
    st = narrow_dgrad(d, dy, lddy, static_cast<const float*>(w_bwd), act_src, ld_act, act,
                      alpha, dx, lddx, s);
    if (timing_on()) timing_end(s, MODE_DGRAD * 8 + KIND_NARROW, conv_flops(d));
    return st;
  }
  const bool tile = (bf16 || x3) && tile_ok(d);
  const bool in_place = add && add == dx && ld_add == lddx;
  const bool ws = tile && bf16 && ws_ok(d, MODE_DGRAD);
  // (bf16 with BN partial sums and key 32: conv_tile_b16, the split body with one plane)
  const bool b16 = tile && bf16 && !ws && (g_tile_b16 == 1 || (bnp && g_bnp_b16));
  GemmArgs a = tile ? tile_args(d, g, MODE_DGRAD, x3, b16, ws)
                    : dgrad_args(d, g, bf16 || x3, in_place);
  const bool g16 = bf16 && !tile && (g_gemm_b16 & 2);       // conv_gemm_x3<..., 1>
  if ((x3 || g16) && !tile) gemm_x3_plan(a);
  if (a.tiles_total == 0)                                // every output already final
    return bnp ? fail(OF_EUNSUPPORTED, "conv dgrad bnp: no GEMM tiles") : OF_OK;
  attach_slab(a, workspace, ws_bytes, tile ? 1 : (bf16 || x3) ? BKH : BK);
  a.A = dy;
  a.lda = lddy;
  a.a_bytes = (int64_t)d->n * d->ho * d->wo * lddy * 4;
  a.B = static_cast<const float*>(w_bwd);
  a.b_plane = g.kd16 * g.nd;
  a.b_bytes = x3 ? 3 * a.b_plane * 2 : bf16 ? a.b_plane * 2 : g.kd * g.nd * 4;
  OF_CHECK_ARG(a.a_bytes < INT32_MAX && a.b_bytes < INT32_MAX,
               "conv dgrad: tensors must be < 2 GiB (32-bit buffer offsets)");
  a.C = dx;
  a.ldc = lddx;
  a.act_src = act_src;
  a.ld_act = ld_act;
  a.act = act;
  a.alpha = alpha;
  a.res = add;
  a.ldr = ld_add;
  a.act_post = act_post;
  hipStream_t s = as_stream(stream);
  const double flops = 2.0 * d->n * d->ho * d->wo * (double)d->cout * g.taps * d->cin;
  a.vec_ep = vec_ep_ok(a);
  if (g_abl_noact && x3 && tile && !bnp) a.act_src = nullptr;   // key 39: timing ablation
  // split 3x3 input gradient, one K slice: the direct epilogue (conv_dev.h direct_dgrad_f32)
  a.direct16 = x3 && tile && (g_x3_direct & 2) && a.splits == 1 && a.vec_ep;
  if (bnp) {
    // the BN partial sums ride on conv_tile_x3's vectorised one-slice epilogue only; any other
    // form: OF_EUNSUPPORTED before anything is launched (the caller runs the separate pass)
    const int64_t m_tiles = a.n_tiles > 0 ? a.tiles_total / a.n_tiles : 0;
    // (conv_tile_x3 / conv_tile_b16 with X3_EPB 1, conv_tile_bf16 or the split conv_gemm_x3
    // with EPC_BATCH; the GEMM's phase groups must produce every input-gradient pixel.  The
    // bf16 GEMM form measured 1780 -> 1726 pairs/s on the bf16 B = 32 step: declined)
    int64_t rows = 0;
    for (int gq = 0; gq < a.ngroups; ++gq) rows += a.grp[gq].M;
    const bool form = tile ? (x3 || b16 ? X3_EPB == 1 : bf16 && !ws && EPC_BATCH)
                           : x3 && EPC_BATCH && rows == (int64_t)d->n * d->h * d->w;
    if (!(form && a.splits == 1 && a.vec_ep && act_src) ||
        a.N % 4 || ((uintptr_t)bnp->gamma & 15) || ((uintptr_t)bnp->beta & 15) ||
        ((uintptr_t)bnp->part & 15) || (bnp->res && (((uintptr_t)bnp->res & 15) || bnp->ld_res % 4)))
      return fail(OF_EUNSUPPORTED, "conv dgrad bnp: not the one-slice split-tile input gradient");
    OF_CHECK_ARG(bnp->gamma && bnp->beta && bnp->part && bnp->nblk, "conv dgrad bnp: args");
    OF_CHECK_ARG(bnp->part_bytes >= (size_t)m_tiles * 2 * a.N * 4, "conv dgrad bnp: part too small");
    a.direct16 = 0;
    a.bnp = bnp->part;
    a.bnp_res = bnp->res;
    a.ld_bnp_res = bnp->ld_res;
    a.bnp_g = bnp->gamma;
    a.bnp_b = bnp->beta;
    *bnp->nblk = (int)m_tiles;
  }
  st = x3     ? (tile ? launch_tile_x3<MODE_DGRAD>(a, s, flops)
                     : launch_gemm_x3<MODE_DGRAD>(a, s, flops))
       : ws   ? launch_tile_ws<MODE_DGRAD>(a, s, flops)
       : b16  ? launch_tile_b16<MODE_DGRAD>(a, s, flops)
       : tile ? launch_tile_bf16<MODE_DGRAD>(a, s, flops)
       : g16  ? launch_gemm_x3<MODE_DGRAD, 1>(a, s, flops)
       : bf16 ? launch_gemm_bf16<MODE_DGRAD>(a, s, flops)
              : launch_gemm<MODE_DGRAD>(a, s, flops);
  return st;
}

int of_conv2d_dgrad(const of_conv_desc* d, const float* dy, int lddy, const float* w_bwd,
                    const float* act_src, int ld_act, int act, float alpha, float* dx,
                    int lddx, void* workspace, size_t ws_bytes, void* stream) {
  return conv_dgrad_impl(0, d, dy, lddy, w_bwd, act_src, ld_act, act, alpha, nullptr, 0,
                         dx, lddx, workspace, ws_bytes, stream);
}

int of_conv2d_dgrad_add(const of_conv_desc* d, const float* dy, int lddy, const float* w_bwd,
                        const float* add, int ld_add, float* dx, int lddx, void* workspace,
                        size_t ws_bytes, void* stream) {
  return conv_dgrad_impl(0, d, dy, lddy, w_bwd, nullptr, 0, OF_ACT_NONE, 0.f, add, ld_add,
                         dx, lddx, workspace, ws_bytes, stream);
}

int of_conv2d_dgrad_bf16(const of_conv_desc* d, const float* dy, int lddy, const void* w16_bwd,
                         const float* act_src, int ld_act, int act, float alpha, float* dx,
                         int lddx, void* workspace, size_t ws_bytes, void* stream) {
  return conv_dgrad_impl(1, d, dy, lddy, w16_bwd, act_src, ld_act, act, alpha, nullptr, 0,
                         dx, lddx, workspace, ws_bytes, stream);
}

int of_conv2d_dgrad_add_bf16(const of_conv_desc* d, const float* dy, int lddy,
                             const void* w16_bwd, const float* add, int ld_add, float* dx,
                             int lddx, void* workspace, size_t ws_bytes, void* stream) {
  return conv_dgrad_impl(1, d, dy, lddy, w16_bwd, nullptr, 0, OF_ACT_NONE, 0.f, add, ld_add,
                         dx, lddx, workspace, ws_bytes, stream);
}

int of_conv_pack_weights_x3(const of_conv_desc* d, const float* w_hwio, void* w3_fwd,
                            void* w3_bwd, void* stream) {
  int st = validate(d);
  if (st) return st;
  OF_CHECK_ARG(w_hwio && w3_fwd && w3_bwd, "pack x3: NULL pointer");
  const int64_t total = pack_work(d, 1);
  OF_CHECK_ARG(total < INT32_MAX, "pack: layer too large");
  const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 4096);
  hipLaunchKernelGGL(pack_one_kernel, dim3(blocks), dim3(256), 0, as_stream(stream),
                     pack_entry(d, w_hwio, w3_fwd, w3_bwd, 2), total);
  return check_launch("pack_x3");
}

size_t of_conv2d_fwd_x3_workspace(const of_conv_desc* d) {
  if (validate(d) != OF_OK || narrow_ok(d)) return 0;
  if (tile_ok(d)) return fd_workspace(tile_args(d, geo(d), MODE_FWD, true));
  GemmArgs a = fwd_args(d, geo(d), true);
  gemm_x3_plan(a);
  return fd_workspace(a);
}

size_t of_conv2d_dgrad_x3_workspace(const of_conv_desc* d) {
  if (validate(d) != OF_OK || narrow_ok(d)) return 0;
  if (tile_ok(d)) return fd_workspace(tile_args(d, geo(d), MODE_DGRAD, true));
  GemmArgs a = dgrad_args(d, geo(d), true);
  gemm_x3_plan(a);
  return fd_workspace(a);
}

int of_conv2d_fwd_x3(const of_conv_desc* d, const float* x, int ldx, const void* w3_fwd,
                     const float* bias, const float* bn_gamma, const float* bn_beta,
                     const float* bn_mean, const float* bn_var, float bn_eps,
                     const float* residual, int ldr, int act, float alpha, float* z, int ldz,
                     float* y, int ldy, void* workspace, size_t ws_bytes, void* stream) {
  return conv_fwd_impl(2, d, x, ldx, w3_fwd, bias, bn_gamma, bn_beta, bn_mean, bn_var,
                       bn_eps, residual, ldr, act, alpha, z, ldz, y, ldy, workspace, ws_bytes,
                       stream);
}

int of_conv2d_dgrad_x3(const of_conv_desc* d, const float* dy, int lddy, const void* w3_bwd,
                       const float* act_src, int ld_act, int act, float alpha, float* dx,
                       int lddx, void* workspace, size_t ws_bytes, void* stream) {
  return conv_dgrad_impl(2, d, dy, lddy, w3_bwd, act_src, ld_act, act, alpha, nullptr, 0,
                         dx, lddx, workspace, ws_bytes, stream);
}

int of_conv2d_dgrad_add_x3(const of_conv_desc* d, const float* dy, int lddy,
                           const void* w3_bwd, const float* add, int ld_add, float* dx,
                           int lddx, void* workspace, size_t ws_bytes, void* stream) {
  return conv_dgrad_impl(2, d, dy, lddy, w3_bwd, nullptr, 0, OF_ACT_NONE, 0.f, add, ld_add,
                         dx, lddx, workspace, ws_bytes, stream);
}

size_t of_conv2d_wgrad_workspace(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return 0;
  if (narrow_ok(d)) return narrow_wgrad_ws(d);
  WgradPlan p = wgrad_plan(d);
  return (size_t)p.splits * p.split_stride * sizeof(float);
}

size_t of_conv2d_wgrad_bf16_workspace(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return 0;
  if (narrow_ok(d)) return narrow_wgrad_ws(d);
  WgradPlan p = wgrad_plan(d, true);
  return (size_t)p.splits * p.split_stride * sizeof(float);
}

size_t of_conv2d_wgrad_x3_workspace(const of_conv_desc* d) {
  if (validate(d) != OF_OK) return 0;
  if (narrow_ok(d)) return narrow_wgrad_ws(d);
  WgradPlan p = wgrad_plan(d, false, wgx3_ok(d) || g_wgx3_gemm);
  return (size_t)p.splits * p.split_stride * sizeof(float);
}

// prec: 0 fp32 MFMA, 1 bf16, 2 fp32 with conv_wgrad_tile_x3 where wgx3_ok (else as 0).
static int conv_wgrad_impl(int prec, const of_conv_desc* d, const float* x, int ldx,
                           const float* dy, int lddy, float* dw, float* db, int accumulate,
                           void* workspace, size_t ws_bytes, void* stream,
                           const float* bn_g = nullptr, const float* bn_v = nullptr,
                           float bn_eps = 0.f) {
  int st = validate(d);
  if (st) return st;
  Geo g = geo(d);
  const bool bf16 = prec == 1, x3 = prec == 2 && wgx3_ok(d);
  const bool b16 = bf16 && g_wgrad_b16 && wgx3_ok(d);   // conv_wgrad_tile_b16
  const bool x3g = prec == 2 && !x3 && g_wgx3_gemm;   // conv_wgrad_x3 (other shapes)
  const bool g16 = bf16 && gemm_b16_wg(d);             // conv_wgrad_x3<..., 1>
  OF_CHECK_ARG(x && dy && dw && workspace, "conv wgrad: NULL pointer");
  OF_CHECK_ARG(ldx >= d->cin_p && ldx % 4 == 0, "conv wgrad: ldx");
  OF_CHECK_ARG(lddy >= g.cout_p && lddy % 4 == 0, "conv wgrad: lddy");
  if (narrow_ok(d)) {
    OF_CHECK_ARG(!bn_g, "conv wgrad: the Cout <= 4 kernels take no BN scale");
    OF_CHECK_ARG(ws_bytes >= narrow_wgrad_ws(d), "conv wgrad: workspace too small");
    hipStream_t s = as_stream(stream);
    if (timing_on()) timing_begin(s);
    st = narrow_wgrad(d, x, ldx, dy, lddy, dw, db, accumulate, workspace, s);
    if (timing_on()) timing_end(s, MODE_WGRAD * 8 + KIND_NARROW, conv_flops(d));
    return st;
  }
  WgradPlan p = wgrad_plan(d, bf16, x3 || x3g);
  OF_CHECK_ARG(ws_bytes >= (size_t)p.splits * p.split_stride * sizeof(float),
               "conv wgrad: workspace too small");
  GemmArgs a = base_args(d);
  a.kc = g.cin_p;
  a.N = d->cout;
  a.K = d->n * d->ho * d->wo;
  single_group(a, d, p.M, a.K);
  a.M = p.M;
  a.A = x;
  a.lda = ldx;
  a.a_bytes = (int64_t)d->n * d->h * d->w * ldx * 4;
  a.B = dy;
  a.ldb = lddy;
  a.b_bytes = (int64_t)a.K * lddy * 4;
  OF_CHECK_ARG(a.a_bytes < INT32_MAX && a.b_bytes < INT32_MAX,
               "conv wgrad: tensors must be < 2 GiB (32-bit buffer offsets)");
  a.nb = g.cout_p;
  a.slab = static_cast<float*>(workspace);
  a.slab_ld = p.ldc;
  a.splits = p.splits;
  a.k_per_split = p.k_per_split;
  a.split_stride = p.split_stride;
  a.colsum = db != nullptr;
  a.vec_ep = vec_ep_ok(a);
  hipStream_t s = as_stream(stream);
  const double flops = 2.0 * a.K * (double)d->cout * g.taps * d->cin;
  if (stem_wg_ok(d) && (!bf16 || g_stem_bf16)) {
    a.K = stem_wg_tiles(d);
    a.lda = ldx;
    if (timing_on()) timing_begin(s);
    if (bf16) hipLaunchKernelGGL(conv_wgrad_stem_x3<1>, dim3(a.splits), dim3(SW_NT), 0, s, a);
    else hipLaunchKernelGGL(conv_wgrad_stem_x3<3>, dim3(a.splits), dim3(SW_NT), 0, s, a);
    if (timing_on()) timing_end(s, bf16 ? 187 : 185, flops);     // bench.py KIND_STEM_*
    st = check_launch("conv_wgrad_stem_x3");
  } else if (b16) {
    // the x3b configurations, all 9-tap: timing kinds 216 + cfg (bench.py X3_WGT 4 + cfg)
    const int cfg = wgx3_cfg(d);
    a.K = d->n * (int)cdiv(d->ho, wgx3_rows(cfg)) * (int)cdiv(d->wo, TT_W);
    int cib, cob;
    wgx3_blocks(d, cib, cob);
    a.n_tiles = (int)cdiv(d->cout, cob);
    a.tiles_total = (int)cdiv(g.cin_p, cib) * a.n_tiles;
    dim3 grid(a.tiles_total * a.splits);
    if (timing_on()) timing_begin(s);
    if (cfg == 4) hipLaunchKernelGGL((conv_wgrad_tile_b16<2, 2, 8>), grid, dim3(256), 0, s, a);
    else if (cfg == 0) hipLaunchKernelGGL((conv_wgrad_tile_b16<2, 4, 8>), grid, dim3(512), 0, s, a);
    else if (cfg == 1) hipLaunchKernelGGL((conv_wgrad_tile_b16<2, 3, 8>), grid, dim3(384), 0, s, a);
    else if (cfg == 2) hipLaunchKernelGGL((conv_wgrad_tile_b16<4, 2, 4>), grid, dim3(512), 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_tile_b16<4, 1, 4>), grid, dim3(256), 0, s, a);
    if (timing_on()) timing_end(s, 216 + cfg, flops);
    st = check_launch("conv_wgrad_tile_b16");
  } else if (x3) {
    a.K = d->n * (int)cdiv(d->ho, wgx3_rows(wgx3_cfg(d))) * (int)cdiv(d->wo, TT_W);
    int cib, cob;
    wgx3_blocks(d, cib, cob);
    const int cfg = wgx3_cfg(d);
    a.n_tiles = (int)cdiv(d->cout, cob);
    a.tiles_total = (int)cdiv(g.cin_p, cib) * a.n_tiles;
    dim3 grid(a.tiles_total * a.splits);
    if (timing_on()) timing_begin(s);
    const bool x3b = g_wgx3b == 2 || (g_wgx3b == 1 && cfg == 0) || cfg == 4;
    if (x3b) {
      if (g_wgx3b_mi == 2) {   // waves of 32 ci x 16 co
        if (cfg == 4) hipLaunchKernelGGL((conv_wgrad_tile_x3b<1, 4, 8, 2>), grid, dim3(256), 0, s, a);
        else if (cfg == 0) hipLaunchKernelGGL((conv_wgrad_tile_x3b<1, 8, 8, 2>), grid, dim3(512), 0, s, a);
        else if (cfg == 1) hipLaunchKernelGGL((conv_wgrad_tile_x3b<1, 6, 8, 2>), grid, dim3(384), 0, s, a);
        else if (cfg == 2) hipLaunchKernelGGL((conv_wgrad_tile_x3b<2, 4, 4, 2>), grid, dim3(512), 0, s, a);
        else hipLaunchKernelGGL((conv_wgrad_tile_x3b<2, 2, 4, 2>), grid, dim3(256), 0, s, a);
      } else if (cfg == 4) hipLaunchKernelGGL((conv_wgrad_tile_x3b<2, 2, 8>), grid, dim3(256), 0, s, a);
      else if (cfg == 0) hipLaunchKernelGGL((conv_wgrad_tile_x3b<2, 4, 8>), grid, dim3(512), 0, s, a);
      else if (cfg == 1) hipLaunchKernelGGL((conv_wgrad_tile_x3b<2, 3, 8>), grid, dim3(384), 0, s, a);
      else if (cfg == 2) hipLaunchKernelGGL((conv_wgrad_tile_x3b<4, 2, 4>), grid, dim3(512), 0, s, a);
      else hipLaunchKernelGGL((conv_wgrad_tile_x3b<4, 1, 4>), grid, dim3(256), 0, s, a);
    } else if (cfg == 0) hipLaunchKernelGGL((conv_wgrad_tile_x3<1, 4, 3, 8>), grid, dim3(768), 0, s, a);
    else if (cfg == 1) hipLaunchKernelGGL((conv_wgrad_tile_x3<1, 3, 3, 8>), grid, dim3(576), 0, s, a);
    else if (cfg == 2) hipLaunchKernelGGL((conv_wgrad_tile_x3<2, 2, 3, 4>), grid, dim3(768), 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_tile_x3<2, 1, 3, 4>), grid, dim3(384), 0, s, a);
    // timing kinds 144-147: the 3-tap form, 148-151: conv_wgrad_tile_x3b, 152: its cfg 4
    // (bench.py X3_WGT)
    if (timing_on()) timing_end(s, cfg == 4 ? 152 : 128 + MODE_WGRAD * 8 + cfg + (x3b ? 4 : 0), flops);
    st = check_launch("conv_wgrad_tile_x3");
  } else if (x3g) {
    const int bn = d->cout > 64 ? 128 : 64;
    a.n_tiles = (int)cdiv(d->cout, bn);
    a.tiles_total = (int)cdiv(a.M, 128) * a.n_tiles;
    dim3 grid(a.tiles_total * a.splits), block(512);
    if (timing_on()) timing_begin(s);
    if (bn == 128) hipLaunchKernelGGL((conv_wgrad_x3<128, 128, 4, 2>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_x3<128, 64, 4, 2>), grid, block, 0, s, a);
    if (timing_on()) timing_end(s, 160 + MODE_WGRAD * 8 + (bn == 128 ? 0 : 1), flops);
    st = check_launch("conv_wgrad_x3");
  } else if (g16) {
    const int bn = d->cout > 64 ? 128 : 64;
    a.n_tiles = (int)cdiv(d->cout, bn);
    a.tiles_total = (int)cdiv(a.M, 128) * a.n_tiles;
    dim3 grid(a.tiles_total * a.splits), block(512);
    if (timing_on()) timing_begin(s);
    if (bn == 128) hipLaunchKernelGGL((conv_wgrad_x3<128, 128, 4, 2, 1>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_x3<128, 64, 4, 2, 1>), grid, block, 0, s, a);
    if (timing_on()) timing_end(s, 240 + MODE_WGRAD * 8 + (bn == 128 ? 0 : 1), flops);
    st = check_launch("conv_wgrad_x3_b16");
  } else if (wgt_ok(d, bf16)) {
    int cib, cob;
    wgt_blocks(d, cib, cob);
    a.K = d->n * (int)cdiv(d->ho, TT_H) * (int)cdiv(d->wo, TT_W);
    a.n_tiles = (int)cdiv(d->cout, cob);
    a.tiles_total = (int)cdiv(g.cin_p, cib) * a.n_tiles;
    const int cfg = wgt_cfg(d);
    dim3 grid(a.tiles_total * a.splits), block(256);
    if (timing_on()) timing_begin(s);
    if (bf16 && !g_wgt_pf) {
      if (cfg == 0) hipLaunchKernelGGL((conv_wgrad_tile_bf16<1, 4, 0>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((conv_wgrad_tile_bf16<2, 2, 0>), grid, block, 0, s, a);
    } else if (bf16) {
      if (cfg == 0) hipLaunchKernelGGL((conv_wgrad_tile_bf16<1, 4>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((conv_wgrad_tile_bf16<2, 2>), grid, block, 0, s, a);
    } else {
      if (cfg == 0) hipLaunchKernelGGL((conv_wgrad_tile_f32<1, 4>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((conv_wgrad_tile_f32<2, 2>), grid, block, 0, s, a);
    }
    if (timing_on()) timing_end(s, (bf16 ? 96 : 32) + MODE_WGRAD * 8 + cfg, flops);
    st = check_launch("conv_wgrad_tile");
  } else if (bf16) {
    const int bn = pick_bn(a.N);
    const int cfg = bn == 128 ? 0 : bn == 96 ? 1 : bn == 64 ? 2 : 3;
    dim3 grid(a.tiles_total * a.splits), block(256);
    if (timing_on()) timing_begin(s);
    if (cfg == 0) hipLaunchKernelGGL((conv_wgrad_bf16<128, 128, 2, 2>), grid, block, 0, s, a);
    else if (cfg == 1) hipLaunchKernelGGL((conv_wgrad_bf16<128, 96, 4, 1>), grid, block, 0, s, a);
    else if (cfg == 2) hipLaunchKernelGGL((conv_wgrad_bf16<256, 64, 4, 1>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv_wgrad_bf16<256, 32, 4, 1>), grid, block, 0, s, a);
    if (timing_on()) timing_end(s, 64 + MODE_WGRAD * 8 + cfg, flops);
    st = check_launch("conv_wgrad_bf16");
  } else {
    st = launch_gemm<MODE_WGRAD>(a, s, flops);
  }
  if (st) return st;
  launch_wgrad_reduce(s, static_cast<const float*>(workspace), p.splits, p.split_stride, g.taps,
                      g.cin_p, d->cin, d->cout, p.ldc, dw, db, accumulate, bn_g, bn_v, bn_eps);
  return check_launch("wgrad_reduce");
}

// ---- the stem's whole backward in one conv kernel (conv_wgrad_stem_x3<NP, true>) -----------
static bool stem_fused_ok(const of_conv_desc* d, int prec) {
  return (prec == 2 || (prec == 1 && g_stem_bf16)) && stem_wg_ok(d) && d->ho % 2 == 0 &&
         d->wo % 2 == 0 && d->cout == 64;
}

size_t of_stem_bwd_fused_workspace(const of_conv_desc* d, int precision) {
  if (validate(d) != OF_OK || !stem_fused_ok(d, precision)) return 0;
  WgradPlan p = wgrad_plan(d, precision == 1, true);
  return (size_t)p.splits * (p.M + 2) * p.ldc * sizeof(float);
}

int of_stem_bwd_fused(const of_conv_desc* d, int precision, const float* x, int ldx,
                      const float* dyp, const float* g, const float* y, const float* gamma,
                      const float* beta, const float* var, float eps, float* dw, float* dbias,
                      float* dgamma, float* dbeta, int accumulate, void* workspace,
                      size_t ws_bytes, void* stream) {
  int st = validate(d);
  if (st) return st;
  if (!stem_fused_ok(d, precision))
    return fail(OF_EUNSUPPORTED, "stem bwd fused: not the 7x7/2 3->64 stem on the split / bf16 "
                                 "kernels with an even output");
  OF_CHECK_ARG(x && dyp && y && gamma && beta && var && dw && workspace, "stem bwd fused: NULL");
  OF_CHECK_ARG(ldx >= d->cin_p && ldx % 4 == 0, "stem bwd fused: ldx");
  WgradPlan p = wgrad_plan(d, precision == 1, true);
  const int64_t stride = (int64_t)(p.M + 2) * p.ldc;
  OF_CHECK_ARG(ws_bytes >= (size_t)p.splits * stride * sizeof(float),
               "stem bwd fused: workspace too small");
  GemmArgs a = base_args(d);
  a.kc = d->cin_p;
  a.N = d->cout;
  a.M = p.M;
  a.A = x;
  a.lda = ldx;
  a.a_bytes = (int64_t)d->n * d->h * d->w * ldx * 4;
  a.B = y;                                     // (only sizes the FUSED resources)
  a.ldb = 64;
  a.b_bytes = (int64_t)d->n * d->ho * d->wo * 64 * 4;
  OF_CHECK_ARG(a.a_bytes < INT32_MAX && a.b_bytes < INT32_MAX, "stem bwd fused: < 2 GiB tensors");
  a.nb = 64;
  a.slab = static_cast<float*>(workspace);
  a.slab_ld = p.ldc;
  a.splits = p.splits;
  a.k_per_split = p.k_per_split;
  a.split_stride = stride;
  a.colsum = 0;
  a.K = stem_wg_tiles(d);
  a.bn_g = gamma;
  a.bn_b = beta;
  a.bn_v = var;
  a.bn_eps = eps;
  a.st_dyp = dyp;
  a.st_g = g;
  a.st_y = y;
  hipStream_t s = as_stream(stream);
  const double flops = 2.0 * (double)d->n * d->ho * d->wo * d->cout * 49 * d->cin;
  if (timing_on()) timing_begin(s);
  if (precision == 1) hipLaunchKernelGGL((conv_wgrad_stem_x3<1, true>), dim3(a.splits), dim3(SW_NT), 0, s, a);
  else hipLaunchKernelGGL((conv_wgrad_stem_x3<3, true>), dim3(a.splits), dim3(SW_NT), 0, s, a);
  if (timing_on()) timing_end(s, precision == 1 ? 187 : 185, flops);   // bench.py KIND_STEM_*
  st = check_launch("conv_wgrad_stem_x3 fused");
  if (st) return st;
  Geo gg = geo(d);
  launch_wgrad_reduce(s, static_cast<const float*>(workspace), p.splits, stride, gg.taps,
                      gg.cin_p, d->cin, d->cout, p.ldc, dw, nullptr, accumulate, nullptr, nullptr,
                      0.f);
  st = check_launch("wgrad_reduce");
  if (st) return st;
  hipLaunchKernelGGL(stem_bn_final, dim3(1), dim3(256), 0, s, static_cast<const float*>(workspace),
                     p.splits, stride, p.ldc, d->cout, gamma, var, eps, dgamma, dbeta, dbias,
                     accumulate);
  return check_launch("stem_bn_final");
}

int of_conv2d_wgrad(const of_conv_desc* d, const float* x, int ldx, const float* dy, int lddy,
                    float* dw, float* db, int accumulate, void* workspace, size_t ws_bytes,
                    void* stream) {
  return conv_wgrad_impl(0, d, x, ldx, dy, lddy, dw, db, accumulate, workspace, ws_bytes,
                         stream);
}

int of_conv2d_wgrad_bf16(const of_conv_desc* d, const float* x, int ldx, const float* dy,
                         int lddy, float* dw, float* db, int accumulate, void* workspace,
                         size_t ws_bytes, void* stream) {
  return conv_wgrad_impl(1, d, x, ldx, dy, lddy, dw, db, accumulate, workspace, ws_bytes,
                         stream);
}

int of_conv2d_wgrad_x3(const of_conv_desc* d, const float* x, int ldx, const float* dy,
                       int lddy, float* dw, float* db, int accumulate, void* workspace,
                       size_t ws_bytes, void* stream) {
  return conv_wgrad_impl(2, d, x, ldx, dy, lddy, dw, db, accumulate, workspace, ws_bytes,
                         stream);
}


// ---- inference-BN folded into the backward (FusedBatchNormGrad) --------
int of_conv_pack_weights_bn(const of_conv_desc* d, int precision, const float* w_hwio,
                            void* w_fwd, void* w_bwd, const float* bn_gamma,
                            const float* bn_var, float bn_eps, void* stream) {
  int st = validate(d);
  if (st) return st;
  OF_CHECK_ARG(precision >= 0 && precision <= 2, "pack bn: precision 0, 1 or 2");
  OF_CHECK_ARG(w_hwio && w_fwd && w_bwd, "pack bn: NULL pointer");
  OF_CHECK_ARG(!bn_gamma || bn_var, "pack bn: gamma without var");
  const int64_t total = pack_work(d, precision ? 1 : 0);
  OF_CHECK_ARG(total < INT32_MAX, "pack: layer too large");
  PackEntry E = pack_entry(d, w_hwio, w_fwd, w_bwd, precision);
  E.bn_g = bn_gamma;
  E.bn_v = bn_var;
  E.bn_eps = bn_eps;
  const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 4096);
  hipLaunchKernelGGL(pack_one_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), E, total);
  return check_launch("pack_bn");
}

int of_conv_pack_table_bn(int nconv, const of_conv_desc* descs, const float* const* w_hwio,
                          void* const* w_fwd, void* const* w_bwd, const int* precision,
                          const float* const* bn_gamma, const float* const* bn_var,
                          float bn_eps, void* host_table) {
  int st = of_conv_pack_table_ex(nconv, descs, w_hwio, w_fwd, w_bwd, precision, host_table);
  if (st || !bn_gamma) return st;
  OF_CHECK_ARG(bn_var != nullptr, "pack table bn: gamma without var");
  PackEntry* e = reinterpret_cast<PackEntry*>(static_cast<char*>(host_table) +
                                              sizeof(PackTableHeader));
  for (int i = 0; i < nconv; ++i) {
    OF_CHECK_ARG(!bn_gamma[i] || bn_var[i], "pack table bn: gamma without var");
    e[i].bn_g = bn_gamma[i];
    e[i].bn_v = bn_var[i];
    e[i].bn_eps = bn_eps;
  }
  return OF_OK;
}

size_t of_conv2d_wgrad_bn_workspace(const of_conv_desc* d, int precision) {
  return precision == 1 ? of_conv2d_wgrad_bf16_workspace(d)
         : precision == 2 ? of_conv2d_wgrad_x3_workspace(d) : of_conv2d_wgrad_workspace(d);
}

int of_conv2d_wgrad_bn(const of_conv_desc* d, int precision, const float* x, int ldx,
                       const float* t, int ldt, float* dw, int accumulate, const float* bn_gamma,
                       const float* bn_var, float bn_eps, void* workspace, size_t ws_bytes,
                       void* stream) {
  OF_CHECK_ARG(precision >= 0 && precision <= 2, "wgrad bn: precision 0, 1 or 2");
  OF_CHECK_ARG(bn_gamma && bn_var, "wgrad bn: gamma / var");
  return conv_wgrad_impl(precision, d, x, ldx, t, ldt, dw, nullptr, accumulate, workspace,
                         ws_bytes, stream, bn_gamma, bn_var, bn_eps);
}

int of_conv2d_dgrad_add_act(const of_conv_desc* d, int precision, const float* dy, int lddy,
                            const void* w_bwd, const float* add, int ld_add,
                            const float* act_src, int ld_act, int act, float alpha, float* dx,
                            int lddx, void* workspace, size_t ws_bytes, void* stream) {
  OF_CHECK_ARG(precision >= 0 && precision <= 2, "dgrad add act: precision 0, 1 or 2");
  OF_CHECK_ARG(act_src && (act == OF_ACT_RELU || act == OF_ACT_LEAKY),
               "dgrad add act: act_src and a relu / leaky act");
  return conv_dgrad_impl(precision, d, dy, lddy, w_bwd, act_src, ld_act, act, alpha, add,
                         ld_add, dx, lddx, workspace, ws_bytes, stream, 1);
}

size_t of_conv2d_dgrad_bnp_bytes(const of_conv_desc* d) {
  if (validate(d)) return 0;
  Geo g = geo(d);
  size_t bytes = 0;
  for (int f = 0; f < 3; ++f) {   // conv_tile_x3, conv_tile_b16, conv_tile_bf16 / the GEMM
    GemmArgs a;
    if (tile_ok(d)) {
      a = tile_args(d, g, MODE_DGRAD, f == 0, f == 1);
    } else {
      a = dgrad_args(d, g, true, f == 1);
      gemm_x3_plan(a);
    }
    if (a.n_tiles > 0) bytes = std::max(bytes, (size_t)(a.tiles_total / a.n_tiles) * 2 * a.N * 4);
  }
  return bytes;
}

int of_conv2d_dgrad_add_act_bnp(const of_conv_desc* d, int precision, const float* dy, int lddy,
                                const void* w_bwd, const float* add, int ld_add,
                                const float* act_src, int ld_act, int act, float alpha,
                                float* dx, int lddx, const float* bn_gamma, const float* bn_beta,
                                const float* bn_res, int ld_bn_res, float* part,
                                size_t part_bytes, int* nblk, void* workspace, size_t ws_bytes,
                                void* stream) {
  OF_CHECK_ARG(precision >= 0 && precision <= 2, "dgrad add act bnp: precision 0, 1 or 2");
  OF_CHECK_ARG(act_src && (act == OF_ACT_RELU || act == OF_ACT_LEAKY),
               "dgrad add act bnp: act_src and a relu / leaky act");
  const BnpArgs b{bn_gamma, bn_beta, bn_res, ld_bn_res, part, part_bytes, nblk};
  return conv_dgrad_impl(precision, d, dy, lddy, w_bwd, act_src, ld_act, act, alpha, add,
                         ld_add, dx, lddx, workspace, ws_bytes, stream, 1, &b);
}

}  // extern "C"
