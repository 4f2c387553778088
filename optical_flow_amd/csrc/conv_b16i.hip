// bf16 3x3 stride-1 convolution (fwd / input gradient) from a bf16 activation IMAGE, for the
// bf16 configs 3-5 (model.py:104-114 decoder convs, the resnet blocks' 3x3 convs).
//
// The round-1..3 bf16 kernels (conv_tile_bf16, conv_tile_b16, conv_tile_ws) read fp32
// activations and round them while staging (VGPR round trip + v_cvt + ds_write), on 128-256
// pixel tiles with a barrier per 24-32 MFMAs; all three measured 400-570 TFLOP/s.  This kernel
// follows the large-tile, DMA-fed structure of the guide's 256x256 GEMM template instead:
//
//   * A is a bf16 NHWC image (channels padded to a multiple of 32 with zeros), so the halo of
//     a 32-channel chunk goes global -> LDS by buffer_load ... lds (LDS DMA, 16 B per lane, no
//     VGPR staging, no conversion); out-of-image halo pixels are out-of-range loads: zeros.
//   * one workgroup of 8 waves per CU owns TH x TW = 16 x 32 output pixels x BN = 128 output
//     channels; each wave 128 pixels x 64 channels = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16.
//   * K runs as (chunk, kernel row) steps: per step 3 taps x 32 channels = 96 MFMAs per wave
//     between barriers (the round-3 kernels: 24-32).  B (the packed bf16 weights, 3 taps x BN
//     rows x 64 B) is DMA'd one step ahead, the next chunk's 18 x 34 halo one chunk ahead.
//   * LDS rows are 64 bytes (32 bf16) with the octet swizzle x3_sw (conflict-free 16x16x32
//     fragment reads, conv_f32.hip tile_x3_body); the DMA keeps the image lane-linear by
//     pre-swizzling each lane's source octet (guide rule 21).
//   * epilogue: the fp32 epilogues of conv_dev.h (bias, BN, residual, activation / the
//     producer's activation derivative) through a per-wave LDS transpose as 16-byte rows.
#include "conv_dev.h"

namespace oflow {

namespace {

constexpr int BI_TH = 16, BI_TW = 32;

template <int BN, int WAVES_M, int WAVES_N, int MODE, int TH, int TW>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N, 1) void conv_halo_b16(GemmArgs a) {
  constexpr int KS = 3;
  constexpr int NT = 64 * WAVES_M * WAVES_N, NW = NT / 64;
  constexpr int BM = TH * TW;
  constexpr int HH = TH + KS - 1, HW = TW + KS - 1, HP = HH * HW;
  constexpr int HPD = (HP + 15) / 16 * 16;             // whole 16-pixel DMA instructions
  constexpr int HDI = HPD / 16, HDW = (HDI + NW - 1) / NW;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int SM = WM / 16, SN = WN / 16;
  static_assert(TW % 16 == 0 && WM % 16 == 0 && WN % 16 == 0 && SM >= 1 && SN >= 1, "tile");
  constexpr int BDI = KS * BN / 16, BDW = (BDI + NW - 1) / NW;   // B DMA instructions per step
  constexpr int H_U4 = HPD * 4, B_U4 = KS * BN * 4;               // uint4 per buffer
  constexpr int LOOP_U4 = 2 * H_U4 + 2 * B_U4;
  constexpr int EJ = NW * WM * 16 * SN * 4 <= LOOP_U4 * 16 ? SN
                     : NW * WM * 16 * 2 * 4 <= LOOP_U4 * 16 && SN % 2 == 0 ? 2 : 1;
  constexpr int EPW = 16 * EJ;
  constexpr int EP_U4 = NW * WM * EPW / 4;
  constexpr int SM_U4 = LOOP_U4 > EP_U4 ? LOOP_U4 : EP_U4;
  static_assert(SM_U4 * 16 <= 160 * 1024, "LDS");
  __shared__ uint4 smem[SM_U4];
  uint4* Hs = smem;                        // [2][HPD pixels][4 octets]
  uint4* Bs = smem + 2 * H_U4;             // [2][3 taps][BN rows][4 octets]

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
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  const int b = tile_m / (tiles_x * tiles_y);
  const int trem = tile_m - b * tiles_x * tiles_y;
  const int oy0 = (trem / tiles_x) * TH, ox0 = (trem % tiles_x) * TW;
  const int hy0 = MODE == MODE_FWD ? oy0 - a.pt : oy0 + a.pt - (KS - 1);
  const int hx0 = MODE == MODE_FWD ? ox0 - a.pl : ox0 + a.pl - (KS - 1);
  const int c_begin = split * a.k_per_split;
  const int c_end = min(a.K, c_begin + a.k_per_split);
  const int nsteps = c_end > c_begin ? (c_end - c_begin) * KS : 0;

  // a.A: the bf16 image, a.lda channels (bf16 elements) per pixel
  const rsrc_t ra = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rb = make_rsrc(a.B, a.b_bytes);

  // ---- halo DMA: instruction g = wave + NW k covers halo pixels 16 g .. 16 g + 15; lane L
  // loads octet (L & 3) ^ x3_sw(pixel) of pixel 16 g + (L >> 2) (the swizzled image stays
  // lane-linear in LDS)
  uint32_t h_off[HDW];
#pragma unroll
  for (int k = 0; k < HDW; ++k) {
    const int g = wave + NW * k;
    const int hp = 16 * g + (lane >> 2);
    const int oct = (lane & 3) ^ x3_sw(hp);
    const int sy = hy0 + hp / HW, sx = hx0 + hp % HW;
    const bool ok = g < HDI && hp < HP && (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW;
    h_off[k] = ok ? (uint32_t)((((int64_t)(b * SH + sy) * SW + sx) * a.lda + 8 * oct) * 2) : kOOB;
  }
  auto dma_halo = [&](int c, int buf) {
#pragma unroll
    for (int k = 0; k < HDW; ++k) {
      const int g = wave + NW * k;
      if (HDI % NW == 0 || g < HDI) dma16_to_lds(ra, Hs + buf * H_U4 + 64 * g, h_off[k], 64 * c);
    }
  };
  // ---- B DMA: instruction g -> tap s = g / (BN / 16), rows 16 (g % (BN / 16)) ..; lane L
  // loads octet (L & 3) ^ x3_sw(L >> 2) of row (L >> 2)
  uint32_t b_off[BDW];
  int b_tap[BDW];
#pragma unroll
  for (int k = 0; k < BDW; ++k) {
    const int g = wave + NW * k;
    const int s = g / (BN / 16), rbk = g % (BN / 16);
    const int n = rbk * 16 + (lane >> 2), o = (lane & 3) ^ x3_sw(lane >> 2);
    b_tap[k] = s;
    b_off[k] = g < BDI && n0 + n < a.nb ? (uint32_t)(((int64_t)(n0 + n) * a.ldb + 8 * o) * 2) : kOOB;
  }
  auto dma_b = [&](int c, int r, int buf) {
#pragma unroll
    for (int k = 0; k < BDW; ++k) {
      const int g = wave + NW * k;
      if (BDI % NW == 0 || g < BDI)
        dma16_to_lds(rb, Bs + buf * B_U4 + 64 * g, b_off[k],
                     ((r * KS + b_tap[k]) * a.kc + 32 * c) * 2);
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
  // halo pixel of this lane's A row of fragment i at tap (0, 0): a_hp0 + the fragment's
  // (compile-time) offset -- fragment i covers tile row (wm0 + 16 i) / TW
  static_assert(WM % TW == 0 || TW % WM == 0, "wave rows");
  const int a_hp0 = [&] {
    const int ty = wm0 / TW, tx = wm0 % TW + l16;
    return MODE == MODE_FWD ? ty * HW + tx : (ty + KS - 1) * HW + tx + KS - 1;
  }();
  auto frag_hp = [&](int i) { return a_hp0 + ((16 * i) / TW) * HW + (16 * i) % TW; };
  const int b_frag = (wn0 + l16) * 4 + (lq ^ x3_sw(l16));

  if (nsteps > 0) {
    dma_b(c_begin, 0, 0);
    dma_halo(c_begin, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int q = 0; q < nsteps; ++q) {
    const int cc = q / KS, r = q - cc * KS;
    const int c = c_begin + cc;
    const int hbuf = cc & 1, bbuf = q & 1;
    // prefetch: the next step's B, then (at a chunk's first row) the next chunk's halo; the
    // buffers they overwrite were last read before the previous step's closing barrier
    if (q + 1 < nsteps) dma_b(r + 1 < KS ? c : c + 1, r + 1 < KS ? r + 1 : 0, bbuf ^ 1);
    if (r == 0 && c + 1 < c_end) dma_halo(c + 1, hbuf ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    const uint4* H = Hs + hbuf * H_U4;
    const uint4* Bq = Bs + bbuf * B_U4;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int dh = MODE == MODE_FWD ? r * HW + s : -(r * HW + s);
      bf16x8 av[SM], bv[SN];
#pragma unroll
      for (int j = 0; j < SN; ++j)
        bv[j] = __builtin_bit_cast(bf16x8, Bq[s * BN * 4 + 64 * j + b_frag]);
#pragma unroll
      for (int i = 0; i < SM; ++i) {
        const int px = frag_hp(i) + dh;
        av[i] = __builtin_bit_cast(bf16x8, H[px * 4 + (lq ^ x3_sw(px))]);
      }
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < SN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs of the next step landed
    __syncthreads();
  }

  // ---- epilogue: the wave's accumulators through a private LDS image (EJ 16-column blocks
  // per pass), back as float4 rows (16-byte loads / stores, 4 EJ lanes per pixel row)
  const int64_t img = (int64_t)b * OH * OW;
  float* E = reinterpret_cast<float*>(smem) + wave * WM * EPW;
  constexpr int LPR = 4 * EJ, RPI = 64 / LPR;
  const int c4 = lane % LPR, rr = lane / LPR;
#pragma unroll
  for (int jp = 0; jp < SN; jp += EJ) {
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < EJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) E[(16 * i + 4 * lq + r) * EPW + 16 * j + l16] = acc[i][jp + j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int n = n0 + wn0 + 16 * jp + 4 * c4;
    constexpr int EB = (WM / RPI) % 4 == 0 ? 4 : 1;
#pragma unroll
    for (int q0 = 0; q0 < WM / RPI; q0 += EB) {
      float4 v[EB];
      int64_t row[EB];
      unsigned ok = 0;
#pragma unroll
      for (int g = 0; g < EB; ++g) {
        const int m = (q0 + g) * RPI + rr;
        v[g] = *reinterpret_cast<const float4*>(&E[m * EPW + 4 * c4]);
        const int mt = wm0 + m;
        const int oy = oy0 + mt / TW, ox = ox0 + mt % TW;
        row[g] = img + (int64_t)oy * OW + ox;
        ok |= (oy < OH && ox < OW && n < a.N ? 1u : 0u) << g;
      }
      epilogue_rows4<MODE, EB>(a, split, row, ok, n, v);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// fp32 -> bf16 NHWC image with ldo channels per pixel, channels [c, ldo) zero (RNE): one
// thread per (pixel, 8-channel octet).
__global__ __launch_bounds__(256) void to_bf16_image_kernel(const float* __restrict__ x,
                                                            int64_t npix, int c, int ldx,
                                                            uint4* __restrict__ y, int ldo) {
  const int no = ldo / 8;
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= npix * no) return;
  const int64_t p = idx / no;
  const int o = (int)(idx - p * no);
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int ch = 8 * o + e;
    v[e] = ch < c ? x[p * ldx + ch] : 0.f;
  }
  const uint2 lo = pack_bf16x4(make_float4(v[0], v[1], v[2], v[3]));
  const uint2 hi = pack_bf16x4(make_float4(v[4], v[5], v[6], v[7]));
  y[idx] = make_uint4(lo.x, lo.y, hi.x, hi.y);
}

}  // namespace

extern "C" {

int of_to_bf16_image(const float* x, int64_t npix, int c, int ldx, void* y16, int ldo,
                     void* stream) {
  OF_CHECK_ARG(x && y16 && npix > 0 && c > 0 && ldx >= c && ldo >= c && ldo % 8 == 0,
               "to_bf16_image: args");
  OF_CHECK_ARG(((uintptr_t)y16 & 15) == 0, "to_bf16_image: 16-byte aligned output");
  const int64_t n = npix * (ldo / 8);
  hipLaunchKernelGGL(to_bf16_image_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), x, npix, c, ldx, static_cast<uint4*>(y16), ldo);
  return check_launch("to_bf16_image");
}

// Experimental entry (round 4): mode 0 fwd / 1 input gradient of a 3x3 stride-1 conv whose
// A source (fwd: x, dgrad: dy) is a bf16 image a16 with lda16 channels per pixel (a multiple
// of 32, >= round_up(kc, 32), the channels past kc zero); w16: the packed bf16 fwd / bwd image
// of of_conv_pack_weights_bf16.  aux: fwd residual / dgrad added gradient (ldr); act_src:
// dgrad activation source.  Unsplit (one K slice).
int of_conv2d_b16i(int mode, const of_conv_desc* d, const void* a16, int lda16, const void* w16,
                   const float* bias, const float* bn_gamma, const float* bn_beta,
                   const float* bn_mean, const float* bn_var, float bn_eps, const float* aux,
                   int ldr, const float* act_src, int ld_act, int act, float alpha, float* y,
                   int ldy, void* stream) {
  OF_CHECK_ARG(d && a16 && w16 && y, "conv b16i: NULL pointer");
  OF_CHECK_ARG(d->kh == 3 && d->kw == 3 && d->stride == 1, "conv b16i: 3x3 stride 1 only");
  OF_CHECK_ARG(mode == 0 || mode == 1, "conv b16i: mode");
  const int cout_p = (int)round_up(d->cout, 4);
  const int kc = mode == 0 ? d->cin_p : cout_p;
  const int N = mode == 0 ? d->cout : d->cin_p;
  OF_CHECK_ARG(lda16 % 32 == 0 && lda16 >= round_up(kc, 32), "conv b16i: lda16");
  OF_CHECK_ARG(N % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)y & 15) == 0, "conv b16i: output");
  GemmArgs a{};
  a.n = d->n, a.h = d->h, a.w = d->w, a.ho = d->ho, a.wo = d->wo;
  a.kh = 3, a.kw = 3, a.stride = 1, a.pt = d->pad_top, a.pl = d->pad_left, a.dt = 1;
  a.kc = kc;
  a.N = N;
  a.nb = mode == 0 ? d->cout : d->cin_p;
  const int kf16 = (int)round_up((int64_t)9 * d->cin_p, 32);
  const int kd16 = (int)round_up((int64_t)9 * cout_p, 32);
  a.ldb = mode == 0 ? kf16 : kd16;
  const int OH = mode == 0 ? d->ho : d->h, OW = mode == 0 ? d->wo : d->w;
  const int SH = mode == 0 ? d->h : d->ho, SW = mode == 0 ? d->w : d->wo;
  constexpr int BN = 128;
  OF_CHECK_ARG(N <= BN, "conv b16i: N <= 128 (experimental)");
  a.n_tiles = (int)cdiv(N, BN);
  const int64_t mt = (int64_t)d->n * cdiv(OH, BI_TH) * cdiv(OW, BI_TW);
  a.tiles_total = (int)(mt * a.n_tiles);
  a.K = (int)cdiv(kc, 32);
  a.k_per_split = a.K;
  a.splits = 1;
  a.A = static_cast<const float*>(a16);
  a.lda = lda16;
  a.a_bytes = (int64_t)d->n * SH * SW * lda16 * 2;
  a.B = static_cast<const float*>(w16);
  a.b_bytes = (int64_t)a.nb * a.ldb * 2;
  OF_CHECK_ARG(a.a_bytes < INT32_MAX && a.b_bytes < INT32_MAX, "conv b16i: < 2 GiB tensors");
  a.C = y, a.ldc = ldy;
  a.bias = mode == 0 ? bias : nullptr;
  a.bn_g = mode == 0 ? bn_gamma : nullptr;
  a.bn_b = bn_beta, a.bn_m = bn_mean, a.bn_v = bn_var, a.bn_eps = bn_eps;
  a.res = aux, a.ldr = ldr;
  a.act_src = mode == 1 ? act_src : nullptr;
  a.ld_act = ld_act;
  a.act = act, a.alpha = alpha;
  a.vec_ep = 1;
  hipStream_t s = as_stream(stream);
  const double flops = 2.0 * d->n * d->ho * d->wo * (double)d->cout * 9 * d->cin;
  if (timing_on()) timing_begin(s);
  if (mode == 0)
    hipLaunchKernelGGL((conv_halo_b16<128, 4, 2, MODE_FWD, BI_TH, BI_TW>), dim3(a.tiles_total),
                       dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((conv_halo_b16<128, 4, 2, MODE_DGRAD, BI_TH, BI_TW>), dim3(a.tiles_total),
                       dim3(512), 0, s, a);
  if (timing_on()) timing_end(s, 256 + 8 * mode, flops);
  return check_launch("conv_halo_b16");
}

}  // extern "C"

}  // namespace oflow
