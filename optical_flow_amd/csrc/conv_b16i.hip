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
#include <algorithm>
#include <type_traits>

#include "conv_dev.h"

namespace oflow {

// of_set_tuning key 21: timing ablations of conv_halo_b16 (WRONG results, A/B only): bit 0
// skips the epilogue's global loads and stores, bit 1 the main loop's DMAs.
int g_b16i_abl = 0;
// of_set_tuning key 22: the forward's direct epilogue for bf16-image-only outputs (1, default)
int g_b16i_direct = 1;
// of_set_tuning key 24: conv_halo_b16 persistent over tile ranges (1; 2: on 8 workgroups,
// for tests) or one tile per workgroup (0, default: the persistent form measured even)
int g_b16i_persist = 0;

namespace {

constexpr int BI_TH = 16, BI_TW = 32;

__device__ __forceinline__ float4 bf16x4_to_f4(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}

// B16I_RING (A/B switch, tools/ab_build.sh): 3 = a 3-deep B ring, two steps' B in flight
// across raw barriers with counted vmcnt waits; measured 2 % SLOWER on the bf16 B=32 step
// than the one-step-ahead form (2, default: 1665 vs 1699 pairs/s, gpurun_out/exp12), so the
// main loop is not waiting on its B DMAs.
#ifndef B16I_RING
#define B16I_RING 2
#endif
// (Reading the next tap's fragments during this tap's MFMAs, two fragment sets, measured
// even: 1766/1768 vs 1771/1767 pairs/s, the compiler's schedule was the same; not kept.)
template <int BN, int WAVES_M, int WAVES_N, int MODE, int TH, int TW, bool PERSIST = false>
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
  // RING: B buffers.  3 (when it fits and not PERSIST): two steps' B in flight, the step's
  // end waits with a counted vmcnt (this step's DMAs stay in flight across a raw s_barrier);
  // 2: one step ahead, vmcnt(0) + __syncthreads() per step.
  constexpr int RING = B16I_RING == 3 && !PERSIST && (2 * H_U4 + 3 * B_U4) * 16 <= 160 * 1024 ? 3 : 2;
  constexpr int LOOP_U4 = 2 * H_U4 + RING * B_U4;
  constexpr int EJ = NW * WM * 16 * SN * 4 + WAVES_M * BN * 4 <= LOOP_U4 * 16 ? SN
                     : NW * WM * 16 * 2 * 4 + WAVES_M * BN * 4 <= LOOP_U4 * 16 && SN % 2 == 0 ? 2
                                                                                     : 1;
  constexpr int EPW = 16 * EJ;
  constexpr int EP_U4 = NW * WM * EPW / 4 + WAVES_M * BN / 4;     // + the column-sum buffer
  // direct epilogue: per-wave row images of WN columns -- bf16 all WM rows (16-byte padded
  // pitch), fp32 WM / 2 rows per pass (32-byte padded: conflict-free 64-bit writes)
  constexpr int P16 = WN * 2 + 16, P32 = WN * 4 + 32;
  static_assert(SM % 2 == 0, "fp32 direct epilogue: two passes of SM / 2 row blocks");
  constexpr int DE_B = NW * WM * P16 > NW * (WM / 2) * P32 ? NW * WM * P16 : NW * (WM / 2) * P32;
  constexpr int D_U4 = DE_B / 16 + WAVES_M * BN / 4;
  constexpr int SM_U4 = (LOOP_U4 > EP_U4 ? LOOP_U4 : EP_U4) > D_U4 ? (LOOP_U4 > EP_U4 ? LOOP_U4 : EP_U4)
                                                                   : D_U4;
  static_assert(SM_U4 * 16 <= 160 * 1024, "LDS");
  static_assert(SM * SN * 4 <= 128, "sign mask: 128 bits per lane");
  // PERSIST: a workgroup per CU walks a contiguous range of tiles; after a tile's main loop it
  // issues the next tile's first B and halo DMAs into the buffers the last step did not read,
  // then runs the direct epilogue in the halo buffer it did read (passes of RB row blocks per
  // wave), so the next tile's first loads are in flight during the epilogue.
  // rows blocks per pass, by output element size e: whole store instructions, one halo buffer
  constexpr auto rb_ok = [](int rb, int e, int sm, int wn, int nw, int hb) {
    return sm % rb == 0 && (16 * rb * (wn * e / 16)) % 64 == 0 &&
           nw * 16 * rb * (wn * e + 16 * (e / 2)) <= hb;
  };
  constexpr int HB = H_U4 * 16;
  constexpr int PRB16 = rb_ok(1, 2, SM, WN, NW, HB) ? 1 : rb_ok(2, 2, SM, WN, NW, HB) ? 2 : 0;
  constexpr int PRB32 = rb_ok(1, 4, SM, WN, NW, HB) ? 1 : rb_ok(2, 4, SM, WN, NW, HB) ? 2 : 0;
  static_assert(!PERSIST || (PRB16 > 0 && PRB32 > 0), "persistent epilogue passes must fit a halo buffer");
  static_assert(!PERSIST || WAVES_M * BN * 4 <= B_U4 * 16, "column sums in a B buffer");
  __shared__ uint4 smem[SM_U4];
  uint4* Hs = smem;                        // [2][HPD pixels][4 octets]
  uint4* Bs = smem + 2 * H_U4;             // [RING][3 taps][BN rows][4 octets]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int OH = MODE == MODE_FWD ? a.ho : a.h, OW = MODE == MODE_FWD ? a.wo : a.w;
  const int SH = MODE == MODE_FWD ? a.h : a.ho, SW = MODE == MODE_FWD ? a.w : a.wo;
  const int tiles_x = (OW + TW - 1) / TW, tiles_y = (OH + TH - 1) / TH;
  // work items: split * tiles_total + tile (PERSIST: one split, this workgroup's range)
  const int w_begin = PERSIST ? (int)((int64_t)wgid * a.tiles_total / gridDim.x) : wgid;
  const int w_end = PERSIST ? (int)((int64_t)(wgid + 1) * a.tiles_total / gridDim.x) : wgid + 1;
  if (w_begin >= w_end) return;                     // (uniform over the workgroup)
  struct Geo { int tile, tile_m, n0, b, oy0, ox0, hy0, hx0, c_begin, c_end; };
  auto geo_of = [&](int wid) {
    Geo g;
    const int split = wid / a.tiles_total;
    g.tile = wid - split * a.tiles_total;
    const int tile_n = g.tile % a.n_tiles;
    g.tile_m = g.tile / a.n_tiles;
    g.n0 = tile_n * BN;
    g.b = g.tile_m / (tiles_x * tiles_y);
    const int trem = g.tile_m - g.b * tiles_x * tiles_y;
    g.oy0 = (trem / tiles_x) * TH, g.ox0 = (trem % tiles_x) * TW;
    g.hy0 = MODE == MODE_FWD ? g.oy0 - a.pt : g.oy0 + a.pt - (KS - 1);
    g.hx0 = MODE == MODE_FWD ? g.ox0 - a.pl : g.ox0 + a.pl - (KS - 1);
    g.c_begin = split * a.k_per_split;
    g.c_end = min(a.K, g.c_begin + a.k_per_split);
    return g;
  };
  Geo G = geo_of(w_begin);

  // a.A: the bf16 image, a.lda channels (bf16 elements) per pixel
  const rsrc_t ra = make_rsrc(a.A, a.a_bytes);
  const rsrc_t rb = make_rsrc(a.B, a.b_bytes);

  // ---- halo DMA: instruction g = wave + NW k covers halo pixels 16 g .. 16 g + 15; lane L
  // loads octet (L & 3) ^ x3_sw(pixel) of pixel 16 g + (L >> 2) (the swizzled image stays
  // lane-linear in LDS)
  uint32_t h_off[HDW];
  auto set_halo = [&](const Geo& t) {
#pragma unroll
    for (int k = 0; k < HDW; ++k) {
      const int g = wave + NW * k;
      const int hp = 16 * g + (lane >> 2);
      const int oct = (lane & 3) ^ x3_sw(hp);
      const int sy = t.hy0 + hp / HW, sx = t.hx0 + hp % HW;
      const bool ok = g < HDI && hp < HP && (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW;
      h_off[k] = ok ? (uint32_t)((((int64_t)(t.b * SH + sy) * SW + sx) * a.lda + 8 * oct) * 2) : kOOB;
    }
  };
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
  auto set_b = [&](const Geo& t) {
#pragma unroll
    for (int k = 0; k < BDW; ++k) {
      const int g = wave + NW * k;
      const int s = g / (BN / 16), rbk = g % (BN / 16);
      const int n = rbk * 16 + (lane >> 2), o = (lane & 3) ^ x3_sw(lane >> 2);
      b_tap[k] = s;
      b_off[k] = g < BDI && t.n0 + n < a.nb ? (uint32_t)(((int64_t)(t.n0 + n) * a.ldb + 8 * o) * 2)
                                            : kOOB;
    }
  };
  auto dma_b = [&](int c, int r, int buf) {
#pragma unroll
    for (int k = 0; k < BDW; ++k) {
      const int g = wave + NW * k;
      if (BDI % NW == 0 || g < BDI)
        dma16_to_lds(rb, Bs + buf * B_U4 + 64 * g, b_off[k],
                     ((r * KS + b_tap[k]) * a.kc + 32 * c) * 2);
    }
  };

  // this wave's DMA instructions per B step / per halo (the counted waits of RING 3)
  const int nb_w = BDI % NW == 0 ? BDW : (BDI - wave + NW - 1) / NW;
  const int nh_w = HDI % NW == 0 ? HDW : (HDI - wave + NW - 1) / NW;
  static_assert(BDW + HDW <= 15, "vm_wait covers 0..15");
  auto vm_wait = [](int n) {               // s_waitcnt vmcnt(n), n wave-uniform
    switch (n) {
      case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
      case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
      case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
      case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
      case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
      case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
      case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
      case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
      case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
      case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
      case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    }
  };
  // a barrier that leaves this wave's LDS DMAs in flight (no vmcnt(0) as __syncthreads() has)
  auto raw_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

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
  const int b_frag0 = (wn0 + l16) * 4 + (lq ^ x3_sw(l16));

  int hoff = 0, boff = 0;          // buffer parity of the tile's first chunk / step (PERSIST)
  for (int wid = w_begin;; ++wid) {
  // (recomputed per tile: nothing but wid and the parities lives across the epilogue)
  G = geo_of(wid);
  set_halo(G);
  set_b(G);
  if (wid == w_begin && G.c_end > G.c_begin) {
    dma_b(G.c_begin, 0, 0);
    dma_halo(G.c_begin, 0);
    if (RING == 3 && (G.c_end - G.c_begin) * KS > 1)      // step 1's B (chunk c_begin, row 1)
      dma_b(G.c_begin, 1, 1);
  }
  const int tile = G.tile, tile_m = G.tile_m, n0 = G.n0, b = G.b, oy0 = G.oy0, ox0 = G.ox0;
  // the fragment bases, opaque per tile: left loop-invariant, the addresses derived from them
  // are hoisted out of the tile loop and stay live through the epilogue (PERSIST: spills)
  int a_hp = a_hp0, b_frag = b_frag0;
  if (PERSIST) asm volatile("" : "+v"(a_hp), "+v"(b_frag));
  auto frag_hp = [&](int i) { return a_hp + ((16 * i) / TW) * HW + (16 * i) % TW; };
  const int c_begin = G.c_begin, c_end = G.c_end;
  const int nsteps = c_end > c_begin ? (c_end - c_begin) * KS : 0;
  f32x4 acc[SM][SN];
#pragma unroll
  for (int i = 0; i < SM; ++i)
#pragma unroll
    for (int j = 0; j < SN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
  if (RING == 3) {                                   // the tile's first B and halo landed
    vm_wait(nsteps > 1 ? nb_w : 0);
    raw_barrier();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int q = 0; q < nsteps; ++q) {
    const int cc = q / KS, r = q - cc * KS;
    const int c = c_begin + cc;
    const int hbuf = (cc + hoff) & 1, bbuf = RING == 3 ? q % 3 : (q + boff) & 1;
    // prefetch: the B RING - 1 steps ahead, then (at a chunk's first row) the next chunk's
    // halo; the buffers they overwrite were last read before the previous step's barrier
    if (!(a.abl & 2)) {
      if (RING == 3) {
        const int q2 = q + 2, c2 = c_begin + q2 / KS;
        if (q2 < nsteps) dma_b(c2, q2 - (q2 / KS) * KS, q2 % 3);
      } else if (q + 1 < nsteps) {
        dma_b(r + 1 < KS ? c : c + 1, r + 1 < KS ? r + 1 : 0, bbuf ^ 1);
      }
      if (r == 0 && c + 1 < c_end) dma_halo(c + 1, hbuf ^ 1);
    }
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
    if (RING == 3) {
      // next step's B (issued a step ago) and, before a chunk's first step, its halo (issued
      // two steps ago) landed; younger DMAs stay in flight: this step's B (q + 2) and the
      // next chunk's halo while its chunk has rows to go
      const bool b_in = !(a.abl & 2) && q + 2 < nsteps;
      const bool h_in = !(a.abl & 2) && r < KS - 1 && c + 1 < c_end;
      vm_wait((b_in ? nb_w : 0) + (h_in ? nh_w : 0));
      raw_barrier();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's next-step DMAs landed
      __syncthreads();
    }
  }
  // PERSIST: the next tile's first B and halo go into the buffers the last step did not read
  // (every wave passed the last step's barrier); the epilogue works in the other halo buffer
  const bool more = PERSIST && wid + 1 < w_end;
  const int hl = ((nsteps > 0 ? nsteps / KS - 1 : 0) + hoff) & 1;
  const int bl = ((nsteps > 0 ? nsteps - 1 : 0) + boff) & 1;
  if (more) {
    const Geo Gn = geo_of(wid + 1);
    set_halo(Gn);
    set_b(Gn);
    if (Gn.c_end > Gn.c_begin) {
      dma_b(Gn.c_begin, 0, bl ^ 1);
      dma_halo(Gn.c_begin, hl ^ 1);
    }
  }

  if (a.direct16) {
    // the lane's column / row-group indices, opaque per tile: left loop-invariant, the LDS and
    // row addresses derived from them are hoisted out of the tile loop (PERSIST: spills)
    int lanee = lane;
    if (PERSIST) asm volatile("" : "+v"(lanee));
    const int l16e = lanee & 15, lqe = lanee >> 4;
    // ---- direct epilogue (one output, bf16 image or fp32; no residual / BN): the epilogue
    // math on the accumulators in their MFMA layout (lanee: column 16 j + l16e, rows
    // 16 i + 4 lqe + r); adjacent columns swapped between lanee pairs (DPP) so each lanee writes
    // 2 rows x 2 columns into a per-wave LDS row image (bf16: 32-bit writes, whole wave rows
    // at once; fp32: 64-bit writes, half the rows per pass), then whole 16-byte row chunks
    // out: every store instruction writes full 128-byte lines (the per-pass transposes of the
    // general epilogue store 32-byte row pieces, measured ~2.4 TB/s).  fwd also writes the
    // act' signs of its output (mask_out: 128 bits per lanee, the input gradient of the next
    // layer reads them as mask_in in the same layout); dgrad takes act' from those signs
    // (or none: ACT_NONE) and sums its columns (bias gradient) in registers.
    // (PERSIST with a next tile: the halo buffer the last step read, and the B buffer likewise
    // for the column sums; the next tile's first DMAs are writing the other two)
    char* Ew = PERSIST ? reinterpret_cast<char*>(Hs + hl * H_U4) : reinterpret_cast<char*>(smem);
    float* colb = PERSIST ? reinterpret_cast<float*>(Bs + bl * B_U4)
                          : reinterpret_cast<float*>(reinterpret_cast<char*>(smem) + DE_B);
    const int64_t img = (int64_t)b * OH * OW;
    const uint4 mk = MODE == MODE_DGRAD && a.mask_in ? a.mask_in[(int64_t)tile * NT + tid]
                                                     : make_uint4(~0u, ~0u, ~0u, ~0u);
    const uint32_t mki[4] = {mk.x, mk.y, mk.z, mk.w};
    uint32_t mo[4] = {0u, 0u, 0u, 0u};
    float bj[SN];
#pragma unroll
    for (int j = 0; j < SN; ++j) {
      const int nn = n0 + wn0 + 16 * j + l16e;
      bj[j] = MODE == MODE_FWD && a.bias && nn < a.N ? a.bias[nn] : 0.f;
    }
    float cs[SN];
#pragma unroll
    for (int j = 0; j < SN; ++j) cs[j] = 0.f;
    const bool even = !(l16e & 1);
    // rows [16 i0, 16 i1) of the wave: epilogue values -> the LDS row image (pitch P bytes,
    // E bytes per value) -> global
    auto emit = [&](auto I0, auto I1, auto PB, auto EB) {
      constexpr int i0 = decltype(I0)::value, i1 = decltype(I1)::value;
      constexpr int P = decltype(PB)::value, E = decltype(EB)::value;
      char* Ewv = Ew + wave * (16 * (i1 - i0)) * P;
#pragma unroll
      for (int i = i0; i < i1; ++i) {
        unsigned rv = 0;                   // row validity of rows 16 i + 4 lqe + r
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mt = wm0 + 16 * i + 4 * lqe + r;
          rv |= (oy0 + mt / TW < OH && ox0 + mt % TW < OW ? 1u : 0u) << r;
        }
#pragma unroll
        for (int j = 0; j < SN; ++j) {
          const bool cv = n0 + wn0 + 16 * j + l16e < a.N;
          float x[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int bit = (i * SN + j) * 4 + r;
            if (MODE == MODE_FWD) {
              x[r] = act_fwd(acc[i][j][r] + bj[j], a.act, a.alpha);
              mo[bit >> 5] |= (x[r] > 0.f ? 1u : 0u) << (bit & 31);
            } else {
              const bool pos = (mki[bit >> 5] >> (bit & 31)) & 1u;
              x[r] = dgrad_ep(a, acc[i][j][r], pos ? 1.f : -1.f, 0.f);
              if (cv && ((rv >> r) & 1)) cs[j] += x[r];
            }
          }
          const float p0 = even ? x[2] : x[0], p1 = even ? x[3] : x[1];
          const float q0 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
                                                         __builtin_bit_cast(int, p0), 0xB1, 0xF, 0xF, false));
          const float q1 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
                                                         __builtin_bit_cast(int, p1), 0xB1, 0xF, 0xF, false));
          const float4 w = even ? make_float4(x[0], q0, x[1], q1) : make_float4(q0, x[2], q1, x[3]);
          const int row0 = 16 * (i - i0) + 4 * lqe + (even ? 0 : 2);
          char* d = Ewv + row0 * P + (16 * j + (l16e & ~1)) * E;
          if (E == 2) {
            const uint2 u = pack_bf16x4(w);
            *reinterpret_cast<uint32_t*>(d) = u.x;
            *reinterpret_cast<uint32_t*>(d + P) = u.y;
          } else {
            *reinterpret_cast<float2*>(d) = make_float2(w.x, w.y);
            *reinterpret_cast<float2*>(d + P) = make_float2(w.z, w.w);
          }
        }
        // pin the sign words / column sums here: left free, the compiler sinks their updates
        // past every LDS write and keeps all the values live (spills)
        if (MODE == MODE_FWD) asm volatile("" : "+v"(mo[0]), "+v"(mo[1]), "+v"(mo[2]), "+v"(mo[3]));
#pragma unroll
        for (int j = 0; j < SN; ++j)
          if (MODE == MODE_DGRAD) asm volatile("" : "+v"(cs[j]));
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      constexpr int LR = WN * E / 16, NR = 16 * (i1 - i0);   // 16-byte chunks per row, rows
      static_assert((NR * LR) % 64 == 0, "whole store instructions");
#pragma unroll
      for (int it = 0; it < NR * LR / 64; ++it) {
        const int c = lanee + 64 * it, row = c / LR, part = c - row * LR;
        const uint4 v = *reinterpret_cast<const uint4*>(Ewv + row * P + 16 * part);
        const int mt = wm0 + 16 * i0 + row;
        const int oy = oy0 + mt / TW, ox = ox0 + mt % TW;
        const int ch = n0 + wn0 + 16 / E * part;
        if (oy < OH && ox < OW && ch < a.N) {
          const int64_t pix = img + (int64_t)oy * OW + ox;
          if (E == 2)
            *reinterpret_cast<uint4*>(&a.C16[pix * a.ldc16 + ch]) = v;
          else
            *reinterpret_cast<uint4*>(&a.C[pix * a.ldc + ch]) = v;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    using std::integral_constant;
    // passes of RB row blocks (PERSIST with a next tile: PRB16 / PRB32, inside one halo buffer)
    auto passes = [&](auto RBc, auto PB, auto EB) {
      constexpr int RB = decltype(RBc)::value;
      auto pass = [&](auto K) {
        constexpr int k = decltype(K)::value;
        if constexpr (RB > 0 && k * RB < SM)
          emit(integral_constant<int, k * RB>{}, integral_constant<int, (k + 1) * RB>{}, PB, EB);
      };
      pass(integral_constant<int, 0>{}), pass(integral_constant<int, 1>{});
      pass(integral_constant<int, 2>{}), pass(integral_constant<int, 3>{});
      pass(integral_constant<int, 4>{}), pass(integral_constant<int, 5>{});
      pass(integral_constant<int, 6>{}), pass(integral_constant<int, 7>{});
    };
    if (PERSIST) {                       // (the last tile too: one code path)
      if (a.C16)
        passes(integral_constant<int, PRB16>{}, integral_constant<int, P16>{}, integral_constant<int, 2>{});
      else
        passes(integral_constant<int, PRB32>{}, integral_constant<int, P32>{}, integral_constant<int, 4>{});
    } else if (a.C16) {
      emit(integral_constant<int, 0>{}, integral_constant<int, SM>{}, integral_constant<int, P16>{},
           integral_constant<int, 2>{});
    } else {
      emit(integral_constant<int, 0>{}, integral_constant<int, SM / 2>{},
           integral_constant<int, P32>{}, integral_constant<int, 4>{});
      emit(integral_constant<int, SM / 2>{}, integral_constant<int, SM>{},
           integral_constant<int, P32>{}, integral_constant<int, 4>{});
    }
    if (MODE == MODE_FWD && a.mask_out)
      a.mask_out[(int64_t)tile * NT + tid] = make_uint4(mo[0], mo[1], mo[2], mo[3]);
    if (MODE == MODE_DGRAD && a.col_part != nullptr) {
#pragma unroll
      for (int j = 0; j < SN; ++j) {        // fixed order: lqe 0+1, 2+3, then the halves
        cs[j] += __shfl_xor(cs[j], 16, 64);
        cs[j] += __shfl_xor(cs[j], 32, 64);
        if (lqe == 0) colb[(wave / WAVES_N) * BN + wn0 + 16 * j + l16e] = cs[j];
      }
      __syncthreads();
      if (tid < BN && n0 + tid < a.N) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < WAVES_M; ++w) v += colb[w * BN + tid];
        a.col_part[(int64_t)tile_m * a.N + n0 + tid] = v;
      }
    }
    if (!more) return;
    hoff = hl ^ 1, boff = bl ^ 1;
    continue;
  }
  if constexpr (PERSIST) return;         // (the host runs PERSIST with the direct epilogue only)

  // ---- epilogue: the wave's accumulators through a private LDS image (EJ 16-column blocks
  // per pass), back as float4 rows (16-byte loads / stores, 4 EJ lanes per pixel row).  Every
  // global load the epilogue needs is issued ahead of the stores that could alias it: the
  // biases of all passes up front, the bf16 act' image rows one pass ahead (row k of the next
  // pass is loaded once row k of this one is used, before its store), so their latency
  // overlaps a pass; fp32 act' sources and fwd residuals (off the bf16-image decoder path) in
  // their own pass, after its LDS transpose.  (The input gradient takes no added gradient.)
  const int64_t img = (int64_t)b * OH * OW;
  float* E = reinterpret_cast<float*>(smem) + wave * WM * EPW;
  float* colbuf = reinterpret_cast<float*>(smem) + NW * WM * EPW;   // [WAVES_M][BN]
  constexpr int LPR = 4 * EJ, RPI = 64 / LPR, ROWS = WM / RPI, NPASS = SN / EJ;
  const int c4 = lane % LPR, rr = lane / LPR;
  const bool colsums = MODE == MODE_DGRAD && a.col_part != nullptr;
  auto col_of = [&](int p) { return n0 + wn0 + 16 * EJ * p + 4 * c4; };
  auto row_of = [&](int k, unsigned& ok, int n) {   // output pixel (< 2^31: image < 2 GiB)
    const int mt = wm0 + k * RPI + rr;
    const int oy = oy0 + mt / TW, ox = ox0 + mt % TW;
    ok |= (oy < OH && ox < OW && n < a.N ? 1u : 0u) << k;
    return (int)img + oy * OW + ox;
  };
  float pb[NPASS][4];                                 // fwd: the bias of every pass's columns
#pragma unroll
  for (int p = 0; p < NPASS; ++p)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = col_of(p) + e;
      pb[p][e] = MODE == MODE_FWD && a.bias && n < a.N ? a.bias[n] : 0.f;
    }
  uint2 s16[ROWS];        // dgrad act' image rows: row k of the next pass once row k is used
  auto load_s16 = [&](int p, int k) {
    const int n = col_of(p);
    unsigned ok = 0;
    const int64_t row = row_of(k, ok, n);
    s16[k] = ok ? *reinterpret_cast<const uint2*>(&a.act16[row * a.ld_act16 + n])
                : make_uint2(0x3f803f80u, 0x3f803f80u);   // 1.0 (unused)
  };
  const bool pipe16 = MODE == MODE_DGRAD && a.act16 != nullptr && !(a.abl & 1);
  if (pipe16) {
#pragma unroll
    for (int k = 0; k < ROWS; ++k) load_s16(0, k);
  }
#pragma unroll
  for (int p = 0; p < NPASS; ++p) {
    const int jp = p * EJ;
    const int n = col_of(p);
    float4 aux[ROWS];
    float ps[4] = {1.f, 1.f, 1.f, 1.f}, pt[4] = {0.f, 0.f, 0.f, 0.f};   // fwd BN scale / shift
    unsigned ok = 0;
    int row[ROWS];
#pragma unroll
    for (int k = 0; k < ROWS; ++k) row[k] = row_of(k, ok, n);
    if (MODE == MODE_FWD && a.bn_g) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float bias;
        if (n + e < a.N) column_params<MODE>(a, n + e, bias, ps[e], pt[e]);
      }
    }
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < EJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) E[(16 * i + 4 * lq + r) * EPW + 16 * j + l16] = acc[i][jp + j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float4 v[ROWS];
#pragma unroll
    for (int k = 0; k < ROWS; ++k) v[k] = *reinterpret_cast<const float4*>(&E[(k * RPI + rr) * EPW + 4 * c4]);
    if (!(a.abl & 1)) {   // fwd residual / dgrad fp32 act' source rows (after the transpose)
#pragma unroll
      for (int k = 0; k < ROWS; ++k) {
        const bool in = (ok >> k) & 1;
        if (MODE == MODE_FWD)
          aux[k] = a.res && in ? *reinterpret_cast<const float4*>(&a.res[(int64_t)row[k] * a.ldr + n])
                               : make_float4(0.f, 0.f, 0.f, 0.f);
        else
          aux[k] = !a.act16 && a.act_src && in
                       ? *reinterpret_cast<const float4*>(&a.act_src[(int64_t)row[k] * a.ld_act + n])
                       : make_float4(1.f, 1.f, 1.f, 1.f);
      }
    }
    if (a.abl & 1) {                                  // ablation: keep the values, store nothing
      asm volatile("" ::"v"(v[0].x), "v"(v[ROWS - 1].w));
    } else {
      float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < ROWS; ++k) {
        const float4 sv = pipe16 ? bf16x4_to_f4(s16[k]) : aux[k];
        if (pipe16 && p + 1 < NPASS) load_s16(p + 1, k);   // refill: the next pass's row k
        if (!((ok >> k) & 1)) continue;
        const float vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        const float sa[4] = {sv.x, sv.y, sv.z, sv.w};
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (MODE == MODE_FWD) {
            float t = vv[e] + pb[p][e];
            if (a.bn_g) t = t * ps[e] + pt[e];
            x[e] = act_fwd(t + sa[e], a.act, a.alpha);
          } else {
            x[e] = dgrad_ep(a, vv[e], sa[e], 0.f);
          }
        }
        if (MODE == MODE_DGRAD) cs.x += x[0], cs.y += x[1], cs.z += x[2], cs.w += x[3];
        if (a.C)
          *reinterpret_cast<float4*>(&a.C[(int64_t)row[k] * a.ldc + n]) = make_float4(x[0], x[1], x[2], x[3]);
        if (a.C16)
          *reinterpret_cast<uint2*>(&a.C16[(int64_t)row[k] * a.ldc16 + n]) =
              pack_bf16x4(make_float4(x[0], x[1], x[2], x[3]));
      }
      if (colsums) {
        // sum over the RPI row groups of lanes with the same column quad, fixed order
#pragma unroll
        for (int o = LPR; o < 64; o <<= 1) {
          cs.x += __shfl_xor(cs.x, o, 64);
          cs.y += __shfl_xor(cs.y, o, 64);
          cs.z += __shfl_xor(cs.z, o, 64);
          cs.w += __shfl_xor(cs.w, o, 64);
        }
        if (rr == 0)
          *reinterpret_cast<float4*>(&colbuf[(wave / WAVES_N) * BN + wn0 + 16 * jp + 4 * c4]) = cs;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (colsums) {          // this tile's column sums: the WAVES_M row blocks in a fixed order
    __syncthreads();
    if (tid < BN && n0 + tid < a.N) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES_M; ++w) v += colbuf[w * BN + tid];
      a.col_part[(int64_t)tile_m * a.N + n0 + tid] = v;
    }
  }
  return;
  }   // tile loop
}

// ---- weight gradient from bf16 images: dW[r][s][ci][co] = sum_p x(p + (r, s) - pad)[ci] .
// dy(p)[co] (Conv2DBackpropFilter of the same convs).  A workgroup owns CIB input x COB output
// channels for all 9 taps and walks a contiguous range of 8 x 16 output-pixel tiles (its K
// slice).  Per tile the x halo (10 x 18 px x CIB) and the dy tile (128 px x COB) go global ->
// LDS by DMA, in the images' own [pixel][channel] layout, double-buffered one tile ahead; the
// MFMA operands want pixels along K, so they are read with ds_read_b64_tr_b16 (the hardware
// transposing read: a 16-lane group reads 4 pixel rows x 16 channels, lane i receives channel
// i's 4 pixels).  Each wave owns 32 ci x 32 co x 9 taps (v_mfma_f32_32x32x16_bf16, 9
// accumulators); per output row kk the B fragment (dy row kk) serves the 9 taps and an x-row
// fragment (halo row j, shift s) serves the output rows j - r, so a tile needs 10 x 3 + 8
// fragment reads for 72 MFMAs.  LDS chunk swizzles (16-byte chunks of a pixel row) make the
// transposing reads conflict-free: 256-byte rows XOR the chunk with (px & 3) << 2, 128-byte
// rows with ((px >> 1) & 1) << 2, 64-byte rows need none.  Output: fp32 slabs [slice][tap][kc][ldc] reduced in a fixed
// order by b16i_wgrad_reduce.
constexpr int WB_TH = 8, WB_TW = 16, WB_HH = WB_TH + 2, WB_HW = WB_TW + 2;
constexpr int WB_HP = WB_HH * WB_HW;          // 180 halo pixels

__device__ __forceinline__ int wb_sw(int px, int row_chunks) {
  // 64-byte rows (32 channels): a 32-lane half reads 4 consecutive rows = 256 contiguous
  // bytes, conflict-free as they lie (and a 4-chunk row has no chunk 4 to swap with)
  return row_chunks >= 16 ? (px & 3) << 2 : row_chunks == 8 ? ((px >> 1) & 1) << 2 : 0;
}

typedef short v4i16 __attribute__((ext_vector_type(4)));

// 8 bf16 (two transposing reads of 4 pixel rows each) of one MFMA operand fragment
__device__ __forceinline__ bf16x8 tr_frag(const char* base, int off0, int off1) {
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4i16*)(base + off0));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4i16*)(base + off1));
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int WAVES_CI, int WAVES_CO>
__global__ __launch_bounds__(64 * WAVES_CI * WAVES_CO, 1) void conv_wgrad_b16i(GemmArgs a) {
  constexpr int NW = WAVES_CI * WAVES_CO, NT = 64 * NW;
  constexpr int CIB = 32 * WAVES_CI, COB = 32 * WAVES_CO;
  constexpr int XC = CIB / 8, DC = COB / 8;                 // 16-byte chunks per pixel row
  constexpr int XPI = 64 / XC, DPI = 64 / DC;               // pixels per DMA instruction
  constexpr int XDI = (WB_HP + XPI - 1) / XPI, DDI = WB_TH * WB_TW / DPI;
  constexpr int XDW = (XDI + NW - 1) / NW, DDW = (DDI + NW - 1) / NW;
  constexpr int X_B = XDI * 1024, D_B = DDI * 1024;         // bytes per buffer (whole instrs)
  constexpr int LDS_B = 2 * (X_B + D_B);
  static_assert(LDS_B <= 160 * 1024, "LDS");
  __shared__ uint4 smem[LDS_B / 16];
  char* lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wgid / a.tiles_total;
  const int tile = wgid - split * a.tiles_total;
  const int tile_co = tile % a.n_tiles, tile_ci = tile / a.n_tiles;
  const int ci0 = tile_ci * CIB, co0 = tile_co * COB;
  const int t_begin = split * a.k_per_split;
  const int t_end = min(a.K, t_begin + a.k_per_split);
  const int ntiles = max(0, t_end - t_begin);
  const int tiles_x = (a.wo + WB_TW - 1) / WB_TW, tiles_y = (a.ho + WB_TH - 1) / WB_TH;
  const rsrc_t rx = make_rsrc(a.A, a.a_bytes);   // x image: a.lda bf16 per pixel
  const rsrc_t rd = make_rsrc(a.B, a.b_bytes);   // dy image: a.ldb bf16 per pixel

  // DMA slots: instruction g covers XPI halo pixels (DPI dy pixels); lane -> (pixel, chunk),
  // the chunk pre-swizzled so the image lands swizzled (recomputed per tile: registers)
  auto dma = [&](int t, int buf) {
    const int b = t / (tiles_x * tiles_y);
    const int trem = t - b * tiles_x * tiles_y;
    const int oy0 = (trem / tiles_x) * WB_TH, ox0 = (trem % tiles_x) * WB_TW;
    char* xb = lds + buf * (X_B + D_B);
    char* db = xb + X_B;
#pragma unroll
    for (int k = 0; k < XDW; ++k) {
      const int g = wave + NW * k;
      if (XDI % NW != 0 && g >= XDI) continue;
      const int hp = g * XPI + lane / XC;
      const int xch = (lane % XC) ^ wb_sw(hp, XC);
      const int iy = oy0 - a.pt + hp / WB_HW, ix = ox0 - a.pl + hp % WB_HW;
      const bool ok = hp < WB_HP && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w &&
                      ci0 + 8 * xch < a.kc;
      const uint32_t off = ok ? (uint32_t)((((int64_t)(b * a.h + iy) * a.w + ix) * a.lda + ci0 +
                                            8 * xch) * 2) : kOOB;
      dma16_to_lds(rx, reinterpret_cast<uint4*>(xb + 1024 * g), off, 0);
    }
#pragma unroll
    for (int k = 0; k < DDW; ++k) {
      const int g = wave + NW * k;
      if (DDI % NW != 0 && g >= DDI) continue;
      const int p = g * DPI + lane / DC;
      const int dch = (lane % DC) ^ wb_sw(p, DC);
      const int oy = oy0 + p / WB_TW, ox = ox0 + p % WB_TW;
      const bool ok = oy < a.ho && ox < a.wo && co0 + 8 * dch < a.nb;
      const uint32_t off = ok ? (uint32_t)((((int64_t)(b * a.ho + oy) * a.wo + ox) * a.ldb + co0 +
                                            8 * dch) * 2) : kOOB;
      dma16_to_lds(rd, reinterpret_cast<uint4*>(db + 1024 * g), off, 0);
    }
  };

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const int wci = (wave / WAVES_CO) * 32, wco = (wave % WAVES_CO) * 32;
  // transposing-read addresses: lane 4q + p of 16-lane group g reads row q, columns 4p..4p+3
  // of the group's 16 channels (16 (g & 1) within the wave's 32), pixels 8 (g >> 1) + q (+4)
  const int grp = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int colx = wci + 16 * (grp & 1) + 4 * pp;          // x channel (within CIB)
  const int cold = wco + 16 * (grp & 1) + 4 * pp;          // dy channel (within COB)
  auto xoff = [&](int px) {                                // byte offset of (px, colx) in a row
    const int ch = colx >> 3;
    return px * (XC * 16) + ((ch ^ wb_sw(px, XC)) << 4) + 2 * (colx & 7);
  };
  auto doff = [&](int px) {
    const int ch = cold >> 3;
    return px * (DC * 16) + ((ch ^ wb_sw(px, DC)) << 4) + 2 * (cold & 7);
  };
  const int kofs = 8 * (grp >> 1) + q;                      // this lane's pixel within K16

  if (ntiles > 0) dma(t_begin, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = 0; i < ntiles; ++i) {
    const int buf = i & 1;
    if (i + 1 < ntiles) dma(t_begin + i + 1, buf ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    const char* xb = lds + buf * (X_B + D_B);
    const char* db = xb + X_B;
    auto afrag = [&](int row, int s) {      // x halo row `row`, shift s: pixels row*18 + s + k
      const int px = row * WB_HW + s + kofs;
      return tr_frag(xb, xoff(px), xoff(px + 4));
    };
    auto bfrag = [&](int kk) {
      const int px = kk * WB_TW + kofs;
      return tr_frag(db, doff(px), doff(px + 4));
    };
    bf16x8 af[WB_HH][3];
#pragma unroll
    for (int row = 0; row < 3; ++row)
#pragma unroll
      for (int s = 0; s < 3; ++s) af[row][s] = afrag(row, s);
#pragma unroll
    for (int kk = 0; kk < WB_TH; ++kk) {
      const bf16x8 bv = bfrag(kk);
      if (kk + 3 < WB_HH) {          // x row kk + 3, first used by output row kk + 1
#pragma unroll
        for (int s = 0; s < 3; ++s) af[kk + 3][s] = afrag(kk + 3, s);
      }
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s)
          acc[r * 3 + s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kk + r][s], bv,
                                                                  acc[r * 3 + s], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- this slice's partial dW: slab [split][tap][kc rows][slab_ld] (32 x 32 layout: column
  // lane & 31, rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5))
  float* S = a.slab + (int64_t)split * a.split_stride;
  const int n = co0 + wco + (lane & 31);
  if (n < a.N) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = ci0 + wci + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (ci < a.M) S[((int64_t)t * a.M + ci) * a.slab_ld + n] = acc[t][r];
      }
  }
}

// dw[tap][ci][co] (+)= sum over slices of slab[slice][tap][ci][co] (fixed order), ci < cin,
// co < cout; one thread per (row, column quad).
__global__ __launch_bounds__(256) void b16i_wgrad_reduce(const float* __restrict__ slab, int slices,
                                                         int64_t stride, int rows, int ld,
                                                         int cout, float* __restrict__ dw, int acc,
                                                         const float* __restrict__ bn_g,
                                                         const float* __restrict__ bn_v,
                                                         float bn_eps) {
  const int cq = (cout + 3) / 4;
  const int64_t item = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (item >= (int64_t)rows * cq) return;
  const int row = (int)(item / cq), q = (int)(item - (int64_t)row * cq);
  const float* src = slab + (int64_t)row * ld + 4 * q;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  int z = 0;
  for (; z + 3 < slices; z += 4) {
    float4 u[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] = *reinterpret_cast<const float4*>(src + (int64_t)(z + k) * stride);
#pragma unroll
    for (int k = 0; k < 4; ++k) add4(v, u[k]);
  }
  for (; z < slices; ++z) add4(v, *reinterpret_cast<const float4*>(src + (int64_t)z * stride));
  float x[4] = {v.x, v.y, v.z, v.w};
  const int nv = min(4, cout - 4 * q);
  float* dst = dw + (int64_t)row * cout + 4 * q;
  for (int e = 0; e < nv; ++e) {
    float t = x[e];
    if (bn_g) t *= bn_g[4 * q + e] * rsqrtf(bn_v[4 * q + e] + bn_eps);
    dst[e] = acc ? dst[e] + t : t;
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

// Tile configurations by N tile: (BN, waves M x N, TH x TW) -- all 8 waves, 512-pixel tiles.
static int b16i_bn(int N) { return N > 96 ? 128 : N > 64 ? 96 : N > 32 ? 64 : 32; }

static int b16i_plan(int mode, const of_conv_desc* d, GemmArgs& a) {
  const int cout_p = (int)round_up(d->cout, 4);
  const int kc = mode == 0 ? d->cin_p : cout_p;
  const int N = mode == 0 ? d->cout : d->cin_p;
  a = GemmArgs{};
  a.n = d->n, a.h = d->h, a.w = d->w, a.ho = d->ho, a.wo = d->wo;
  a.kh = 3, a.kw = 3, a.stride = 1, a.pt = d->pad_top, a.pl = d->pad_left, a.dt = 1;
  a.kc = kc;
  a.N = N;
  a.nb = mode == 0 ? d->cout : d->cin_p;
  a.ldb = mode == 0 ? (int)round_up((int64_t)9 * d->cin_p, 32) : (int)round_up((int64_t)9 * cout_p, 32);
  const int OH = mode == 0 ? d->ho : d->h, OW = mode == 0 ? d->wo : d->w;
  const int bn = b16i_bn(N);
  a.n_tiles = (int)cdiv(N, bn);
  const int64_t mt = (int64_t)d->n * cdiv(OH, BI_TH) * cdiv(OW, BI_TW);
  if (mt * a.n_tiles >= INT32_MAX) return fail(OF_EINVAL, "conv b16i: too many tiles");
  a.tiles_total = (int)(mt * a.n_tiles);
  a.bm = BI_TH * BI_TW;
  a.K = (int)cdiv(kc, 32);
  a.k_per_split = a.K;
  a.splits = 1;
  a.M = (int)mt;                 // M tiles: rows of the column-sum partials
  return OF_OK;
}

size_t of_conv2d_b16i_mask_bytes(const of_conv_desc* d) {
  GemmArgs a;
  if (!d || b16i_plan(0, d, a)) return 0;
  return (size_t)a.tiles_total * 512 * 16;
}

int of_conv2d_b16i_tiles(int mode, const of_conv_desc* d) {
  GemmArgs a;
  if (!d || b16i_plan(mode, d, a)) return -1;
  return a.M;
}

int of_conv2d_b16i(int mode, const of_conv_desc* d, const of_b16i_io* io, const void* w16,
                   const float* bias, const float* bn_gamma, const float* bn_beta,
                   const float* bn_mean, const float* bn_var, float bn_eps, int act, float alpha,
                   void* stream) {
  OF_CHECK_ARG(d && io && io->a16 && w16, "conv b16i: NULL pointer");
  OF_CHECK_ARG(io->y || io->y16, "conv b16i: no output");
  OF_CHECK_ARG(d->kh == 3 && d->kw == 3 && d->stride == 1, "conv b16i: 3x3 stride 1 only");
  OF_CHECK_ARG(mode == 0 || mode == 1, "conv b16i: mode");
  GemmArgs a;
  if (int st = b16i_plan(mode, d, a)) return st;
  OF_CHECK_ARG(io->lda16 % 32 == 0 && io->lda16 >= round_up(a.kc, 32), "conv b16i: lda16");
  OF_CHECK_ARG(a.N % 4 == 0, "conv b16i: N % 4");
  OF_CHECK_ARG(!io->y || (io->ldy >= a.N && io->ldy % 4 == 0 && ((uintptr_t)io->y & 15) == 0),
               "conv b16i: fp32 output");
  OF_CHECK_ARG(!io->y16 || (io->ldy16 >= a.N && io->ldy16 % 4 == 0 && ((uintptr_t)io->y16 & 7) == 0),
               "conv b16i: bf16 output");
  OF_CHECK_ARG(!io->aux || (mode == 0 && io->ldr >= a.N && io->ldr % 4 == 0 &&
                            ((uintptr_t)io->aux & 15) == 0), "conv b16i: aux (fwd residual)");
  OF_CHECK_ARG(!io->act_src || (io->ld_act >= a.N && io->ld_act % 4 == 0 &&
                                ((uintptr_t)io->act_src & 15) == 0), "conv b16i: act_src");
  OF_CHECK_ARG(!io->act16 || (io->ld_act16 >= a.N && io->ld_act16 % 4 == 0 &&
                              ((uintptr_t)io->act16 & 7) == 0), "conv b16i: act16");
  OF_CHECK_ARG(mode == 1 || !io->col_part, "conv b16i: column sums are a dgrad output");
  const int SH = mode == 0 ? d->h : d->ho, SW = mode == 0 ? d->w : d->wo;
  a.A = static_cast<const float*>(io->a16);
  a.lda = io->lda16;
  a.a_bytes = (int64_t)d->n * SH * SW * io->lda16 * 2;
  a.B = static_cast<const float*>(w16);
  a.b_bytes = (int64_t)a.nb * a.ldb * 2;
  OF_CHECK_ARG(a.a_bytes < INT32_MAX && a.b_bytes < INT32_MAX, "conv b16i: < 2 GiB tensors");
  a.C = io->y, a.ldc = io->ldy;
  a.C16 = static_cast<uint16_t*>(io->y16), a.ldc16 = io->ldy16;
  a.bias = mode == 0 ? bias : nullptr;
  a.bn_g = mode == 0 ? bn_gamma : nullptr;
  a.bn_b = bn_beta, a.bn_m = bn_mean, a.bn_v = bn_var, a.bn_eps = bn_eps;
  a.res = io->aux, a.ldr = io->ldr;
  a.act_src = mode == 1 ? io->act_src : nullptr;
  a.ld_act = io->ld_act;
  a.act16 = mode == 1 ? static_cast<const uint16_t*>(io->act16) : nullptr;
  a.ld_act16 = io->ld_act16;
  a.col_part = mode == 1 ? io->col_part : nullptr;
  a.act = act, a.alpha = alpha;
  a.vec_ep = 1;
  a.abl = g_b16i_abl;
  // the direct epilogue: one output (a bf16 image, or fp32), N and its pitch in whole 16-byte
  // chunks; fwd without residual / BN; dgrad with act' from mask_in or no activation
  const bool one16 = io->y16 && !io->y && a.N % 8 == 0 && io->ldy16 % 8 == 0 &&
                     ((uintptr_t)io->y16 & 15) == 0;
  const bool one32 = io->y && !io->y16 && a.N % 4 == 0 && io->ldy % 4 == 0 &&
                     ((uintptr_t)io->y & 15) == 0;
  const bool direct_ok = (one16 || one32) && (mode == 1 || (!io->aux && !bn_gamma));
  OF_CHECK_ARG(!io->mask_out || (mode == 0 && direct_ok),
               "conv b16i: mask_out needs the forward with one output (N % 8 == 0 for bf16)");
  OF_CHECK_ARG(!io->mask_in || (mode == 1 && direct_ok),
               "conv b16i: mask_in needs the input gradient with one output");
  OF_CHECK_ARG(!io->mask_out || ((uintptr_t)io->mask_out & 15) == 0, "conv b16i: mask alignment");
  OF_CHECK_ARG(!io->mask_in || ((uintptr_t)io->mask_in & 15) == 0, "conv b16i: mask alignment");
  a.direct16 = direct_ok && !(a.abl & 1) &&
               (mode == 0 ? g_b16i_direct != 0
                          : io->mask_in != nullptr ||
                                (g_b16i_direct && act == OF_ACT_NONE && !io->act_src && !io->act16));
  OF_CHECK_ARG(!io->mask_out || a.direct16, "conv b16i: mask_out with the direct epilogue off");
  a.mask_out = static_cast<uint4*>(io->mask_out);
  a.mask_in = static_cast<const uint4*>(io->mask_in);
  hipStream_t s = as_stream(stream);
  const double flops = 2.0 * d->n * d->ho * d->wo * (double)d->cout * 9 * d->cin;
  const int bn = b16i_bn(a.N);
  const int cfg = bn == 128 ? 0 : bn == 96 ? 1 : bn == 64 ? 2 : 3;
  const dim3 grid(a.tiles_total), block(512);
  if (timing_on()) timing_begin(s);
  // persistent form (key 24): one workgroup per CU over contiguous tile ranges, the next
  // tile's first loads in flight during the epilogue; direct epilogue only
  // (key 24 = 2: a grid of 8 workgroups whatever the size: the tests' multi-tile walks)
  const int pg = g_b16i_persist == 2 ? 8 : device_cus();
  const bool persist = g_b16i_persist && a.direct16 && a.splits == 1 && a.tiles_total > pg;
  const dim3 pgrid(persist ? pg : 1);
#define B16I_LAUNCH(MODE, P, G)                                                                  \
  if (cfg == 0) hipLaunchKernelGGL((conv_halo_b16<128, 4, 2, MODE, BI_TH, BI_TW, P>), G, block, 0, s, a); \
  else if (cfg == 1) hipLaunchKernelGGL((conv_halo_b16<96, 4, 2, MODE, BI_TH, BI_TW, P>), G, block, 0, s, a); \
  else if (cfg == 2) hipLaunchKernelGGL((conv_halo_b16<64, 8, 1, MODE, BI_TH, BI_TW, P>), G, block, 0, s, a); \
  else hipLaunchKernelGGL((conv_halo_b16<32, 8, 1, MODE, BI_TH, BI_TW, P>), G, block, 0, s, a);
  if (mode == 0) {
    if (persist) { B16I_LAUNCH(MODE_FWD, true, pgrid) } else { B16I_LAUNCH(MODE_FWD, false, grid) }
  } else {
    if (persist) { B16I_LAUNCH(MODE_DGRAD, true, pgrid) } else { B16I_LAUNCH(MODE_DGRAD, false, grid) }
  }
#undef B16I_LAUNCH
  if (timing_on()) timing_end(s, 288 + 8 * mode + cfg, flops);   // bench.py kind_parts
  return check_launch("conv_halo_b16");
}

// ---- weight gradient from bf16 images (conv_wgrad_b16i) ------------------------------------
struct WgB16iPlan {
  int wci, wco;          // waves
  GemmArgs a;
};

static void wgrad_b16i_plan(const of_conv_desc* d, WgB16iPlan& P) {
  GemmArgs& a = P.a;
  a = GemmArgs{};
  if (d->cout > 64) P.wci = 2, P.wco = 4;
  else if (d->cout > 32) P.wci = 4, P.wco = 2;
  else P.wci = 4, P.wco = 1;
  const int cib = 32 * P.wci, cob = 32 * P.wco;
  a.n = d->n, a.h = d->h, a.w = d->w, a.ho = d->ho, a.wo = d->wo;
  a.kh = 3, a.kw = 3, a.stride = 1, a.pt = d->pad_top, a.pl = d->pad_left, a.dt = 1;
  a.kc = d->cin_p;
  a.M = d->cin;                           // slab rows per tap
  a.N = d->cout;
  a.nb = d->cout;
  a.n_tiles = (int)cdiv(d->cout, cob);
  a.tiles_total = (int)cdiv(d->cin_p, cib) * a.n_tiles;
  const int64_t T = (int64_t)d->n * cdiv(d->ho, WB_TH) * cdiv(d->wo, WB_TW);
  a.K = (int)T;
  int S = std::max(1, (int)(device_cus() / a.tiles_total));
  S = (int)std::min<int64_t>(S, std::max<int64_t>(1, T / 4));
  a.k_per_split = (int)cdiv(T, S);
  a.splits = (int)cdiv(T, a.k_per_split);
  a.slab_ld = (int)round_up(d->cout, 4);
  a.split_stride = (int64_t)9 * d->cin * a.slab_ld;
}

size_t of_conv2d_wgrad_b16i_workspace(const of_conv_desc* d) {
  if (!d || d->kh != 3 || d->kw != 3 || d->stride != 1) return 0;
  WgB16iPlan P;
  wgrad_b16i_plan(d, P);
  return (size_t)P.a.splits * P.a.split_stride * sizeof(float);
}

int of_conv2d_wgrad_b16i(const of_conv_desc* d, const void* x16, int ldx16, const void* dy16,
                         int lddy16, float* dw, int accumulate, const float* bn_gamma,
                         const float* bn_var, float bn_eps, void* workspace, size_t ws_bytes,
                         void* stream) {
  OF_CHECK_ARG(d && x16 && dy16 && dw && workspace, "conv wgrad b16i: NULL pointer");
  OF_CHECK_ARG(d->kh == 3 && d->kw == 3 && d->stride == 1, "conv wgrad b16i: 3x3 stride 1 only");
  OF_CHECK_ARG(ldx16 % 8 == 0 && ldx16 >= d->cin_p && lddy16 % 8 == 0 && lddy16 >= d->cout,
               "conv wgrad b16i: image strides");
  OF_CHECK_ARG(!bn_gamma || bn_var, "conv wgrad b16i: BN scale needs gamma and var");
  WgB16iPlan P;
  wgrad_b16i_plan(d, P);
  GemmArgs& a = P.a;
  OF_CHECK_ARG(ws_bytes >= (size_t)a.splits * a.split_stride * sizeof(float),
               "conv wgrad b16i: workspace too small");
  a.A = static_cast<const float*>(x16);
  a.lda = ldx16;
  a.a_bytes = (int64_t)d->n * d->h * d->w * ldx16 * 2;
  a.B = static_cast<const float*>(dy16);
  a.ldb = lddy16;
  a.b_bytes = (int64_t)d->n * d->ho * d->wo * lddy16 * 2;
  OF_CHECK_ARG(a.a_bytes < INT32_MAX && a.b_bytes < INT32_MAX, "conv wgrad b16i: < 2 GiB images");
  a.slab = static_cast<float*>(workspace);
  hipStream_t s = as_stream(stream);
  const double flops = 2.0 * d->n * d->ho * d->wo * (double)d->cout * 9 * d->cin;
  const int cfg = P.wco == 4 ? 0 : P.wco == 2 ? 1 : 2;
  if (timing_on()) timing_begin(s);
  const dim3 grid(a.tiles_total * a.splits);
  if (cfg == 0) hipLaunchKernelGGL((conv_wgrad_b16i<2, 4>), grid, dim3(512), 0, s, a);
  else if (cfg == 1) hipLaunchKernelGGL((conv_wgrad_b16i<4, 2>), grid, dim3(512), 0, s, a);
  else hipLaunchKernelGGL((conv_wgrad_b16i<4, 1>), grid, dim3(256), 0, s, a);
  if (timing_on()) timing_end(s, 304 + cfg, flops);     // (the kernel, not the reduce)
  int st = check_launch("conv_wgrad_b16i");
  if (st) return st;
  const int rows = 9 * d->cin;
  const int64_t items = (int64_t)rows * cdiv(d->cout, 4);
  hipLaunchKernelGGL(b16i_wgrad_reduce, dim3((unsigned)cdiv(items, 256)), dim3(256), 0, s, a.slab,
                     a.splits, a.split_stride, rows, a.slab_ld, d->cout, dw, accumulate, bn_gamma,
                     bn_var, bn_eps);
  return check_launch("b16i_wgrad_reduce");
}

// out[n] (+)= sum over rows of part[rows][n] in a fixed order (the bias gradient from the dgrad
// kernels' per-tile column sums): 8 row groups x 32 columns per workgroup, rows strided by 8,
// the 8 group sums added in order.
// out[col] (+)= sum over rows of part[row][col]: one workgroup per column quad, 256 threads
// over the rows (thread t sums rows t, t + 256, ... with 8 loads in flight), then a fixed-order
// tree over the threads -- deterministic.  (One thread per column walking all rows was
// latency-bound: 0.3 ms for 3072 x 128.)
__global__ __launch_bounds__(256) void col_part_reduce_kernel(const float* __restrict__ part,
                                                              int rows, int n,
                                                              float* __restrict__ out, int acc) {
  __shared__ float4 red[256];
  const int t = threadIdx.x, col = 4 * blockIdx.x;
  const bool vec = (n & 3) == 0;
  auto ld = [&](int r) {
    const float* p = part + (int64_t)r * n + col;
    if (vec) return *reinterpret_cast<const float4*>(p);
    return make_float4(p[0], col + 1 < n ? p[1] : 0.f, col + 2 < n ? p[2] : 0.f,
                       col + 3 < n ? p[3] : 0.f);
  };
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  int r = t;
  for (; r + 7 * 256 < rows; r += 8 * 256) {
    float4 u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = ld(r + 256 * k);
#pragma unroll
    for (int k = 0; k < 8; ++k) add4(s, u[k]);
  }
  for (; r < rows; r += 256) add4(s, ld(r));
  red[t] = s;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) add4(red[t], red[t + w]);
    __syncthreads();
  }
  if (t < 4 && col + t < n) {
    const float v[4] = {red[0].x, red[0].y, red[0].z, red[0].w};
    out[col + t] = acc ? out[col + t] + v[t] : v[t];
  }
}

int of_col_part_reduce(const float* part, int rows, int n, float* out, int accumulate,
                       void* stream) {
  OF_CHECK_ARG(part && out && rows > 0 && n > 0, "col_part_reduce: args");
  hipLaunchKernelGGL(col_part_reduce_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0,
                     as_stream(stream), part, rows, n, out, accumulate);
  return check_launch("col_part_reduce");
}

}  // extern "C"

}  // namespace oflow
