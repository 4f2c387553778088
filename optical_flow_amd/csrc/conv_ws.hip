// bf16 3x3 stride-1 fwd / dgrad halo convolution, warp-specialised (conv_tile_ws).
// Replaces Conv2D / Conv2DBackpropInput of the decoder's 3x3 convs (model.py:104-113) in the
// bf16 configurations (BASELINE configs 3-5); launched from conv_f32.hip's dispatch.
#include "common.h"
#include "conv_dev.h"

namespace oflow {

// ---- bf16 3x3 stride-1 fwd / dgrad, warp-specialised (conv_tile_ws) ----------------------
// The halo kernels above stage their operands from the same waves that issue the MFMAs, so a
// tap step (16-24 MFMAs per wave) exposes the staging latency and the barrier: 20-25 % of the
// bf16 peak.  Here the waves of a workgroup have one job each:
//   - NC = CWM x CWN compute waves, each a WM x WN block (128 x 64 for BN = 128) of
//     v_mfma_f32_16x16x32_bf16 tiles, never touch global memory in the main loop: during tap
//     step q they read step q + 1's A (halo) and B fragments from LDS while step q's MFMAs
//     issue from registers;
//   - 2 halo waves load the next 32-channel chunk's fp32 input halo into registers at the
//     chunk's first tap, round it to bf16 and store it into the other of two halo buffers at
//     tap WS_HALO_T (swizzled 64-byte rows, the tile_x3_body layout);
//   - 2 B waves keep a ring of WS_NB per-tap B buffers filled by LDS DMA (buffer_load ... lds)
//     WS_PF steps ahead and retire them with counted vmcnt -- no VGPR-destination load shares
//     their counter, so the count is exact.
// One raw s_barrier per tap step, after each wave's own LDS traffic (lgkmcnt) or its own DMA
// (vmcnt) for the step after next has retired.  Buffer hazards:
//   - B of step q is read during step q - 1 (step 0's during step 0); DMA(q + WS_PF) in step q
//     overwrites the buffer of step q - 1, and the B waves retire DMA(q + 2) before barrier
//     q + 1 (the compute waves read it in q + 1);
//   - halo(c + 1) is written during chunk c, step WS_HALO_T < 8, into the buffer last read in
//     chunk c - 1; the compute waves first read it in step (c, 8).
#ifdef WS_STAMP
__device__ uint64_t g_ws_stamps[4 * 8 * 128];
#endif
#ifdef WS_EP_SYNCTHREADS
#define WS_EP_SYNC() __syncthreads()
#else
#define WS_EP_SYNC() ws_sync()
#endif
// B ring of WS_NB buffers filled WS_PF = WS_NB - 1 steps ahead: DMA(q + 3) in step q lands
// in the buffer of step q - 1, read during step q - 2 (the compute waves read a step's B one
// step early, and step 0's in step 0 itself -- so a distance of WS_NB would race with it).
constexpr int WS_NB = 4;
constexpr int WS_PF = WS_NB - 1;
static_assert(WS_PF == 3, "the B waves' vmcnt counts assume a prefetch distance of 3");
constexpr int WS_HG = 4;        // halo slot groups (loads at taps 0..3)
constexpr int WS_HALO_T = 4;    // tap step of the first group's store (stores at taps 4..7)

template <int N>
__device__ __forceinline__ void ws_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void ws_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int BN, int TH, int CWM, int CWN, int MODE>
__global__ __launch_bounds__(64 * (CWM * CWN + 4), 1) void conv_tile_ws(GemmArgs a) {
  constexpr int KS = 3, BM = TH * TF_W, HH = TH + KS - 1, HW = TF_W + KS - 1, HP = HH * HW;
  constexpr int NC = CWM * CWN;
  constexpr int WM = BM / CWM, WN = BN / CWN, SM = WM / 16, SN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0 && BN % 32 == 0, "tile");
  // halo pixels 80 bytes apart (5 x 16-byte slots): a fragment read's 16 consecutive pixels
  // fall on 16 distinct bank slots, and a tap is an immediate offset from the tap-0 address
  constexpr int HPU = 5;
  constexpr int AH_U4 = 2 * HP * HPU, BS_U4 = WS_NB * BN * 4, LDS_U4 = AH_U4 + BS_U4;
#ifdef WS_STAMP
  // probe builds (tools/ws_probe.py): per-wave s_memtime stamps in LDS past the images, copied to
  // a.slab (uint64 [block < 4][wave][128]) at the end; never in the shipped library
  __shared__ uint4 smem[LDS_U4 + 8 * 128 / 2];
  uint64_t* stl = reinterpret_cast<uint64_t*>(smem + LDS_U4) + (threadIdx.x >> 6) * 128;
#define WS_ST(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    if ((threadIdx.x & 63) == 0 && (k) < 128) stl[(k)] = t_; } while (0)
#define WS_ST_OUT() do { if (blockIdx.x < 4 && (threadIdx.x & 63) == 0) { \
    uint64_t* g_ = g_ws_stamps + (blockIdx.x * 8 + (threadIdx.x >> 6)) * 128; \
    for (int k_ = 0; k_ < 128; ++k_) g_[k_] = stl[k_]; } } while (0)
#else
  __shared__ uint4 smem[LDS_U4];
#define WS_ST(k) do {} while (0)
#define WS_ST_OUT() do {} while (0)
#endif
  uint4* Ah = smem;                      // [2][halo pixel][4 octets + pad]
  uint4* Bs = smem + AH_U4;              // [WS_NB][BN rows][4 octets]

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
  const int nch = max(0, min(a.K, c_begin + a.k_per_split) - c_begin);
  const int steps = nch * 9;

  f32x4 acc[SM][SN];      // (compute waves; zero in the staging waves, which only store)
#pragma unroll
  for (int i = 0; i < SM; ++i)
#pragma unroll
    for (int j = 0; j < SN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
  const int wm0 = (wave / CWN) * WM;
  const int wn0 = (wave % CWN) * WN;
  const int l16 = lane & 15, lq = lane >> 4;
  if (wave >= NC + 2) {
    // ---- B waves: the per-tap B ring by LDS DMA -------------------------------------------
    const rsrc_t rb_src = make_rsrc(a.B, a.b_bytes);
    constexpr int BDI = BN / 16, BDW = BDI / 2;       // wave-instructions per step, per wave
    const int bw = wave - NC - 2;
    uint32_t bd_off[BDW];
    int bd_lds[BDW];
#pragma unroll
    for (int k = 0; k < BDW; ++k) {
      const int g = bw + 2 * k;
      const int n = g * 16 + (lane >> 2), o = (lane & 3) ^ x3_sw(lane >> 2);
      bd_off[k] = n0 + n < a.nb ? (uint32_t)(((int64_t)(n0 + n) * a.ldb + 8 * o) * 2) : kOOB;
      bd_lds[k] = g * 16 * 4;
    }
    auto dma = [&](int q) {
      const int c = c_begin + q / 9, t = q % 9;
      const int so = (t * a.kc + 32 * c) * 2;
      uint4* dst = Bs + (q & (WS_NB - 1)) * BN * 4;
#pragma unroll
      for (int k = 0; k < BDW; ++k) dma16_to_lds(rb_src, dst + bd_lds[k], bd_off[k], so);
    };
    if (steps > 0) {
      const int pro = min(WS_PF, steps);
      for (int p = 0; p < pro; ++p) dma(p);
      if (pro == 3) ws_vmcnt<BDW>();                   // DMA(0), DMA(1) landed
      else ws_vmcnt<0>();
      ws_sync();
      WS_ST(0);
      for (int q = 0; q < steps; ++q) {
        if (q + WS_PF < steps) dma(q + WS_PF);
        WS_ST(3 * q + 1);
        if (q + 3 < steps) ws_vmcnt<BDW>();            // DMA(q + 2) landed, DMA(q + 3) may fly
        else ws_vmcnt<0>();
        WS_ST(3 * q + 2);
        ws_sync();
        WS_ST(3 * q + 3);
      }
    }
  } else if (wave >= NC) {
    // ---- halo waves: fp32 halo -> bf16, two buffers ---------------------------------------
    const rsrc_t ra_src = make_rsrc(a.A, a.a_bytes);
    constexpr int HQ = HP * 8, HSW = (HQ + 127) / 128;
    static_assert(HSW <= 64, "halo slots");
    const int ht = tid - 64 * NC;
    const int hcq = ht & 7;
    int h_off[HSW];
    uint64_t h_ok = 0;
#pragma unroll
    for (int j = 0; j < HSW; ++j) {
      const int q = ht + 128 * j;
      const int hp = q >> 3;
      const int sy = hy0 + hp / HW, sx = hx0 + hp % HW;
      const bool ok = q < HQ && (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW;
      h_off[j] = ok ? (((b * SH + sy) * SW + sx) * a.lda + 4 * hcq) * 4 : 0;
      h_ok |= (ok ? 1ull : 0ull) << j;
    }
    float4 hv[HSW];
    // slot group g (of WS_HG) is loaded at tap g and stored at tap WS_HALO_T + g: the issue of
    // 20-40 loads, and of their LDS stores after the wait, spread over the steps instead of
    // holding one barrier each (a single group measured ~1000 cycles at both points)
    constexpr int HGS = (HSW + WS_HG - 1) / WS_HG;
    auto load_halo = [&](int c, int g) {
      const bool cok = 32 * c + 4 * hcq < a.kc;
#pragma unroll
      for (int j = 0; j < HSW; ++j)
        if (j / HGS == g)
          hv[j] = bload4(ra_src, cok && ((h_ok >> j) & 1) ? (uint32_t)(h_off[j] + 128 * c) : kOOB);
    };
    auto store_halo = [&](int buf, int g) {
      char* base = reinterpret_cast<char*>(Ah + buf * HP * HPU);
#pragma unroll
      for (int j = 0; j < HSW; ++j) {
        if (g >= 0 && j / HGS != g) continue;
        const int q = ht + 128 * j;
        if (HQ % 128 == 0 || j < HSW - 1 || q < HQ) {
          const int hp = q >> 3;
          const int off = hp * (HPU * 16) + 8 * (q & 7);
          *reinterpret_cast<uint2*>(base + off) = pack_bf16x4(hv[j]);
        }
      }
    };
    if (steps > 0) {
#pragma unroll
      for (int g = 0; g < WS_HG; ++g) load_halo(c_begin, g);
      store_halo(0, -1);
      ws_sync();
      WS_ST(0);
      for (int cc = 0; cc < nch; ++cc) {
        const bool more_c = cc + 1 < nch;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          if (t < WS_HG && more_c) load_halo(c_begin + cc + 1, t);
          WS_ST(3 * (9 * cc + t) + 1);
          if (t >= WS_HALO_T && t < WS_HALO_T + WS_HG && more_c) store_halo((cc + 1) & 1, t - WS_HALO_T);
          WS_ST(3 * (9 * cc + t) + 2);
          ws_sync();
          WS_ST(3 * (9 * cc + t) + 3);
        }
      }
    }
  } else {
    // ---- compute waves ------------------------------------------------------------------
  int a_hp16[SM];
#pragma unroll
  for (int i = 0; i < SM; ++i) {
    const int m = wm0 + 16 * i + l16;
    const int ty = m / TF_W, tx = m % TF_W;
    a_hp16[i] = MODE == MODE_FWD ? ty * HW + tx : (ty + KS - 1) * HW + tx + KS - 1;
  }
  const int b_frag = (wn0 + l16) * 4 + (lq ^ x3_sw(l16));
  // A fragment i / B fragment j of tap t from halo buffer ah / B buffer bs
  auto afrag = [&](const uint4* ah, int t, int i) {
    const int r = t / KS, s = t % KS;
    const int dh = MODE == MODE_FWD ? r * HW + s : -(r * HW + s);
    return __builtin_bit_cast(bf16x8, ah[(a_hp16[i] + dh) * HPU + lq]);
  };
  auto bfrag = [&](const uint4* bs, int j) { return __builtin_bit_cast(bf16x8, bs[64 * j + b_frag]); };
  if (steps > 0) {
    ws_sync();
    WS_ST(0);
    bf16x8 av[SM], bv[SN];
#pragma unroll
    for (int i = 0; i < SM; ++i) av[i] = afrag(Ah, 0, i);
#pragma unroll
    for (int j = 0; j < SN; ++j) bv[j] = bfrag(Bs, j);
    for (int cc = 0; cc < nch; ++cc) {
      const uint4* ah = Ah + (cc & 1) * HP * HPU;
      const uint4* ahn = Ah + ((cc + 1) & 1) * HP * HPU;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        // step q's MFMAs from registers; the next step's fragments (always valid LDS, read
        // even past the last step) refill each A row as soon as its MFMAs are issued
        const int q = 9 * cc + t;
        const uint4* bsn = Bs + ((q + 1) & (WS_NB - 1)) * BN * 4;
        const uint4* an = t < 8 ? ah : ahn;
        const int tn = t < 8 ? t + 1 : 0;
        bf16x8 bn[SN];
#pragma unroll
        for (int j = 0; j < SN; ++j) bn[j] = bfrag(bsn, j);
#pragma unroll
        for (int i = 0; i < SM; ++i) {
#pragma unroll
          for (int j = 0; j < SN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
          av[i] = afrag(an, tn, i);
        }
        // issue order pinned: the next step's B reads, then per A row its SN MFMAs and the
        // read that refills it (the scheduler otherwise sinks the reads to their first use
        // after the barrier and exposes their latency there)
        __builtin_amdgcn_sched_group_barrier(0x100, SN, 0);
#pragma unroll
        for (int i = 0; i < SM; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, SN, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        WS_ST(3 * q + 2);
        ws_sync();
        WS_ST(3 * q + 3);
#pragma unroll
        for (int j = 0; j < SN; ++j) bv[j] = bn[j];
      }
    }
  }

  }

  // ---- epilogue (16 x 16 C layout: column = lane & 15, rows 4 (lane >> 4) + r); every wave
  // passed the last barrier after its last LDS read / DMA of the loop
  const int64_t img = (int64_t)b * OH * OW;
  WS_ST(126);
#ifdef WS_EP_PERWAVE
  if (a.vec_ep && wave < NC) {
    constexpr int EJ = SN % 2 == 0 ? 2 : 1, EPW = 16 * EJ;
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
          for (int r = 0; r < 4; ++r)
            E[(16 * i + 4 * lq + r) * EPW + 16 * j + l16] = acc[i][jp + j][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int n = n0 + wn0 + 16 * jp + 4 * c4;
#pragma unroll
      for (int q = 0; q < WM / RPI; ++q) {
        const int m = q * RPI + rr;
        const float4 v = *reinterpret_cast<const float4*>(&E[m * EPW + 4 * c4]);
        const int mt = wm0 + m;
        const int oy = oy0 + mt / TF_W, ox = ox0 + mt % TF_W;
        if (oy < OH && ox < OW && n < a.N)
          epilogue_store4<MODE>(a, split, img + (int64_t)oy * OW + ox, n, v);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    return;
  }
  if (a.vec_ep) return;
#endif
  if (a.vec_ep) {
    // All 8 waves store: per pass the compute waves park EJP of their 16-column blocks in an
    // LDS row image (BM rows x W columns), and every wave writes rows of float4 through
    // epilogue_rows4 (a 4-wave store tail measured as long as the main loop).
    constexpr int EJP = SN % 2 == 0 ? 2 : 1, W = CWN * 16 * EJP, PITCH = W + 4;
    constexpr int QPR = W / 4, RPS = 512 / QPR, ITER = BM / RPS, QG = 4;
    static_assert(BM * PITCH <= LDS_U4 * 4 && BM % RPS == 0 && ITER % QG == 0, "epilogue image");
    float* S = reinterpret_cast<float*>(smem);
    const int cq = tid % QPR, rg = tid / QPR;
    const int lc = 4 * cq;                                    // staged column of this quad
#pragma unroll
    for (int p = 0; p < SN / EJP; ++p) {
      if (wave < NC) {
#pragma unroll
        for (int i = 0; i < SM; ++i)
#pragma unroll
          for (int jj = 0; jj < EJP; ++jj)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              S[(wm0 + 16 * i + 4 * lq + r) * PITCH + (wave % CWN) * 16 * EJP + 16 * jj + l16] =
                  acc[i][p * EJP + jj][r];
      }
      WS_EP_SYNC();
      const int n = n0 + (lc / (16 * EJP)) * WN + 16 * (p * EJP + (lc % (16 * EJP)) / 16) + lc % 16;
#pragma unroll
      for (int q0 = 0; q0 < ITER; q0 += QG) {
        float4 v[QG];
        int64_t row[QG];
        unsigned ok = 0;
#pragma unroll
        for (int g = 0; g < QG; ++g) {
          const int m = (q0 + g) * RPS + rg;
          v[g] = *reinterpret_cast<const float4*>(&S[m * PITCH + lc]);
          const int oy = oy0 + m / TF_W, ox = ox0 + m % TF_W;
          row[g] = img + (int64_t)oy * OW + ox;
          ok |= (oy < OH && ox < OW && n < a.N ? 1u : 0u) << g;
        }
        epilogue_rows4<MODE, QG>(a, split, row, ok, n, v);
      }
      WS_EP_SYNC();
    }
    WS_ST(127);
    WS_ST_OUT();
    return;
  }
  if (wave >= NC) return;
#pragma unroll
  for (int j = 0; j < SN; ++j) {
    const int n = n0 + wn0 + 16 * j + l16;
    if (n >= a.N) continue;
    float bias = 0.f, scale = 1.f, shift = 0.f;
    if (a.splits == 1) column_params<MODE>(a, n, bias, scale, shift);
#pragma unroll
    for (int i = 0; i < SM; ++i) {
      EpAux aux[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm0 + 16 * i + 4 * lq + r;
        const int oy = oy0 + m / TF_W, ox = ox0 + m % TF_W;
        aux[r] = a.splits == 1 && oy < OH && ox < OW
                     ? epilogue_aux<MODE>(a, img + (int64_t)oy * OW + ox, n) : EpAux{0.f, 0.f};
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm0 + 16 * i + 4 * lq + r;
        const int oy = oy0 + m / TF_W, ox = ox0 + m % TF_W;
        if (oy >= OH || ox >= OW) continue;
        const int64_t row = img + (int64_t)oy * OW + ox;
        if (a.splits > 1)
          a.slab[(int64_t)split * a.split_stride + row * a.slab_ld + n] = acc[i][j][r];
        else
          epilogue_store<MODE>(a, row, n, acc[i][j][r], bias, scale, shift, aux[r]);
      }
    }
  }
}

// Kernel launch only (timing and the split-K epilogue stay with the caller).
int launch_tile_ws_kernel(const GemmArgs& a, int mode, hipStream_t s) {
  dim3 grid(a.tiles_total * a.splits), block(512);
  const bool b128 = a.N > 96;
  if (mode == MODE_FWD) {
    if (b128) hipLaunchKernelGGL((conv_tile_ws<128, 8, 2, 2, MODE_FWD>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv_tile_ws<96, 8, 2, 2, MODE_FWD>), grid, block, 0, s, a);
  } else {
    if (b128) hipLaunchKernelGGL((conv_tile_ws<128, 8, 2, 2, MODE_DGRAD>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv_tile_ws<96, 8, 2, 2, MODE_DGRAD>), grid, block, 0, s, a);
  }
  return check_launch("conv_tile_ws");
}

}  // namespace oflow

#ifdef WS_STAMP
extern "C" int of_ws_stamps(void* host_dst) {   // probe builds: the stamps of the last launch
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(oflow::g_ws_stamps), sizeof(oflow::g_ws_stamps)) ==
                 hipSuccess ? 0 : -1;
}
#endif
