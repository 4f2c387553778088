// BatchNormalization in training mode (the build's bn_mode flag).
//
// The reference's train.py:51 calls flow_net(batch_imgs) without training=True, so Keras runs
// its BatchNormalization layers (model.py:14 and inside the resnet blocks) in inference mode --
// the default path of this build (conv epilogues with the moving statistics, misc.hip's folded
// backward).  The legacy loop passes training=True (old/train.py:59): then each BN layer
// normalises with the statistics of the batch it is called on and updates its moving
// statistics.  These kernels are that mode:
//
//   of_bn_train_stats : per channel, per row group, mean and biased variance of z (two fixed-order
//                       passes: sum, then sum of squared deviations), invstd = 1/sqrt(var + eps),
//                       and the moving-statistics update of Keras' fused path
//                       (FusedBatchNormV3 with exponential_avg_factor f = 1 - momentum:
//                       moving = (1 - f) moving + f stat, the variance with Bessel's correction),
//                       group by group in order;
//   of_bn_train_apply : y = act(gamma (z - mean) invstd + beta + res);
//   of_bn_train_bwd   : t = dy act'(y); per group st = sum t, stz = sum t zhat;
//                       dz = gamma invstd (t - st / n - zhat stz / n); dgamma += sum_g stz,
//                       dbeta += sum_g st (FusedBatchNormGradV3, is_training = true).
//
// Groups: the Siamese encoder runs image1s and image2s as ONE (2B, ...) batch, but the reference
// calls the encoder once per image (model.py:131-132), so each call normalises with its own
// batch statistics: the rows are `groups` contiguous ranges with separate statistics.
// Every reduction is partial sums per row block + a final pass in block order: bitwise
// reproducible.  HBM-bound elementwise / reduction kernels (not on the benchmarked path).
#include <algorithm>

#include "common.h"

namespace oflow {
namespace {

constexpr int BT_THREADS = 256;
constexpr int BT_ROWS = 1024;       // rows per partial block

struct BtGeo {
  int cq, lanes;                    // channel quads, row lanes per block (256 / cq)
  int64_t rows_g;                   // rows per group
  int nb;                           // blocks per group
};

BtGeo bt_geo(int64_t npix, int c, int groups) {
  BtGeo g;
  g.cq = c / 4;
  g.lanes = BT_THREADS / g.cq;
  g.rows_g = npix / groups;
  g.nb = (int)cdiv(g.rows_g, BT_ROWS);
  return g;
}

__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

__device__ __forceinline__ float act_d(int act, float y) {   // derivative from the output
  return act == OF_ACT_RELU ? (y > 0.f ? 1.f : 0.f) : act == OF_ACT_LEAKY ? (y > 0.f ? 1.f : 0.3f)
                                                                          : 1.f;
}

// MODE 0: sum z.  MODE 1: sum (z - mean)^2.  MODE 2: t = dy act'(y) (-> t_out), sums t and
// t (z - mean) invstd.  One block = BT_ROWS rows of one group; partial[(g nb + blk) * 2 + k][c].
template <int MODE>
__global__ __launch_bounds__(BT_THREADS) void bt_partial(int64_t rows_g, int c, int cq, int lanes,
                                                         int nb, const float* __restrict__ z,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ dy,
                                                         const float* __restrict__ y, int act,
                                                         float* __restrict__ t_out,
                                                         float* __restrict__ part) {
  __shared__ float4 red[2][BT_THREADS];
  const int grp = blockIdx.x / nb, blk = blockIdx.x - grp * nb;
  const int q = threadIdx.x % cq, lane = threadIdx.x / cq;
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
  if (lane < lanes) {
    const int64_t r0 = blk * (int64_t)BT_ROWS, r1 = min(rows_g, r0 + BT_ROWS);
    float4 mu = s0, is = s0;
    if (MODE >= 1) mu = *reinterpret_cast<const float4*>(mean + grp * c + 4 * q);
    if (MODE == 2) is = *reinterpret_cast<const float4*>(invstd + grp * c + 4 * q);
    for (int64_t r = r0 + lane; r < r1; r += lanes) {
      const int64_t off = (grp * rows_g + r) * c + 4 * q;
      const float4 v = *reinterpret_cast<const float4*>(z + off);
      if (MODE == 0) {
        add4(s0, v);
      } else if (MODE == 1) {
        const float dx = v.x - mu.x, dyy = v.y - mu.y, dzz = v.z - mu.z, dw = v.w - mu.w;
        add4(s0, make_float4(dx * dx, dyy * dyy, dzz * dzz, dw * dw));
      } else {
        const float4 g = *reinterpret_cast<const float4*>(dy + off);
        const float4 yy = *reinterpret_cast<const float4*>(y + off);
        const float4 t = make_float4(g.x * act_d(act, yy.x), g.y * act_d(act, yy.y),
                                     g.z * act_d(act, yy.z), g.w * act_d(act, yy.w));
        if (t_out) *reinterpret_cast<float4*>(t_out + off) = t;
        add4(s0, t);
        add4(s1, make_float4(t.x * ((v.x - mu.x) * is.x), t.y * ((v.y - mu.y) * is.y),
                             t.z * ((v.z - mu.z) * is.z), t.w * ((v.w - mu.w) * is.w)));
      }
    }
  }
  red[0][threadIdx.x] = s0;
  red[1][threadIdx.x] = s1;
  __syncthreads();
  if (lane != 0) return;
  for (int l = 1; l < lanes; ++l) {            // fixed order over the row lanes
    add4(s0, red[0][l * cq + q]);
    add4(s1, red[1][l * cq + q]);
  }
  float* dst = part + (int64_t)blockIdx.x * 2 * c + 4 * q;
  *reinterpret_cast<float4*>(dst) = s0;
  *reinterpret_cast<float4*>(dst + c) = s1;
}

// One thread per (group, channel): the blocks' partials of that group in block order.
__global__ void bt_sum(const float* __restrict__ part, int nb, int c, int groups,
                       float* __restrict__ s0, float* __restrict__ s1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= groups * c) return;
  const int grp = i / c, ch = i - grp * c;
  float a = 0.f, b = 0.f;
  for (int k = 0; k < nb; ++k) {
    const float* p = part + ((int64_t)(grp * nb + k) * 2) * c + ch;
    a += p[0];
    b += p[c];
  }
  s0[i] = a;
  if (s1) s1[i] = b;
}

__global__ void bt_mean(const float* __restrict__ sum, int n, int64_t rows_g,
                        float* __restrict__ mean) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) mean[i] = sum[i] / (float)rows_g;
}

// invstd from the sum of squared deviations; moving statistics group by group (each group is
// one encoder call of the reference, in call order).
__global__ void bt_var(const float* __restrict__ ssq, const float* __restrict__ mean, int c,
                       int groups, int64_t rows_g, float eps, float momentum,
                       float* __restrict__ invstd, float* __restrict__ moving_mean,
                       float* __restrict__ moving_var) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const float f = 1.f - momentum;
  const float bessel = rows_g > 1 ? (float)rows_g / (float)(rows_g - 1) : 1.f;
  float mm = moving_mean ? moving_mean[ch] : 0.f, mv = moving_var ? moving_var[ch] : 0.f;
  for (int g = 0; g < groups; ++g) {
    const float var = ssq[g * c + ch] / (float)rows_g;
    invstd[g * c + ch] = 1.f / sqrtf(var + eps);
    mm = (1.f - f) * mm + f * mean[g * c + ch];
    mv = (1.f - f) * mv + f * (var * bessel);
  }
  if (moving_mean) moving_mean[ch] = mm;
  if (moving_var) moving_var[ch] = mv;
}

__global__ void bt_apply(int64_t total4, int c, int64_t rows_g, const float* __restrict__ z,
                         const float* __restrict__ mean, const float* __restrict__ invstd,
                         const float* __restrict__ gamma, const float* __restrict__ beta,
                         const float* __restrict__ res, int act, float* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = 4 * i;
    const int64_t row = e / c;
    const int ch = (int)(e - row * c);
    const int grp = (int)(row / rows_g);
    const float4 v = *reinterpret_cast<const float4*>(z + e);
    const float vv[4] = {v.x, v.y, v.z, v.w};
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
    if (res) r = *reinterpret_cast<const float4*>(res + e);
    const float rr[4] = {r.x, r.y, r.z, r.w};
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cc = ch + k;
      float u = (vv[k] - mean[grp * c + cc]) * invstd[grp * c + cc] * gamma[cc] + beta[cc] + rr[k];
      if (act == OF_ACT_RELU) u = fmaxf(u, 0.f);
      else if (act == OF_ACT_LEAKY) u = u > 0.f ? u : 0.3f * u;
      o[k] = u;
    }
    *reinterpret_cast<float4*>(y + e) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

__global__ void bt_bwd_apply(int64_t total4, int c, int64_t rows_g, const float* __restrict__ t,
                             const float* __restrict__ z, const float* __restrict__ mean,
                             const float* __restrict__ invstd, const float* __restrict__ gamma,
                             const float* __restrict__ st, const float* __restrict__ stz,
                             float* __restrict__ dz) {
  const float inv_n = 1.f / (float)rows_g;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = 4 * i;
    const int64_t row = e / c;
    const int ch = (int)(e - row * c);
    const int grp = (int)(row / rows_g);
    const float4 tv = *reinterpret_cast<const float4*>(t + e);
    const float4 zv = *reinterpret_cast<const float4*>(z + e);
    const float ta[4] = {tv.x, tv.y, tv.z, tv.w}, za[4] = {zv.x, zv.y, zv.z, zv.w};
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int gc = grp * c + ch + k;
      const float is = invstd[gc];
      const float zh = (za[k] - mean[gc]) * is;
      o[k] = gamma[ch + k] * is * (ta[k] - st[gc] * inv_n - zh * (stz[gc] * inv_n));
    }
    *reinterpret_cast<float4*>(dz + e) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

__global__ void bt_param_grads(const float* __restrict__ st, const float* __restrict__ stz,
                               int c, int groups, float* __restrict__ dgamma,
                               float* __restrict__ dbeta, int accum) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  float a = 0.f, b = 0.f;
  for (int g = 0; g < groups; ++g) {
    a += stz[g * c + ch];
    b += st[g * c + ch];
  }
  if (dgamma) dgamma[ch] = accum ? dgamma[ch] + a : a;
  if (dbeta) dbeta[ch] = accum ? dbeta[ch] + b : b;
}

int bt_check(int64_t npix, int c, int groups, const char* what) {
  OF_CHECK_ARG(npix > 0 && groups >= 1 && npix % groups == 0,
               std::string(what) + ": npix must be a positive multiple of groups");
  OF_CHECK_ARG(c > 0 && c % 4 == 0 && c / 4 <= BT_THREADS,
               std::string(what) + ": c must be a multiple of 4, at most 1024");
  return OF_OK;
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

dim3 ew_grid(int64_t total4) {
  return dim3((unsigned)std::min<int64_t>(cdiv(total4, 256), 8 * device_cus()));
}

}  // namespace
}  // namespace oflow

using namespace oflow;

extern "C" {

size_t of_bn_train_workspace(int64_t npix, int c, int groups) {
  if (npix <= 0 || groups < 1 || c <= 0) return 0;
  const BtGeo g = bt_geo(npix, c, groups);
  // partials (groups * nb * 2 * c) + four (groups * c) vectors
  return ((size_t)groups * g.nb * 2 * c + 4 * (size_t)groups * c) * sizeof(float);
}

int of_bn_train_stats(int64_t npix, int c, int groups, const float* z, float eps, float momentum,
                      float* mean, float* invstd, float* moving_mean, float* moving_var,
                      void* workspace, void* stream) {
  int st = bt_check(npix, c, groups, "bn_train_stats");
  if (st) return st;
  OF_CHECK_ARG(z && mean && invstd && workspace, "bn_train_stats: NULL pointer");
  OF_CHECK_ARG(al16(z) && al16(mean), "bn_train_stats: 16-byte alignment");
  hipStream_t s = as_stream(stream);
  const BtGeo g = bt_geo(npix, c, groups);
  float* part = static_cast<float*>(workspace);
  float* sum = part + (size_t)groups * g.nb * 2 * c;
  const int n = groups * c;
  hipLaunchKernelGGL(bt_partial<0>, dim3(groups * g.nb), dim3(BT_THREADS), 0, s, g.rows_g, c, g.cq,
                     g.lanes, g.nb, z, nullptr, nullptr, nullptr, nullptr, 0, nullptr, part);
  hipLaunchKernelGGL(bt_sum, dim3(cdiv(n, 256)), dim3(256), 0, s, part, g.nb, c, groups, sum,
                     nullptr);
  hipLaunchKernelGGL(bt_mean, dim3(cdiv(n, 256)), dim3(256), 0, s, sum, n, g.rows_g, mean);
  hipLaunchKernelGGL(bt_partial<1>, dim3(groups * g.nb), dim3(BT_THREADS), 0, s, g.rows_g, c, g.cq,
                     g.lanes, g.nb, z, mean, nullptr, nullptr, nullptr, 0, nullptr, part);
  hipLaunchKernelGGL(bt_sum, dim3(cdiv(n, 256)), dim3(256), 0, s, part, g.nb, c, groups, sum,
                     nullptr);
  hipLaunchKernelGGL(bt_var, dim3(cdiv(c, 256)), dim3(256), 0, s, sum, mean, c, groups, g.rows_g,
                     eps, momentum, invstd, moving_mean, moving_var);
  return check_launch("bn_train_stats");
}

int of_bn_train_apply(int64_t npix, int c, int groups, const float* z, const float* mean,
                      const float* invstd, const float* gamma, const float* beta,
                      const float* res, int act, float* y, void* stream) {
  int st = bt_check(npix, c, groups, "bn_train_apply");
  if (st) return st;
  OF_CHECK_ARG(z && mean && invstd && gamma && beta && y, "bn_train_apply: NULL pointer");
  OF_CHECK_ARG(al16(z) && al16(y) && al16(res), "bn_train_apply: 16-byte alignment");
  OF_CHECK_ARG(act == OF_ACT_NONE || act == OF_ACT_RELU || act == OF_ACT_LEAKY,
               "bn_train_apply: act");
  const int64_t total4 = npix * c / 4;
  hipLaunchKernelGGL(bt_apply, ew_grid(total4), dim3(256), 0, as_stream(stream), total4, c,
                     npix / groups, z, mean, invstd, gamma, beta, res, act, y);
  return check_launch("bn_train_apply");
}

int of_bn_train_bwd(int64_t npix, int c, int groups, int act, const float* dy, const float* y,
                    const float* z, const float* mean, const float* invstd, const float* gamma,
                    float* dz, float* t_out, float* dgamma, float* dbeta, int accumulate,
                    void* workspace, void* stream) {
  int st = bt_check(npix, c, groups, "bn_train_bwd");
  if (st) return st;
  OF_CHECK_ARG(dy && y && z && mean && invstd && gamma && dz && workspace,
               "bn_train_bwd: NULL pointer");
  OF_CHECK_ARG(al16(dy) && al16(y) && al16(z) && al16(dz) && al16(t_out) && al16(mean) &&
                   al16(invstd),
               "bn_train_bwd: 16-byte alignment");
  OF_CHECK_ARG(act == OF_ACT_NONE || act == OF_ACT_RELU || act == OF_ACT_LEAKY,
               "bn_train_bwd: act");
  hipStream_t s = as_stream(stream);
  const BtGeo g = bt_geo(npix, c, groups);
  float* part = static_cast<float*>(workspace);
  float* sums = part + (size_t)groups * g.nb * 2 * c;
  float* s_t = sums + 2 * (size_t)groups * c;
  float* s_tz = s_t + (size_t)groups * c;
  const int n = groups * c;
  // t = dy act'(y): kept in dz's buffer when the caller wants no t (read back by the apply)
  float* t = t_out ? t_out : dz;
  hipLaunchKernelGGL(bt_partial<2>, dim3(groups * g.nb), dim3(BT_THREADS), 0, s, g.rows_g, c, g.cq,
                     g.lanes, g.nb, z, mean, invstd, dy, y, act, t, part);
  hipLaunchKernelGGL(bt_sum, dim3(cdiv(n, 256)), dim3(256), 0, s, part, g.nb, c, groups, s_t,
                     s_tz);
  const int64_t total4 = npix * c / 4;
  hipLaunchKernelGGL(bt_bwd_apply, ew_grid(total4), dim3(256), 0, s, total4, c, g.rows_g, t, z,
                     mean, invstd, gamma, s_t, s_tz, dz);
  hipLaunchKernelGGL(bt_param_grads, dim3(cdiv(c, 256)), dim3(256), 0, s, s_t, s_tz, c, groups,
                     dgamma, dbeta, accumulate);
  return check_launch("bn_train_bwd");
}

}  // extern "C"
