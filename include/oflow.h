/*
 * oflow.h -- C ABI of the MI355X-native optical-flow training hot path (liboflow.so).
 *
 * The reference (xianlopez/optical_flow) has no FFI: its hot path is Python functions on
 * TensorFlow tensors.  Each entry point below replaces the TF kernels behind one reference
 * call site (cited per function), so the Python mirror in optical_flow_amd/ can keep the
 * reference's function names and signatures (see INTEGRATION.md for the ctypes binding).
 *
 * Conventions
 *   - Activations are NHWC; "ld" arguments are pixel strides in elements (>= channels),
 *     so producers can write straight into a channel slice of a wider buffer (virtual
 *     concat, model.py:100-102).
 *   - Kernels are HWIO (Keras layout).  Conv weights are re-packed once per step by
 *     of_conv_pack_weights() into the GEMM-ready layouts the conv kernels read.
 *   - Every launch is stream-ordered on `stream` (a hipStream_t passed as void*); no entry
 *     point synchronises, allocates, or frees device memory, so the calls are graph-capturable.
 *     The caller owns every buffer; scratch comes from a caller-provided workspace whose size
 *     is returned by a *_workspace() query.
 *   - Return value: OF_OK (0) or an error code; of_last_error() gives a thread-local message.
 *     No C++ exception crosses the ABI.
 *   - dtype: fp32 everywhere in ABI v1 (the reference computes in fp32).
 */
#ifndef OFLOW_H
#define OFLOW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OF_ABI_VERSION 1

enum { OF_OK = 0, OF_EINVAL = 1, OF_EHIP = 2, OF_EUNSUPPORTED = 3, OF_ETIMEOUT = 4 };
enum { OF_ACT_NONE = 0, OF_ACT_RELU = 1, OF_ACT_LEAKY = 2 };

/* Convolution geometry.  Replaces layers.Conv2D(padding='same') (model.py:12,104-114 and the
 * resnet submodule's convs), whose TF kernels are Conv2D / Conv2DBackpropInput /
 * Conv2DBackpropFilter. */
typedef struct of_conv_desc {
  int32_t n, h, w;       /* input batch, height, width                                     */
  int32_t cin;           /* logical input channels (the kernel's I dimension)             */
  int32_t cin_p;         /* channels per pixel the kernel reads (>= cin, multiple of 4;
                            channels [cin, cin_p) of the input must hold zeros)            */
  int32_t cout;          /* output channels (the kernel's O dimension)                    */
  int32_t kh, kw, stride;
  int32_t pad_top, pad_left;   /* TF 'same' split, see of_same_pads()                     */
  int32_t ho, wo;        /* output height, width                                           */
} of_conv_desc;

int         of_abi_version(void);
const char* of_last_error(void);
/* Keras/TF padding='same' split for one spatial dim (P3): out = ceil(n/s),
 * total = max((out-1)*s + k - n, 0), before = total/2, after = total - before. */
int of_same_pads(int n, int k, int s, int* before, int* after, int* out);

/* Packed weight sizes (elements) for of_conv_pack_weights(): fwd = [Kf][Nf], bwd = [Kd][Nd]. */
int64_t of_conv_wfwd_elems(const of_conv_desc* d);
int64_t of_conv_wbwd_elems(const of_conv_desc* d);
/* w_hwio: [kh][kw][cin][cout] fp32 -> w_fwd (GEMM B for the forward) and, if non-NULL,
 * w_bwd (GEMM B for the input-gradient pass: per tap, the (cout x cin) transpose). */
int of_conv_pack_weights(const of_conv_desc* d, const float* w_hwio, float* w_fwd,
                         float* w_bwd, void* stream);

/* Packing every conv of a model in ONE launch (weights change once per optimizer step):
 * build the table once on the host with of_conv_pack_table() into a buffer of
 * of_conv_pack_table_bytes(nconv) bytes, copy it to device memory, then call
 * of_conv_pack_many(dev_table, total_work, stream) per step; total_work is the 64-bit value at
 * byte offset 8 of the table. */
size_t of_conv_pack_table_bytes(int nconv);
int of_conv_pack_table(int nconv, const of_conv_desc* descs, const float* const* w_hwio,
                       float* const* w_fwd, float* const* w_bwd, void* host_table);
int of_conv_pack_many(const void* dev_table, int64_t total_work, void* stream);

/* Forward: z = conv(x, w) + bias;  y = act(BN(z) + residual) with the inference-mode
 * BatchNorm BN(z) = (z - mean) * gamma / sqrt(var + bn_eps) + beta (identity when
 * bn_gamma == NULL); z is also stored when z != NULL (needed for the BN gamma gradient).
 * x: [n][h][w] pixels of ldx elements (cin_p used); y/z: [n][ho][wo] pixels of ldy/ldz;
 * bias and bn_*: [cout] or NULL; residual: NULL or pixels of ldr; act: OF_ACT_*, alpha is
 * the LeakyReLU slope.  Replaces Conv2D + BiasAdd + FusedBatchNorm(inference) + AddV2 +
 * Relu/LeakyRelu. */
size_t of_conv2d_fwd_workspace(const of_conv_desc* d);
int of_conv2d_fwd(const of_conv_desc* d, const float* x, int ldx, const float* w_fwd,
                  const float* bias, const float* bn_gamma, const float* bn_beta,
                  const float* bn_mean, const float* bn_var, float bn_eps,
                  const float* residual, int ldr, int act, float alpha,
                  float* z, int ldz, float* y, int ldy, void* workspace, size_t ws_bytes,
                  void* stream);

/* Workspace (fwd / dgrad): grids with fewer tiles than CUs split K over workgroups into fp32
 * slabs of of_conv2d_{fwd,dgrad}_workspace() bytes; with workspace == NULL (or too small) the
 * call runs unsplit (same result). */

/* Input gradient (Conv2DBackpropInput; for stride 2 this is the transposed convolution, run
 * as four row/column-parity phase groups that each visit only their taps):
 * dx[.., ci] = sum_{tap,co} dy * w, for ci < cin_p, then (fused) multiplied by the
 * activation derivative of act_src (the forward output that fed this conv) when
 * act_src != NULL: relu' = [s>0], leaky' = s>0 ? 1 : alpha.
 * dy: [n][ho][wo] pixels of lddy elements, round_up(cout,4) channels read (pad must be 0). */
size_t of_conv2d_dgrad_workspace(const of_conv_desc* d);
int of_conv2d_dgrad(const of_conv_desc* d, const float* dy, int lddy, const float* w_bwd,
                    const float* act_src, int ld_act, int act, float alpha,
                    float* dx, int lddx, void* workspace, size_t ws_bytes, void* stream);

/* Weight (+ bias) gradient (Conv2DBackpropFilter + BiasAddGrad): dw in HWIO [kh][kw][cin][cout],
 * db [cout] (NULL to skip); accumulate != 0 adds into dw/db (gradient arenas).
 * Deterministic split-K with a slab reduction in `workspace`. */
size_t of_conv2d_wgrad_workspace(const of_conv_desc* d);
int of_conv2d_wgrad(const of_conv_desc* d, const float* x, int ldx, const float* dy, int lddy,
                    float* dw, float* db, int accumulate, void* workspace, size_t ws_bytes,
                    void* stream);

/* bf16 MFMA variants (BASELINE configs 3-5: "bf16 with MFMA direct-conv path"): same
 * geometry, epilogues and error behaviour as of_conv2d_{fwd,dgrad,wgrad}; activations stay
 * fp32 in memory and are rounded to bf16 (RNE) while staged, weights are the bf16 images of
 * of_conv_pack_weights_bf16 (of_conv_w{fwd,bwd}16_elems bf16 elements each), accumulation is
 * fp32.  of_conv_path(d) == 1 marks the narrow (cout <= 4) layers, which stay on the f32
 * VALU kernels in every precision. */
int of_conv_path(const of_conv_desc* d);
int64_t of_conv_wfwd16_elems(const of_conv_desc* d);
int64_t of_conv_wbwd16_elems(const of_conv_desc* d);
int of_conv_pack_weights_bf16(const of_conv_desc* d, const float* w_hwio, void* w16_fwd,
                              void* w16_bwd, void* stream);
/* of_conv_pack_table with a per-conv precision flag (bf16[i] != 0: bf16 images). */
int of_conv_pack_table_ex(int nconv, const of_conv_desc* descs, const float* const* w_hwio,
                          void* const* w_fwd, void* const* w_bwd, const int* bf16,
                          void* host_table);
size_t of_conv2d_fwd_bf16_workspace(const of_conv_desc* d);
int of_conv2d_fwd_bf16(const of_conv_desc* d, const float* x, int ldx, const void* w16_fwd,
                       const float* bias, const float* bn_gamma, const float* bn_beta,
                       const float* bn_mean, const float* bn_var, float bn_eps,
                       const float* residual, int ldr, int act, float alpha, float* z, int ldz,
                       float* y, int ldy, void* workspace, size_t ws_bytes, void* stream);
size_t of_conv2d_wgrad_bf16_workspace(const of_conv_desc* d);
int of_conv2d_wgrad_bf16(const of_conv_desc* d, const float* x, int ldx, const float* dy,
                         int lddy, float* dw, float* db, int accumulate, void* workspace,
                         size_t ws_bytes, void* stream);
/* Input gradient plus an added gradient: dx = dgrad(dy) + add (add may alias dx).  The
 * residual block's two input-gradient branches (conv_a and the shortcut, AddV2 in the
 * resnet block of model.py:18-22) sum in this epilogue instead of a separate add pass.
 * Same workspace as of_conv2d_dgrad; not for Cout <= 4 layers. */
int of_conv2d_dgrad_add(const of_conv_desc* d, const float* dy, int lddy, const float* w_bwd,
                        const float* add, int ld_add, float* dx, int lddx, void* workspace,
                        size_t ws_bytes, void* stream);
int of_conv2d_dgrad_add_bf16(const of_conv_desc* d, const float* dy, int lddy,
                             const void* w16_bwd, const float* add, int ld_add, float* dx,
                             int lddx, void* workspace, size_t ws_bytes, void* stream);
size_t of_conv2d_dgrad_bf16_workspace(const of_conv_desc* d);
int of_conv2d_dgrad_bf16(const of_conv_desc* d, const float* dy, int lddy, const void* w16_bwd,
                         const float* act_src, int ld_act, int act, float alpha, float* dx,
                         int lddx, void* workspace, size_t ws_bytes, void* stream);

/* fp32 3x3 stride-1 fwd / dgrad on bf16 MFMA by an exact three-term operand split
 * (x = hi + mid + lo, 8 significand bits each; six of the nine bf16 products, each exact,
 * accumulated in fp32; the dropped terms are below 2^-23 |a||b|).  Same arguments and
 * epilogues as the bf16 variants; the weights are the three split planes of the bf16 images
 * (3 * of_conv_w{fwd,bwd}16_elems bf16 elements: hi, mid, lo), packed by
 * of_conv_pack_weights_x3 or of_conv_pack_table_ex with flag 2.  Replaces the same
 * Conv2D / Conv2DBackpropInput as of_conv2d_fwd / of_conv2d_dgrad (model.py:104-114, the
 * resnet blocks' 3x3 convs); OF_EINVAL for any other kernel shape or stride. */
int of_conv_pack_weights_x3(const of_conv_desc* d, const float* w_hwio, void* w3_fwd,
                            void* w3_bwd, void* stream);
size_t of_conv2d_fwd_x3_workspace(const of_conv_desc* d);
size_t of_conv2d_dgrad_x3_workspace(const of_conv_desc* d);
int of_conv2d_fwd_x3(const of_conv_desc* d, const float* x, int ldx, const void* w3_fwd,
                     const float* bias, const float* bn_gamma, const float* bn_beta,
                     const float* bn_mean, const float* bn_var, float bn_eps,
                     const float* residual, int ldr, int act, float alpha, float* z, int ldz,
                     float* y, int ldy, void* workspace, size_t ws_bytes, void* stream);
int of_conv2d_dgrad_x3(const of_conv_desc* d, const float* dy, int lddy, const void* w3_bwd,
                       const float* act_src, int ld_act, int act, float alpha, float* dx,
                       int lddx, void* workspace, size_t ws_bytes, void* stream);
int of_conv2d_dgrad_add_x3(const of_conv_desc* d, const float* dy, int lddy,
                           const void* w3_bwd, const float* add, int ld_add, float* dx,
                           int lddx, void* workspace, size_t ws_bytes, void* stream);
/* Weight gradient with the same split (Conv2DBackpropFilter of those layers): 3x3 stride-1
 * layers with Cout in {32, 64, 96} or Cout % 128 == 0 run conv_wgrad_tile_x3, every other layer as
 * of_conv2d_wgrad; arguments and workspace rules as of_conv2d_wgrad. */
size_t of_conv2d_wgrad_x3_workspace(const of_conv_desc* d);
int of_conv2d_wgrad_x3(const of_conv_desc* d, const float* x, int ldx, const float* dy,
                       int lddy, float* dw, float* db, int accumulate, void* workspace,
                       size_t ws_bytes, void* stream);

/* Activation backward: dz = dy * act'(y) over n elements (y = forward output). */
int of_act_bwd(const float* dy, const float* y, int act, float alpha, float* dz, int64_t n,
               void* stream);

/* Per-channel column sums of a [npix][ld] matrix (first c channels): out[c] (+)= sum.
 * Workspace: of_colsum_workspace(npix, c) bytes. */
size_t of_colsum_workspace(int64_t npix, int c);
int of_colsum(const float* x, int64_t npix, int c, int ld, float* out, int accumulate,
              void* workspace, void* stream);

/* Inference BatchNorm + (residual) + activation backward (model.py:14-15, resnet blocks):
 * dt = dy * act'(y) (act: OF_ACT_NONE or OF_ACT_RELU); dres = dt (if dres);
 * dz = dt * gamma*invstd (if dz); dgamma = sum dt*(z-mean)*invstd; dbeta = sum dt;
 * dbias = sum dt * gamma*invstd (each of the three [c] vectors optional; accumulate != 0 adds
 * into them).  With dz == NULL and dres this is of_bn_bwd_reduce from the stored z: the
 * layers whose gamma came near 0 (ops.BNZGuard), where zhat cannot be recovered from y.
 * y, z, dy, dz, dres dense [npix][c]; workspace: of_bn_act_bwd_workspace(npix, c) bytes. */
size_t of_bn_act_bwd_workspace(int64_t npix, int c);
int of_bn_act_bwd(int64_t npix, int c, int act, const float* dy, const float* y,
                  const float* z, const float* gamma, const float* mean, const float* var,
                  float eps, float* dz, float* dres, float* dgamma, float* dbeta, float* dbias,
                  int accumulate, void* workspace, void* stream);
/* The stem's backward in one pass (model.py:12-17: conv1 -> layer1_bn -> ReLU -> out0 and
 * MaxPool2D): dy(out0) = max-pool backward of dyp (first maximum of each 2x2 window of y,
 * strict >) + g (out0's gradient from its other consumer; NULL = none); then the
 * of_bn_act_bwd math with act = ReLU (y = out0 = the max-pool input, z = pre-BN conv output).
 * n, h, w, c: out0's shape (h, w even); dyp: (n, h/2, w/2, c). */
size_t of_maxpool_bn_act_bwd_workspace(int n, int h, int w, int c);
int of_maxpool_bn_act_bwd(int n, int h, int w, int c, const float* dyp, const float* g,
                          const float* y, const float* z, const float* gamma, const float* mean,
                          const float* var, float eps, float* dz, float* dgamma, float* dbeta,
                          float* dbias, int accumulate, void* workspace, void* stream);

/* Max-pool 2x2/2 'valid' (layers.MaxPool2D(), model.py:17) and its gradient (to the first
 * maximum in row-major window order). x: [n][h][w][c] dense. */
int of_maxpool2_fwd(const float* x, int n, int h, int w, int c, float* y, void* stream);
int of_maxpool2_bwd(const float* x, const float* dy, int n, int h, int w, int c, float* dx,
                    void* stream);

/* Cost volume (create_cost_volume, model.py:29-42; P8): out[p][k], k=i*(2d+1)+j =
 * sum_c f1[p][c]*f2[p+(i-d, j-d)][c] with zero padding.  out has ldo >= (2d+1)^2.
 * The channel reduction may be split into slab groups whose partial sums live in the
 * workspace (which shapes split depends on the level's tile count and the device's CU
 * count): always size it with of_corr_fwd_workspace(), which returns 0 when none is needed.
 * Same rule for of_corr_concat_fwd. */
size_t of_corr_fwd_workspace(int n, int h, int w, int c, int max_disp);
int of_corr_fwd(const float* f1, int ld1, const float* f2, int ld2, int n, int h, int w,
                int c, int max_disp, float* out, int ldo, void* workspace, size_t ws_bytes,
                void* stream);
/* Its gradient: df1 = (accumulate ? df1 : 0) + sum_k dcv*f2_shift; df2 likewise. */
int of_corr_bwd(const float* dcv, int lddcv, const float* f1, int ld1, const float* f2,
                int ld2, int n, int h, int w, int c, int max_disp, float* df1, int lddf1,
                int acc1, float* df2, int lddf2, int acc2, void* stream);
/* The flow-module input concat([features1, cost_volume, flow_up]) (model.py:97-102) built in
 * one launch: cat[p] = [f1[p] (c) | cv[p] (49) | flow[p] (2, if flow) | zeros up to cp].
 * f1, f2: dense [n][h][w][c]; flow: dense [n][h][w][2] or NULL. */
int of_corr_concat_fwd(const float* f1, const float* f2, const float* flow, int n, int h, int w,
                       int c, int max_disp, float* cat, int cp, void* workspace,
                       size_t ws_bytes, void* stream);
/* The concat row [f1 | cost volume | flow | 0] of of_corr_concat_fwd written as a bf16 NHWC
 * image with ld16 channels per pixel (>= c + 49 (+ 2), a multiple of 4; channels past the row
 * zero): the only form the bf16 flow head's first conv reads (ops._stack_fwd_img16), so no
 * fp32 row is written and converted (round 4).  Grids that need slab groups (small levels,
 * of_corr_concat_fwd16_ok(n, h, w, c) == 0) are refused. */
int of_corr_concat_fwd16(const float* f1, const float* f2, const float* flow, int n, int h,
                         int w, int c, int max_disp, void* cat16, int ld16, void* stream);
int of_corr_concat_fwd16_ok(int n, int h, int w, int c);
/* The gradient of of_corr_concat_fwd from dcat (row stride cp): df1 = dcat[:, :c] +
 * d(cv)/d(f1); df2 = d(cv)/d(f2) (skipped if NULL); dflow = dcat[:, c+49 : c+51] (skipped if
 * NULL).  All written. */
int of_corr_concat_bwd(const float* dcat, int cp, const float* f1, const float* f2, int n,
                       int h, int w, int c, int max_disp, float* df1, float* df2, float* dflow,
                       void* stream);

/* Bilinear backward warp with the reference index convention (warp_features, model.py:55-73
 * + bilinear_interpolation, transformations.py:85-129; P1, P2):
 * out[b,i,j] = bilinear(inp[b], x = i + flow[b,i,j,0], y = j + flow[b,i,j,1]). */
int of_warp_fwd(const float* inp, int n, int h, int w, int c, const float* flow, float* out,
                void* stream);
/* dinp += scatter (atomics; caller zeroes or accumulates), dflow = d/d(flow) (written). */
int of_warp_bwd(const float* dout, const float* inp, int n, int h, int w, int c,
                const float* flow, float* dinp, float* dflow, void* stream);
/* of_warp_bwd with d(flow) = dflow_add + d(warp)/d(flow): dflow_add (2 channels, row stride
 * ld_add) is the gradient of the same flow through its other consumer -- in flow_module
 * (model.py:93-102) flow_up feeds both warp_features and the concat, and this sums the concat
 * slice in the store instead of a separate add pass (the same fp32 sum). */
int of_warp_bwd_add(const float* dout, const float* inp, int n, int h, int w, int c,
                    const float* flow, float* dinp, float* dflow, const float* dflow_add,
                    int ld_add, void* stream);
/* bilinear_interpolation(input, sampling_points) (transformations.py:85-129): the same sampler
 * with absolute (x, y) points instead of grid + flow. */
int of_bilinear_fwd(const float* inp, int n, int h, int w, int c, const float* pts, float* out,
                    void* stream);
int of_bilinear_bwd(const float* dout, const float* inp, int n, int h, int w, int c,
                    const float* pts, float* dinp, float* dpts, void* stream);
/* Deterministic mode of the three backward entry points above (no atomics in the
 * warp backward; the gradient of the gathers of transformations.py:110-113,128): the float
 * scatter into dinp becomes either a fixed-order gather -- every destination sums its (source
 * pixel, corner) entries in ascending source order, found by a window scan around the source
 * position (relative flows) -- or, for absolute points and flows the window cannot cover, an
 * exact int64 fixed-point sum (scale from max |dout|: each term exact to max|dout| 2^(L-61),
 * 4 n h w <= 2^L; integer adds, so in any order the same).  Bitwise reproducible either way.
 * dinp is WRITTEN (not accumulated; NULL skips it), dflow = d/d(flow) (+ dflow_add with row
 * stride ld_add if non-NULL); absolute != 0: flow holds absolute (x, y) sampling points
 * (of_bilinear_bwd).  Workspace: of_warp_bwd_det_workspace(n, h, w, c) bytes; its int header
 * at byte of_warp_bwd_det_header(n, h, w, c) holds after a call [1] = R = floor(max |flow|) +
 * 2 (the window is mode A when R <= of_set_tuning key 28, else mode B) and at ints 64 (1 + s),
 * s < 32, the hits mode B found (their sum is 4 n h w when its window served). */
size_t of_warp_bwd_det_workspace(int n, int h, int w, int c);
size_t of_warp_bwd_det_header(int n, int h, int w, int c);
int of_warp_bwd_det(const float* dout, const float* inp, int n, int h, int w, int c,
                    const float* flow, int absolute, float* dinp, float* dflow,
                    const float* dflow_add, int ld_add, void* workspace, size_t ws_bytes,
                    void* stream);

/* upscale_flow (model.py:76-77; P6, P7): out = resize_bilinear_x2(in) * scale, half-pixel
 * centres.  in: [n][h][w][c] dense, out: [n][2h][2w] pixels of ldo (channel slice). */
int of_upscale2x_fwd(const float* in, int n, int h, int w, int c, float scale, float* out,
                     int ldo, void* stream);
int of_upscale2x_bwd(const float* dout, int lddo, int n, int h, int w, int c, float scale,
                     float* din, int accumulate, void* stream);
/* of_upscale2x_bwd into din with row stride lddi (the flow head's channel-padded gradient). */
int of_upscale2x_bwd_ld(const float* dout, int lddo, int n, int h, int w, int c, float scale,
                        float* din, int lddi, int accumulate, void* stream);

/* Image pyramid of LossLayer (loss.py:17-18): for s=1..levels, out_s = resize(batch, H/2^s,
 * W/2^s) (half-pixel bilinear, no antialias == mean of 2x2 taps); each out_s dense 6-ch. */
int of_pyramid6(const float* batch, int n, int h, int w, int levels, float* const* outs,
                void* stream);
/* Split (B,H,W,6) pairs into the Siamese encoder batch (2B,H,W,4): image1s, then image2s,
 * channel 3 zero (model.py:122-123, 131-132). */
int of_split_pair(const float* batch, int n, int h, int w, float* out, void* stream);

/* Photometric L1 term of one scale (loss.py:26-28): sum over (b,i,j,c<3) of
 * |img[...,c] - warp(img[...,3:], flow)[...,c]| ; written as per-block partials to
 * `partials` (of_photo_l1_partials(n,h,w) floats), then of_sum_partials reduces. */
int of_photo_l1_partials(int n, int h, int w);
int of_photo_l1_fwd(const float* img6, const float* flow, int n, int h, int w,
                    float* partials, void* stream);
/* d/d(flow) of g * coef * sum|...| (coef = 1/(levels*n*h*w*3) on the host, g = *dloss read
 * on the device, 1 if dloss == NULL); dflow written (ld 2). */
int of_photo_l1_bwd(const float* img6, const float* flow, int n, int h, int w, float coef,
                    const float* dloss, float* dflow, void* stream);
/* of_photo_l1_bwd writing d(flow) with row stride lddf (>= 2). */
int of_photo_l1_bwd_ld(const float* img6, const float* flow, int n, int h, int w, float coef,
                       const float* dloss, float* dflow, int lddf, void* stream);
/* out[0] = sum_i coef_j * partials_j[i] over `count` groups (deterministic). */
/* Every scale of the loss in one launch (levels <= 8; level l at hs[l] x ws[l]): the forward's
 * partials concatenated in level order (sum over l of of_photo_l1_partials(n, hs[l], ws[l])
 * floats; level l's are the ones of_photo_l1_fwd would write), the backward's d(flow) of level
 * l times coefs[l] (* dloss[0] if dloss) at row stride lds[l]. */
int of_photo_l1_fwd_multi(const float* const* img6s, const float* const* flows, int n,
                          const int* hs, const int* ws, int levels, float* partials,
                          void* stream);
int of_photo_l1_bwd_multi(const float* const* img6s, const float* const* flows, int n,
                          const int* hs, const int* ws, int levels, const float* coefs,
                          const float* dloss, float* const* dflows, const int* lds,
                          void* stream);
int of_sum_partials(const float* const* parts, const int* counts, const float* coefs,
                    int ngroups, float* out, void* stream);

/* Keras Adam (train.py:34,56; P13), one launch over a flat parameter arena, g' = g*gscale
 * (gscale folds the 1/world of a data-parallel gradient average):
 * m += (g'-m)(1-b1); v += (g'^2-v)(1-b2); p -= lr_t * m / (sqrt(v) + eps). */
int of_adam_keras(float* p, const float* g, float* m, float* v, int64_t n, float lr_t,
                  float beta1, float beta2, float eps, float gscale, void* stream);
/* The same update with its schedule in device memory, so a captured step (HIP graph) replays
 * correctly: one thread first sets t = ++*iter and sched[1] = sched[0] * sqrt(1-b2^t) /
 * (1-b1^t) (sched[0] = lr, written by the host, e.g. the epoch-15 drop of train.py:69-70),
 * then the arena update reads lr_t = sched[1]. */
int of_adam_keras_dev(float* p, const float* g, float* m, float* v, int64_t n, float* sched,
                      int32_t* iter, float beta1, float beta2, float eps, float gscale,
                      void* stream);

/* Elementwise helpers used by the host glue. */
int of_add_inplace(float* y, const float* x, int64_t n, void* stream);        /* y += x */
int of_copy_strided(const float* src, int lds, float* dst, int ldd, int64_t npix, int c,
                    void* stream);                                             /* per pixel */
int of_fill(float* y, float v, int64_t n, void* stream);
/* Order stream `waiter` after everything enqueued so far on stream `signaller` (same device):
 * a hipEvent created with hipEventDisableSystemFence, so the record / wait pair fences at
 * device scope only (the side-stream forks and joins of the backward; torch's
 * Stream.wait_stream records a default event).  Works inside a stream capture. */
int of_stream_wait(void* waiter, void* signaller);

/* Per-launch timing of the conv kernels (bench instrumentation): when enabled (on = 1), every
 * conv launch records a hipEvent pair on its stream; on = 2 times the next conv launch only
 * (then timing is off again); of_timing_read() returns the count and fills kinds (the kernel
 * family / pass / tile configuration code, bench.py kind_parts), flops and elapsed ms
 * (synchronises the events). */
int of_timing_enable(int on);
/* Kernel-variant switches for A/B measurements: key 1 = fwd/dgrad split-K target workgroups
 * per CU (1-16, default 4), key 2 = minimum 16-deep K chunks per split slice (2-64, default 12),
 * key 3 = the tile kernels' 16-byte (float4-column) epilogue (1, default) or per-element (0),
 * key 4 = the 9-tap split-bf16 weight gradient for Cout % 128 == 0 (1, default), for every
 * Cout (2) or never (0: the 3-tap form), key 5 = its wave shape, 16 MI input x 32 / MI output
 * channels (MI = 1 default, or 2), key 6 = the other shapes' fp32 weight gradient (stem,
 * stride 2, 1x1) on the split-bf16 implicit GEMM (1, default) or the fp32 MFMA GEMM (0),
 * key 7 = the feature-warp backward as a per-tile gather (counting sort of the tile's corner
 * destinations in LDS, one atomic add per touched destination; 1, default) or with LDS
 * aggregation of the clipped border corners only (0), key 8 = the 7x7 stride-2 stem forward
 * (of_conv2d_fwd_x3) on its own split kernel with two 32-channel workgroups per CU (1,
 * default), one 64-channel workgroup (2), or on the generic split implicit GEMM (0), key 9 =
 * the cost-volume kernel forms (of_corr_*): bit 0 the register-blocked persistent forward
 * (default 1), bit 1 the register-blocked backward (default off: measured slower), key 10 =
 * the fp32 / bf16 GEMM weight gradients' split-K target workgroups per CU (1-16, default 4),
 * key 11 = the split weight gradient of Cout-64 layers whose Cin is not a multiple of 64 on
 * 32 x 64 channel blocks (1, default) or on 64 x 64 blocks (0);
 * key 12 = bf16 3x3 stride-1 fwd / dgrad on the single-plane halo kernel conv_tile_b16 (1;
 * timing kinds 192 + 8 mode + cfg), on the warp-specialised conv_tile_ws for N tiles of 128 /
 * 96 (2: fwd and dgrad, 3: fwd only; timing kinds 224 + 8 mode + cfg) or the round-1
 * conv_tile_bf16 (0, default);
 * key 13 = bf16 3x3 stride-1 weight gradient on the single-plane 9-tap kernel
 * conv_wgrad_tile_b16 (1; timing kinds 216 + cfg) or conv_wgrad_tile_bf16 (0, default);
 * key 14 = the stem's fp32 weight gradient (7x7 stride 2, 3 input channels padded to 4, 64
 * outputs) on conv_wgrad_stem_x3 (1, default; timing kind 185) or the fp32 MFMA GEMM (0);
 * key 15 = the bf16 stem (forward and weight gradient) on the one-plane stem kernels
 * conv_stem_x3<32, 1> / conv_wgrad_stem_x3<1> (1, default; timing kinds 186 / 187) or on the
 * bf16 implicit GEMMs (0);
 * key 16 = which bf16 implicit GEMMs (stride-2 convs, 1x1 projections) run on the one-plane
 * split-GEMM forms conv_gemm_x3<..., 1> / conv_wgrad_x3<..., 1> (timing kinds 240 + 8 mode +
 * cfg): bit 0 forward, bit 1 input gradient, bit 2 weight gradient (default 6);
 * key 18 = bf16 3x3 input gradients with N tiles of 128 on the tall 8 x 32 output tiles where
 * the grid allows (1) or on 4 x 32 tiles (0, default);
 * key 9 bit 2 = the fused cost-volume backward corr_bwd_fused when both gradients are wanted
 * (default on: key 9 = 5);
 * key 21 = conv_halo_b16 timing ablations (bit 0: no epilogue loads / stores, bit 1: no main-loop
 * DMAs; RESULTS ARE WRONG, A/B timing only; default 0);
 * key 22 = conv_halo_b16's direct epilogue for forwards with a bf16 image output alone (1,
 * default; the input gradient takes it whenever it is given mask_in);
 * key 23 = the split 3x3 kernels' direct fp32 epilogues, bit 0 forward, bit 1 input
 * gradient (1, default: the input gradient's measured slower; 0 = per-pass transposes);
 * key 24 = conv_halo_b16 persistent over contiguous tile ranges, the next tile's first loads
 * in flight during the epilogue (1; 2: on 8 workgroups, for tests) or one tile per workgroup
 * (0, default: the persistent form measured even);
 * keys 25 / 26 = the K-split cost models' slab-pass term (tenths of a chunk per slice and tile
 * round; default 5) of the fp32 halo-tile kernels and of the split implicit GEMMs;
 * key 27 = fp32 split 3x3 layers whose BN = 128 grid has fewer than this many workgroups run
 * BN = 64 tiles, two workgroups per CU (default 1200, A/B-measured +1.3 % on the bench step;
 * 0 = never);
 * key 28 = of_warp_bwd_det's window gather: mode A (a window of radius R around the
 * transposed position) when R = floor(max |flow|) + 2 <= this, else mode B (default 8; 0 =
 * no window, always the fixed-point path; 1 = always mode B);
 * key 29 = wgrad_reduce lane rule (0 = default, 1-4 = the measured alternatives);
 * key 30 = the split implicit GEMMs (conv_gemm_x3: stride-2 and 1x1 layers) on an LDS-DMA ring
 * with both operands DMA'd: 3 slots, one chunk in flight across each barrier (1), or 2 slots,
 * two workgroups per CU where the LDS allows (2, default); or register-staged A with one chunk
 * in flight (0); bitwise the same results;
 * key 31 = the stem forward (conv_stem_x3) persistent over its tiles with this many workgroups
 * per CU (-1 = default: as many as the LDS holds, 2 fp32 / 3 bf16; 0 = one tile per
 * workgroup); bitwise the same results;
 * key 32 = bf16 input gradients that carry BN partial sums (of_conv2d_dgrad_add_act_bnp) on
 * conv_tile_b16 (1) or declined with OF_EUNSUPPORTED (0, default: the separate pass);
 * key 33 = the fp32 split 9-tap weight gradient keeps at least this many K tiles per slice
 * (default 2; 1 = the round-5 plan);
 * key 34 = of_warp_bwd_det mode A by 4 x 4 destination tiles with LDS-binned sources in a
 * kernel of their own, own_tile, the last row / column and overflowed bins then scanned by
 * own_window (2, default), the tiles inside own_window (1), or the per-destination window scan
 * (0); bitwise the same results;
 * key 35 = that tiled form with its d(flow) loads issued first (1) or after the gather (0,
 * default); bitwise the same results;
 * key 36 = the fp32 split 3x3 form for 64-column N tiles: 0 (default) conv_tile_x3<64, 4, 2,
 * MODE, 4>; 1 the 4-wave 8 x 32 form on large grids; 2 / 3 the 4-wave 4 x 32 forms (timing
 * kinds 128 + 8 mode + 7);
 * key 37 = workgroups per CU of of_warp_bwd_det's fixed-point kernels (0 = default: 8 for the
 * element passes, 2 for the scatter);
 * key 38 = extra dynamic LDS bytes per own_window workgroup (an occupancy probe; default 0);
 * key 39 = timing ablation: the split 3x3 input gradients without their act' source reads
 * (RESULTS ARE WRONG; default 0). */
int of_set_tuning(int key, int value);
int of_timing_read(int max, int* kinds, double* flops, float* ms);

/* ==== bf16 activation images (configs 3-5, round 4) ====================================== */
/* x (npix pixels of ldx fp32, c used) -> y16: npix pixels of ldo bf16 (RNE), channels [c, ldo)
 * zero; ldo % 8 == 0. */
int of_to_bf16_image(const float* x, int64_t npix, int c, int ldx, void* y16, int ldo,
                     void* stream);
/* 3x3 stride-1 forward (mode 0) / input gradient (mode 1) of the convs of model.py:104-114 and
 * the resnet blocks, on the DMA-fed large-tile kernel conv_halo_b16, with bf16 activation
 * images at both ends: the GEMM A source (fwd: x, dgrad: dy) is the bf16 image a16 (lda16
 * channels per pixel, a multiple of 32 and >= round_up(kc, 32), kc = cin_p (fwd) /
 * round_up(cout, 4) (dgrad); channels past kc zero), the weights the packed bf16 images of
 * of_conv_pack_weights_bf16.  Epilogue as of_conv2d_fwd (bias, BN, aux = residual, act) /
 * of_conv2d_dgrad (the producer's act' from act_src (fp32), act16 (bf16 image) or mask_in (the
 * signs its b16i forward wrote); no added gradient); the result goes to y (fp32) and / or y16
 * (bf16 image, RNE).  col_part
 * (dgrad, optional): per output tile the column sums of the fp32 result, [tiles][N] with tiles =
 * of_conv2d_b16i_tiles(1, d) -- the bias gradient of the layer that produced dy, reduced by
 * of_col_part_reduce.  No workspace (one K slice). */
typedef struct of_b16i_io {
  const void* a16; int lda16;
  float* y; int ldy;
  void* y16; int ldy16;
  const float* aux; int ldr;
  const float* act_src; int ld_act;
  const void* act16; int ld_act16;
  float* col_part;
  void* mask_out;        /* fwd (optional): the output's act' signs, of_conv2d_b16i_mask_bytes */
  const void* mask_in;   /* dgrad (optional): mask_out of the forward that produced the act'
                          * source (same N = its cout, same n, h, w); replaces act16 / act_src */
} of_b16i_io;
int of_conv2d_b16i_tiles(int mode, const of_conv_desc* d);
size_t of_conv2d_b16i_mask_bytes(const of_conv_desc* d);
int of_conv2d_b16i(int mode, const of_conv_desc* d, const of_b16i_io* io, const void* w16,
                   const float* bias, const float* bn_gamma, const float* bn_beta,
                   const float* bn_mean, const float* bn_var, float bn_eps, int act, float alpha,
                   void* stream);
/* Weight gradient of the same convs from bf16 images (x16: ldx16 bf16 per pixel, >= cin_p;
 * dy16: lddy16 >= cout), dw HWIO [3][3][cin][cout] (accumulate != 0 adds), scaled per output
 * channel by gamma / sqrt(var + eps) when bn_gamma (the folded inference BN); no bias gradient
 * (of_col_part_reduce gives it).  Deterministic: per-slice fp32 slabs in workspace
 * (of_conv2d_wgrad_b16i_workspace(d) bytes), reduced in a fixed order. */
size_t of_conv2d_wgrad_b16i_workspace(const of_conv_desc* d);
int of_conv2d_wgrad_b16i(const of_conv_desc* d, const void* x16, int ldx16, const void* dy16,
                         int lddy16, float* dw, int accumulate, const float* bn_gamma,
                         const float* bn_var, float bn_eps, void* workspace, size_t ws_bytes,
                         void* stream);
/* out[c] (+)= sum_r part[r][c], fixed order (deterministic). */
int of_col_part_reduce(const float* part, int rows, int n, float* out, int accumulate,
                       void* stream);

/* ==== SURVEY.md §8 f row 1: the KITTI data path (data_reader.py) ========================== */

/* One decoded frame inside a raw batch buffer: 8-bit BGR, h x w x 3, at byte `offset` from the
 * start of the buffer.  A raw batch = of_image_desc[2*batch] (frame 2i = image1 of pair i,
 * 2i+1 = image2, swaps already applied) padded to 256 bytes, then the frames. */
typedef struct of_image_desc {
  int64_t offset;
  int32_t h, w;
} of_image_desc;

/* PNG header: size, channels and bit depth (no pixel decode). */
int of_png_info(const char* path, int* h, int* w, int* channels, int* depth);
/* cv2.imread(path) (data_reader.py:53-54; IMREAD_COLOR): 8-bit BGR h x w x 3 into out
 * (cap bytes).  Gray is replicated, palettes expanded, alpha dropped, 16-bit -> high byte. */
int of_png_read_bgr(const char* path, uint8_t* out, int64_t cap, int* h, int* w);
/* Write an 8-bit image (c = 1 gray, 3 BGR, 4 BGRA) as PNG.  flags = filter | (level+1) << 8:
 * filter 0-4 fixed, 5 adaptive, 6 cycle by row; level bits 0 -> zlib level 6. */
int of_png_write(const char* path, const uint8_t* img, int h, int w, int c, int flags);
/* Largest height / width over n PNG headers, read by nthreads threads. */
int of_png_scan(int n, const char* const* paths, int nthreads, int* max_h, int* max_w);

/* AsyncReader (data_reader.py:81-124): nworkers decode threads fill nslots batch slots of raw
 * frames (each frame <= max_h x max_w) in shuffled order with a p=0.5 pair swap, seeded;
 * nbatches = npairs / batch (remainder dropped), reshuffled at each epoch wrap.  pinned != 0
 * allocates the slots with hipHostMalloc (needed by of_reader_next). */
typedef struct of_reader of_reader;
int of_reader_create(int npairs, const char* const* path1, const char* const* path2, int batch,
                     int nworkers, int nslots, int max_h, int max_w, uint64_t seed, int pinned,
                     of_reader** out);
int64_t of_reader_raw_bytes(const of_reader* r);
int of_reader_nbatches(const of_reader* r);
/* get_batch() (data_reader.py:121-124): waits for the next batch in order, copies its raw
 * frames into dev_raw (cap >= of_reader_raw_bytes) on `stream`, then runs
 * of_preprocess_pairs into out (batch, out_h, out_w, 6) on the same stream.  pair_index /
 * swapped (may be NULL) receive the batch's pair ids and swap flags.  The slot is refilled
 * with the next batch once that copy has completed. */
int of_reader_next(of_reader* r, void* dev_raw, int64_t cap, float* out, int out_h, int out_w,
                   int32_t* pair_index, int32_t* swapped, void* stream);
/* The same hand-out without a GPU: the raw batch is copied to host memory dst. */
int of_reader_next_host(of_reader* r, void* dst, int64_t cap, int32_t* pair_index,
                        int32_t* swapped);
int of_reader_destroy(of_reader* r);

/* read_item's cv2.resize(img, (out_w, out_h)) (INTER_LINEAR, 8-bit fixed point) + /255 - mean
 * (data_reader.py:56-63) + packing into (npairs, out_h, out_w, 6) float32 (:36-41), from a
 * raw batch already in device memory. */
int of_preprocess_pairs(const void* dev_raw, int npairs, int out_h, int out_w, float* out,
                        void* stream);

/* ==== SURVEY.md §8 f row 2: TensorFlow checkpoint bundles (save_weights / load_weights) ===== */

/* CRC32C (Castagnoli) of n bytes, continuing from crc (0 to start; unmasked).  The bundle's
 * table blocks and tensor entries carry masked CRC32C values (optical_flow_amd/checkpoint.py). */
uint32_t of_crc32c(const void* data, int64_t n, uint32_t crc);

/* ==== SURVEY.md §8 f row 4: flow pictures (drawing.py) ==================================== */

/* draw_optical_flow_color (drawing.py:45-53) for n flows (n, h, w, 2) -> (n, h, w, 3) BGR
 * bytes; ws: 2*n floats of workspace (per-image magnitude min/max). */
int of_flow_color(const float* flow, int n, int h, int w, uint8_t* bgr, float* ws, void* stream);
/* draw_optical_flow_intensity (drawing.py:37-42): min(sqrt(u^2 + u^2) / 20, 1) per pixel. */
int of_flow_intensity(const float* flow, int64_t npix, float* out, void* stream);

/* ==== Inference BatchNorm folded into the backward (FusedBatchNormGrad, model.py:14 and the
 * resnet blocks; P5).  With y = act(BN(z) + res), BN(z) = gamma zhat + beta, zhat = (z - mean) /
 * sqrt(var + eps), and t = dL/dy * act'(y):  dbeta = sum t, dgamma = sum t zhat, dbias = s sum t
 * and dz = t s with s = gamma / sqrt(var + eps).  dz is never formed: s is folded into the
 * conv's packed input-gradient weights (of_conv_pack_weights_bn / of_conv_pack_table_bn) and its
 * weight-gradient reduction (of_conv2d_wgrad_bn), both then take t.  z is not stored either:
 * zhat is recovered from y where t != 0, zhat = (y - res - beta) / gamma (gamma != 0). */
int of_conv_pack_weights_bn(const of_conv_desc* d, int precision, const float* w_hwio,
                            void* w_fwd, void* w_bwd, const float* bn_gamma,
                            const float* bn_var, float bn_eps, void* stream);
/* precision[i]: 0 fp32, 1 bf16, 2 fp32 split planes; bn_gamma[i] == NULL: no BN on conv i. */
int of_conv_pack_table_bn(int nconv, const of_conv_desc* descs, const float* const* w_hwio,
                          void* const* w_fwd, void* const* w_bwd, const int* precision,
                          const float* const* bn_gamma, const float* const* bn_var,
                          float bn_eps, void* host_table);
/* dw = s * (x^T t) (HWIO; accumulate != 0 adds); precision as above, workspace of
 * of_conv2d_wgrad_bn_workspace(d, precision) bytes. */
size_t of_conv2d_wgrad_bn_workspace(const of_conv_desc* d, int precision);
int of_conv2d_wgrad_bn(const of_conv_desc* d, int precision, const float* x, int ldx,
                       const float* t, int ldt, float* dw, int accumulate, const float* bn_gamma,
                       const float* bn_var, float bn_eps, void* workspace, size_t ws_bytes,
                       void* stream);
/* Input gradient of a layer whose input x = relu(u) has several consumers:
 * dx = act'(act_src) * (dgrad(dy) + add), the derivative applied after the sum (add may be
 * NULL; add == dx in place).  The producer-side t of the layer before. */
int of_conv2d_dgrad_add_act(const of_conv_desc* d, int precision, const float* dy, int lddy,
                            const void* w_bwd, const float* add, int ld_add,
                            const float* act_src, int ld_act, int act, float alpha, float* dx,
                            int lddx, void* workspace, size_t ws_bytes, void* stream);
/* of_conv2d_dgrad_add_act with the BN backward partial sums of the layer whose output is
 * act_src fused into its epilogue (round 5): besides dx = t, per channel sum t and sum t zhat
 * with zhat = (act_src - bn_res - bn_beta) / bn_gamma (bn_res: the residual added before the
 * activation, or NULL) into part ([*nblk][2][cin] floats, of_conv2d_dgrad_bnp_bytes(d)
 * bytes), for of_bn_bwd_final.  The fp32 split 3x3 input gradient with one K slice only:
 * OF_EUNSUPPORTED (nothing launched) otherwise. */
size_t of_conv2d_dgrad_bnp_bytes(const of_conv_desc* d);
int of_conv2d_dgrad_add_act_bnp(const of_conv_desc* d, int precision, const float* dy, int lddy,
                                const void* w_bwd, const float* add, int ld_add,
                                const float* act_src, int ld_act, int act, float alpha,
                                float* dx, int lddx, const float* bn_gamma, const float* bn_beta,
                                const float* bn_res, int ld_bn_res, float* part,
                                size_t part_bytes, int* nblk, void* workspace, size_t ws_bytes,
                                void* stream);
/* dgamma / dbeta / dbias from nblk partial rows [nblk][2][c] (sum t, sum t zhat) in a fixed
 * order: dbeta = sum t, dgamma = sum t zhat, dbias = dbeta gamma / sqrt(var + eps);
 * accumulate: add to the outputs. */
int of_bn_bwd_final(const float* part, int nblk, int c, const float* gamma, const float* var,
                    float eps, float* dgamma, float* dbeta, float* dbias, int accumulate,
                    void* stream);
/* BN backward reductions from t (act NONE: dy is t) or from dy (act RELU: t = dy [y > 0],
 * written to t_out if non-NULL); res: the residual added before the activation, or NULL.
 * dgamma / dbeta / dbias: [c] (NULL to skip).  Workspace: of_bn_act_bwd_workspace(npix, c). */
int of_bn_bwd_reduce(int64_t npix, int c, int act, const float* dy, const float* y,
                     const float* res, const float* gamma, const float* beta, const float* var,
                     float eps, float* t_out, float* dgamma, float* dbeta, float* dbias,
                     int accumulate, void* workspace, void* stream);
/* Recovering zhat = (y - res - beta) / gamma from y loses precision as |gamma| -> 0 (and is
 * undefined at 0); the host keeps z for a BN layer once any of its gammas falls below a
 * threshold (ops.BNZGuard).  This gives min |gamma| per layer in one launch: out[i] =
 * min |dev_ptrs[i][0 .. dev_lens[i])| (both arrays in device memory). */
int of_min_abs_segments(const float* const* dev_ptrs, const int* dev_lens, int nseg, float* out,
                        void* stream);
/* of_maxpool_bn_act_bwd without z (zhat from y) for the stem: conv1 -> BN -> ReLU -> max-pool. */
int of_maxpool_bn_relu_bwd(int n, int h, int w, int c, const float* dyp, const float* g,
                           const float* y, const float* gamma, const float* beta,
                           const float* var, float eps, float* dz, float* dgamma, float* dbeta,
                           float* dbias, int accumulate, void* workspace, void* stream);

/* The stem forward (conv1 + layer1_bn + ReLU, model.py:12-15) with the following MaxPool2D
 * (model.py:17) in its epilogue: y as of_conv2d_fwd_x3 / _bf16 (precision 2 / 1) writes it, and
 * pool (n, ho/2, wo/2, cout) = the 2x2 / stride-2 max of y, bit-identical to of_maxpool2_fwd.
 * OF_EUNSUPPORTED unless the stem kernel takes the layer with an even output. */
int of_conv2d_fwd_pool(const of_conv_desc* d, int precision, const float* x, int ldx,
                       const void* w_fwd, const float* bias, const float* bn_gamma,
                       const float* bn_beta, const float* bn_mean, const float* bn_var,
                       float bn_eps, int act, float alpha, float* z, int ldz, float* y, int ldy,
                       float* pool, void* workspace, size_t ws_bytes, void* stream);
/* The stem's whole backward in one conv kernel (model.py:12-17, reset18_encoder's conv1 ->
 * layer1_bn -> ReLU -> {out0, MaxPool2D}): dz = relu'(y) (g + the max-pool gradient dyp at the
 * first maximum of each 2x2 window) * gamma / sqrt(var + eps) is formed while the weight
 * gradient stages it (of_maxpool_bn_relu_bwd's math, dz never stored), with dw (HWIO, 7x7x3x64),
 * dbias = s sum t, dgamma = sum t zhat (zhat = (y - beta) / gamma), dbeta = sum t (accumulate
 * != 0 adds into them).  y: the stem output (n, ho, wo, 64), g: its other consumer's gradient or
 * NULL, dyp: the pooled gradient (n, ho/2, wo/2, 64).  precision 2 (the fp32 split) or 1 (bf16);
 * OF_EUNSUPPORTED for other shapes (then of_maxpool_bn_relu_bwd + of_conv2d_wgrad*).
 * Workspace: of_stem_bwd_fused_workspace(d, precision) bytes (0: unsupported). */
size_t of_stem_bwd_fused_workspace(const of_conv_desc* d, int precision);
int of_stem_bwd_fused(const of_conv_desc* d, int precision, const float* x, int ldx,
                      const float* dyp, const float* g, const float* y, const float* gamma,
                      const float* beta, const float* var, float eps, float* dw, float* dbias,
                      float* dgamma, float* dbeta, int accumulate, void* workspace,
                      size_t ws_bytes, void* stream);

/* ==== SURVEY.md §8 P5: BatchNormalization in training mode (bn_mode = "training") ========= */
/* keras BatchNormalization called with training=True (old/train.py:59; the reference's
 * train.py:51 runs inference mode, the build default): z is the conv output (bias included),
 * npix rows x c channels (NHWC, c % 4 == 0, c <= 1024), split into `groups` contiguous row
 * ranges with separate statistics (the Siamese (2B) batch: model.py:131-132 calls the encoder
 * once per image).  Fixed-order reductions (bitwise reproducible).
 * Workspace of all three: of_bn_train_workspace(npix, c, groups) bytes. */
size_t of_bn_train_workspace(int64_t npix, int c, int groups);
/* mean[g][c], invstd[g][c] = 1 / sqrt(biased var + eps); moving statistics (NULL to skip)
 * updated group by group in order as FusedBatchNormV3 does with exponential_avg_factor
 * f = 1 - momentum: moving = (1 - f) moving + f stat, the variance Bessel-corrected. */
int of_bn_train_stats(int64_t npix, int c, int groups, const float* z, float eps, float momentum,
                      float* mean, float* invstd, float* moving_mean, float* moving_var,
                      void* workspace, void* stream);
/* y = act(gamma (z - mean[g]) invstd[g] + beta + res)   (res may be NULL; act OF_ACT_*) */
int of_bn_train_apply(int64_t npix, int c, int groups, const float* z, const float* mean,
                      const float* invstd, const float* gamma, const float* beta,
                      const float* res, int act, float* y, void* stream);
/* FusedBatchNormGradV3 (is_training): t = dy act'(y) (to t_out if non-NULL: the residual's
 * gradient); per group st = sum t, stz = sum t zhat; dz = gamma invstd (t - st/n - zhat stz/n);
 * dgamma (+)= sum over groups of stz, dbeta (+)= sum of st (NULL to skip). */
int of_bn_train_bwd(int64_t npix, int c, int groups, int act, const float* dy, const float* y,
                    const float* z, const float* mean, const float* invstd, const float* gamma,
                    float* dz, float* t_out, float* dgamma, float* dbeta, int accumulate,
                    void* workspace, void* stream);

/* ==== SURVEY.md §8 b / §8 e: gradient all-reduce over RCCL (build-added K14) ============= */
/* The reference is single-process (train.py:47-61); batch data parallelism sums the
 * gradients tape.gradient() returns (train.py:55) across ranks before the Adam update
 * (train.py:56).  One communicator per process / GPU; the id is made by rank 0 and handed to
 * the other ranks by the caller (optical_flow_amd/comm.py: the torch.distributed TCPStore).
 * librccl.so.1 is dlopen-ed on first use (OF_EUNSUPPORTED if absent). */
typedef struct of_comm of_comm;
int of_comm_id_bytes(void);                      /* bytes of a unique id (128) */
int of_comm_get_unique_id(void* id);
/* OF_OK when librccl loads with every entry point used here and a HIP device is current:
 * checked (and agreed on over the rendezvous store) before any rank enters of_comm_init. */
int of_comm_probe(void);
/* Collective over the nranks processes; binds the communicator to the current HIP device. */
int of_comm_init(of_comm** comm, const void* id, int nranks, int rank);
/* The same with a deadline: a non-blocking RCCL init (ncclConfig_t.blocking = 0) polled until
 * it completes; a rendezvous a peer never reaches is aborted after timeout_s seconds and
 * OF_ETIMEOUT is returned (timeout_s <= 0 or an RCCL without ncclCommInitRankConfig: the
 * blocking of_comm_init). */
int of_comm_init_timeout(of_comm** comm, const void* id, int nranks, int rank,
                         double timeout_s);
int of_comm_info(const of_comm* comm, int* nranks, int* rank, int* device);
/* recv = sum over ranks of send (count fp32 elements; send == recv is in place), enqueued on
 * `stream` and ordered after the work already on it; returns without waiting. */
int of_comm_allreduce_async(of_comm* comm, const float* send, float* recv, int64_t count,
                            void* stream);
/* The same with the reduction chosen: OF_REDUCE_SUM (the gradient buckets; the 1/N average
 * is folded into the Adam launch) or OF_REDUCE_AVG (recv = the mean over ranks: the BN moving
 * statistics of bn_mode "training", once per data-parallel step). */
#define OF_REDUCE_SUM 0
#define OF_REDUCE_AVG 1
int of_comm_allreduce_ex_async(of_comm* comm, const float* send, float* recv, int64_t count,
                               int op, void* stream);
/* OF_OK unless the communicator has failed asynchronously (or was aborted). */
int of_comm_async_error(of_comm* comm);
/* Aborts the communicator's in-flight operations (ncclCommAbort) WITHOUT freeing the handle:
 * safe from a watchdog thread while the owner may still hold the handle -- every later call
 * on it returns an error, and the owner frees it with of_comm_destroy. */
int of_comm_abort(of_comm* comm);
/* Frees the communicator (abort != 0: without waiting for in-flight operations). */
int of_comm_destroy(of_comm* comm, int abort);

#ifdef __cplusplus
}
#endif
#endif /* OFLOW_H */
