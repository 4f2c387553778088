"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

Restatement, in plain torch-CPU (float32 or float64), of the TensorFlow/Keras semantics of
xianlopez/optical_flow's training hot path: ``model.py`` (encoder, cost volume, warp,
upscale, flow modules), ``transformations.py`` (bilinear sampler), ``loss.py`` (photometric
L1 pyramid) and the Keras Adam step of ``train.py``.  Every function cites the reference
line it follows.  Autodiff here is torch autograd over these literal restatements, which
reproduces TF's gradients for the same ops (GatherNd -> scatter-add, floor/cast -> no grad,
Abs -> sign, ResizeBilinear -> its adjoint).

PARITY UNPINNED: TensorFlow/Keras are not installed in this image, the reference ships no
tests, golden vectors or fixtures, and the encoder blocks live in an un-vendored submodule
(``resnet``).  This oracle is therefore pinned only by hand-derived known-answer tests of
the TF op semantics (tests/test_oracle.py) and a second, numpy gather_nd restatement of the
warp (``oracle/warp_np.py``) -- not by outputs of the reference itself.

Layout: NHWC activations, HWIO kernels (the reference's layouts).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

LEAKY_ALPHA = 0.3        # keras.layers.LeakyReLU() default (model.py:105, P4)
BN_EPS = 1e-3            # keras BatchNormalization default epsilon (model.py:14, P5)


# ----------------------------------------------------------------------------- conv ----
def same_pads(n: int, k: int, s: int):
    """Keras/TF padding='same': out = ceil(n/s), total pad = max((out-1)*s + k - n, 0),
    floor(total/2) before, the rest after (P3; model.py:12)."""
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


# Conv operand precision of the build under test: "fp32" (config 2) or "bf16" (configs 3-5:
# forward, input-gradient and weight-gradient contractions on bf16-rounded operands, fp32
# accumulation; the bias gradient and the narrow cout <= 4 layers stay fp32 -- the HIP
# build's policy).
CONV_PRECISION = "fp32"


def set_conv_precision(p):
    global CONV_PRECISION
    assert p in ("fp32", "bf16"), p
    CONV_PRECISION = p


def bf16_round(t):
    """Round to bf16 (round-to-nearest-even) and back to t's dtype."""
    return t.to(torch.bfloat16).to(t.dtype)


def _narrow(w, stride):
    """The build's narrow-conv rule (conv_narrow.hip narrow_ok): those stay fp32."""
    kh, kw, cin, cout = w.shape
    nq = (cin + 3) // 4
    return cout <= 4 and stride == 1 and kh == 3 and kw == 3 and nq in (1, 2, 4, 8, 16)


class _Bf16Conv(torch.autograd.Function):
    """conv2d_same with bf16-rounded operands (x, w, and dz for both gradients), exact bias
    gradient."""

    @staticmethod
    def forward(ctx, x, w, b, stride):
        ctx.save_for_backward(x, w)
        ctx.stride = stride
        return _conv2d_same_exact(bf16_round(x), bf16_round(w), b, stride)

    @staticmethod
    def backward(ctx, dz):
        x, w = [t.detach() for t in ctx.saved_tensors]
        with torch.enable_grad():
            xv = x.clone().requires_grad_(True)
            (_conv2d_same_exact(xv, bf16_round(w), None, ctx.stride) * bf16_round(dz)).sum().backward()
            wv = w.clone().requires_grad_(True)
            (_conv2d_same_exact(bf16_round(x), wv, None, ctx.stride) *
             bf16_round(dz)).sum().backward()
        db = dz.sum(dim=(0, 1, 2)) if ctx.needs_input_grad[2] else None
        return xv.grad, wv.grad, db, None


def conv2d_same(x, w, b, stride=1):
    """layers.Conv2D(padding='same') on NHWC x, HWIO w (model.py:12,104-114)."""
    if CONV_PRECISION == "bf16" and not _narrow(w, stride):
        return _Bf16Conv.apply(x, w, b, stride)
    return _conv2d_same_exact(x, w, b, stride)


def _conv2d_same_exact(x, w, b, stride=1):
    kh, kw = w.shape[0], w.shape[1]
    pt, pb = same_pads(x.shape[1], kh, stride)
    pl, pr = same_pads(x.shape[2], kw, stride)
    xn = x.permute(0, 3, 1, 2)
    xn = F.pad(xn, (pl, pr, pt, pb))
    y = F.conv2d(xn, w.permute(3, 2, 0, 1).contiguous(), b, stride=stride)
    return y.permute(0, 2, 3, 1)


class _Bf16ConvBN(torch.autograd.Function):
    """bf16 mode, conv + inference BN (the encoder's conv_a / conv_b / proj): the operand
    rounding points of the build's folded BN backward (ops._conv_backward): with t = dL/du the
    gradient of the BN output u and s = gamma / sqrt(var + eps), the input gradient is
    conv^T(bf16(t), bf16(W s)) and the weight gradient s * (bf16(x)^T bf16(t)); the bias,
    gamma and beta gradients are exact.  (The stem keeps dz = t s: its fused max-pool / BN
    backward forms dz, see encoder().)"""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, mean, var, stride):
        ctx.save_for_backward(x, w, gamma, mean, var)
        ctx.stride = stride
        z = _conv2d_same_exact(bf16_round(x), bf16_round(w), b, stride)
        ctx.zhat = (z - mean) / torch.sqrt(var + BN_EPS)
        return ctx.zhat * gamma + beta

    @staticmethod
    def backward(ctx, t):
        x, w, gamma, mean, var = [v.detach() for v in ctx.saved_tensors]
        sc = gamma / torch.sqrt(var + BN_EPS)
        tr = bf16_round(t)
        with torch.enable_grad():
            xv = x.clone().requires_grad_(True)
            (_conv2d_same_exact(xv, bf16_round(w * sc), None, ctx.stride) * tr).sum().backward()
            wv = w.clone().requires_grad_(True)
            (_conv2d_same_exact(bf16_round(x), wv, None, ctx.stride) * tr).sum().backward()
        dw = wv.grad * sc
        red = tuple(range(t.dim() - 1))
        db = t.sum(dim=red) * sc
        dgamma = (t * ctx.zhat).sum(dim=red)
        dbeta = t.sum(dim=red)
        return xv.grad, dw, db, dgamma, dbeta, None, None, None


# BatchNormalization mode of the build under test: "inference" -- the
# reference's train.py:51 calls flow_net(batch_imgs) without training=True -- or "training",
# the legacy loop's model(images, training=True) (old/train.py:59).
BN_MODE = "inference"
BN_MOMENTUM = 0.99       # keras BatchNormalization default momentum


def set_bn_mode(m):
    global BN_MODE
    assert m in ("inference", "training"), m
    BN_MODE = m


def batchnorm_training(x, p: Dict[str, torch.Tensor], prefix: str):
    """keras BatchNormalization called with training=True (old/train.py:59), on Keras' fused
    path (FusedBatchNormV3, is_training): normalise with this call's batch mean and BIASED
    variance over (N, H, W), eps=1e-3; the moving statistics are updated in place as the fused
    op does with exponential_avg_factor f = 1 - momentum: moving = (1 - f) moving + f stat,
    the variance with Bessel's correction n / (n - 1).  Gradients flow through the batch
    statistics (FusedBatchNormGradV3)."""
    g, be = p[prefix + "/gamma"], p[prefix + "/beta"]
    red = tuple(range(x.dim() - 1))
    mu = x.mean(dim=red)
    var = ((x - mu) ** 2).mean(dim=red)
    n = x.numel() // x.shape[-1]
    with torch.no_grad():
        f = 1.0 - BN_MOMENTUM
        mm, mv = p[prefix + "/moving_mean"], p[prefix + "/moving_variance"]
        mm.copy_((1 - f) * mm + f * mu.detach().to(mm.dtype))
        mv.copy_((1 - f) * mv + f * (var.detach() * (n / max(n - 1, 1))).to(mv.dtype))
    return (x - mu) / torch.sqrt(var + BN_EPS) * g + be


def batchnorm(x, p, prefix):
    return batchnorm_training(x, p, prefix) if BN_MODE == "training" else \
        batchnorm_inference(x, p, prefix)


def batchnorm_inference(x, p: Dict[str, torch.Tensor], prefix: str):
    """keras BatchNormalization called with training unset -> inference mode: moving
    statistics, eps=1e-3, no statistic update; gamma/beta trainable (P5; train.py:51)."""
    g, be = p[prefix + "/gamma"], p[prefix + "/beta"]
    mu, var = p[prefix + "/moving_mean"], p[prefix + "/moving_variance"]
    return (x - mu) * (g / torch.sqrt(var + BN_EPS)) + be


def leaky_relu(x):
    return torch.where(x > 0, x, LEAKY_ALPHA * x)


def maxpool2(x):
    """layers.MaxPool2D() default pool 2, stride 2, 'valid' (model.py:17)."""
    return F.max_pool2d(x.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)


# -------------------------------------------------------------------------- encoder ----
def _conv_bn(x, p, conv, bn, stride):
    if BN_MODE == "training":      # batch statistics: the plain conv, then the BN (P5)
        return batchnorm_training(conv2d_same(x, p[conv + "/kernel"], p[conv + "/bias"], stride),
                                  p, bn)
    if CONV_PRECISION == "bf16":
        return _Bf16ConvBN.apply(x, p[conv + "/kernel"], p[conv + "/bias"], p[bn + "/gamma"],
                                 p[bn + "/beta"], p[bn + "/moving_mean"],
                                 p[bn + "/moving_variance"], stride)
    y = conv2d_same(x, p[conv + "/kernel"], p[conv + "/bias"], stride)
    return batchnorm_inference(y, p, bn)


def resnet_block(x, p, prefix, stride, proj):
    """ASSUMED standard ResNet-18 basic block (the ``resnet`` submodule
    behind model.py:2,18,20,22 is absent -> parity unpinned)."""
    y = torch.relu(_conv_bn(x, p, prefix + "/conv_a", prefix + "/bn_a", stride))
    y = _conv_bn(y, p, prefix + "/conv_b", prefix + "/bn_b", 1)
    sc = _conv_bn(x, p, prefix + "/proj", prefix + "/bn_proj", stride) if proj else x
    return torch.relu(y + sc)


def encoder(x, p, blocks):
    """reset18_encoder (model.py:10-26) -> [H/2 x64, H/4 x64, H/8 x128, H/16 x256]."""
    x = conv2d_same(x, p["ResNet18/conv1/kernel"], p["ResNet18/conv1/bias"], 2)
    x = torch.relu(batchnorm(x, p, "ResNet18/layer1_bn"))
    outs = [x]
    x = maxpool2(x)
    for i, (prefix, cin, cout, stride, proj) in enumerate(blocks):
        x = resnet_block(x, p, prefix, stride, proj)
        if i % 2 == 1:
            outs.append(x)
    return outs


# ---------------------------------------------------------------- flow primitives ----
def create_cost_volume(f1, f2, max_disp):
    """model.py:29-42 literally: zero-pad f2 by max_disp, channel k = i*(2d+1)+j holds
    sum_c f1 * f2[:, i:i+h, j:j+w] (P8)."""
    h, w = f1.shape[1], f1.shape[2]
    f2p = F.pad(f2, (0, 0, max_disp, max_disp, max_disp, max_disp))
    cor = []
    for i in range(2 * max_disp + 1):
        for j in range(2 * max_disp + 1):
            cor.append((f1 * f2p[:, i:i + h, j:j + w, :]).sum(-1))
    return torch.stack(cor, -1)


def evaluate_tensor_on_xy_grid(inp, x, y):
    """transformations.py:70-81: gather_nd(inp, stack([b, y, x])) -> (B,h,w,C)."""
    bsz = inp.shape[0]
    bidx = torch.arange(bsz).view(bsz, 1, 1).expand_as(x)
    return inp[bidx, y, x]


def bilinear_interpolation(inp, pts):
    """transformations.py:85-129 literally (P2): ch0 of ``pts`` is x (column), ch1 is y
    (row); x0/x1/y0/y1 clipped; weights from the CLIPPED x1/y1 and unclipped x/y; no
    gradient through floor/cast."""
    _, h, w, _ = inp.shape
    x = pts[..., 0]
    y = pts[..., 1]
    x0 = torch.floor(x).to(torch.int64)
    y0 = torch.floor(y).to(torch.int64)
    x1 = x0 + 1
    y1 = y0 + 1
    x0 = x0.clamp(0, w - 1)
    x1 = x1.clamp(0, w - 1)
    y0 = y0.clamp(0, h - 1)
    y1 = y1.clamp(0, h - 1)
    v00 = evaluate_tensor_on_xy_grid(inp, x0, y0)
    v01 = evaluate_tensor_on_xy_grid(inp, x0, y1)
    v10 = evaluate_tensor_on_xy_grid(inp, x1, y0)
    v11 = evaluate_tensor_on_xy_grid(inp, x1, y1)
    a = x1.to(x.dtype) - x
    b = y1.to(y.dtype) - y
    w00 = (a * b).unsqueeze(-1)
    w01 = (a * (1.0 - b)).unsqueeze(-1)
    w10 = ((1.0 - a) * b).unsqueeze(-1)
    w11 = ((1.0 - a) * (1.0 - b)).unsqueeze(-1)
    return w00 * v00 + w01 * v01 + w10 * v10 + w11 * v11


def warp_features(flow, f2):
    """model.py:55-73: grid = meshgrid(range(h), range(w), 'ij') stacked [row, col] + flow,
    then sampled as (x=ch0, y=ch1) -- the reference's transposed convention (P1, F6)."""
    _, h, w, _ = f2.shape
    ii, jj = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    grid = torch.stack([ii, jj], -1).to(torch.float32).unsqueeze(0)
    # The reference forms the sampling coordinates in float32 (model.py:69-71: tf.cast(...,
    # tf.float32) + flow); floor() of them decides the gather corners, so they are rounded to
    # float32 here too even when the oracle runs in float64.
    pts = (grid + flow.to(torch.float32)).to(flow.dtype)
    return bilinear_interpolation(f2, pts)


def resize_bilinear(x, h, w):
    """tf.image.resize(method=bilinear, antialias=False) == half-pixel-centre bilinear ==
    torch interpolate(align_corners=False) (P6; loss.py:18, model.py:77)."""
    y = F.interpolate(x.permute(0, 3, 1, 2), size=(h, w), mode="bilinear",
                      align_corners=False, antialias=False)
    return y.permute(0, 2, 3, 1)


def upscale_flow(flow):
    """model.py:76-77: resize x2, times 2.0 on both channels (P7)."""
    return resize_bilinear(flow, flow.shape[1] * 2, flow.shape[2] * 2) * 2.0


def flow_head(x, p, prefix, masks=None):
    """model.py:104-114: 6 convs 3x3 'same', LeakyReLU(0.3) after the first five.
    masks (tests only): per LeakyReLU, a boolean tensor choosing the slope-1 side instead of
    the sign of the pre-activation -- the slopes another implementation took, so that a
    comparison is not dominated by pre-activations within rounding of the kink at 0."""
    for i in range(6):
        x = conv2d_same(x, p["%s/conv%d/kernel" % (prefix, i)],
                        p["%s/conv%d/bias" % (prefix, i)], 1)
        if i < 5:
            x = leaky_relu(x) if masks is None else torch.where(masks[i], x, LEAKY_ALPHA * x)
    return x


def flow_module(f1, f2, prev, max_disp, p, prefix, masks=None):
    """model.py:80-116 (masks: see flow_head)."""
    if prev is not None:
        flow_up = upscale_flow(prev)
        f2w = warp_features(flow_up, f2)
    else:
        f2w = f2
    cv = create_cost_volume(f1, f2w, max_disp)
    if prev is not None:
        x = torch.cat([f1, cv, flow_up], -1)
    else:
        x = torch.cat([f1, cv], -1)
    return flow_head(x, p, prefix, masks)


def flow_net(batch_imgs, p, blocks, max_disp=3):
    """build_flow_net's graph (model.py:119-143); returns [flow3, flow2, flow1, flow0]
    (fine -> coarse, P10).  The shared encoder is applied to both images (P12)."""
    img1 = batch_imgs[..., :3]
    img2 = batch_imgs[..., 3:]
    e1 = encoder(img1, p, blocks)
    e2 = encoder(img2, p, blocks)
    flows = []
    prev = None
    n = len(e1)                  # 4, or 5 with the commented-out stage 5 (model.py:24-25,138)
    for level in range(n):
        prev = flow_module(e1[n - 1 - level], e2[n - 1 - level], prev, max_disp, p,
                           "flow_module_%d" % level)
        flows.append(prev)
    return flows[::-1]


def two_layer_head(batch_imgs, p):
    """Config-1 plumbing head (build-defined; SURVEY.md §8 d)."""
    x = leaky_relu(conv2d_same(batch_imgs, p["head2/conv0/kernel"], p["head2/conv0/bias"], 2))
    return [conv2d_same(x, p["head2/conv1/kernel"], p["head2/conv1/bias"], 1)]


# ------------------------------------------------------------------------------ loss ----
def photometric_loss(batch_imgs, flows):
    """LossLayer.__call__ (loss.py:5-32): per scale s, resize all 6 channels to
    H/2^(s+1), warp image2 by flows[s], mean |img1 - warped|; average over scales."""
    n = len(flows)
    loss = batch_imgs.new_zeros(())
    H, W = batch_imgs.shape[1], batch_imgs.shape[2]
    for s in range(n):
        h = int(H / (2.0 ** (s + 1)))
        w = int(W / (2.0 ** (s + 1)))
        assert flows[s].shape[1] == h and flows[s].shape[2] == w
        if h != H or w != W:
            r = resize_bilinear(batch_imgs, h, w)
        else:
            r = batch_imgs
        warped = warp_features(flows[s], r[..., 3:])
        loss = loss + (r[..., :3] - warped).abs().mean()
    return loss / float(n)


# ------------------------------------------------------------------------------ adam ----
class KerasAdam:
    """tf.keras.optimizers.Adam(learning_rate=1e-4) (train.py:34): beta1 0.9, beta2 0.999,
    epsilon 1e-7 in the 'epsilon hat' form of ResourceApplyAdam:
    lr_t = lr*sqrt(1-b2^t)/(1-b1^t); var -= lr_t*m/(sqrt(v)+eps)   (P13)."""

    def __init__(self, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-7):
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps
        self.t = 0
        self.m: Dict[str, torch.Tensor] = {}
        self.v: Dict[str, torch.Tensor] = {}

    @torch.no_grad()
    def step(self, params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor]):
        self.t += 1
        lr_t = self.lr * math.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        for k, g in grads.items():
            if k not in self.m:
                self.m[k] = torch.zeros_like(g)
                self.v[k] = torch.zeros_like(g)
            m, v = self.m[k], self.v[k]
            m.add_((g - m) * (1 - self.b1))          # training_ops ApplyAdam form
            v.add_((g * g - v) * (1 - self.b2))
            params[k].sub_(lr_t * m / (v.sqrt() + self.eps))


# ------------------------------------------------------------------------ train step ----
def train_step(batch_imgs, params, blocks, opt: Optional[KerasAdam], max_disp=3,
               model="full"):
    """train.py:47-61: forward, loss, gradients of the trainable weights, Adam update.
    Returns (loss, flows, grads).  ``params`` holds leaf tensors; trainable ones are
    updated in place when ``opt`` is given."""
    trainable = {k: v for k, v in params.items()
                 if not (k.endswith("moving_mean") or k.endswith("moving_variance"))}
    for v in trainable.values():
        v.requires_grad_(True)
        v.grad = None
    if model == "full":
        flows = flow_net(batch_imgs, params, blocks, max_disp)
    else:
        flows = two_layer_head(batch_imgs, params)
    loss = photometric_loss(batch_imgs, flows)
    names = list(trainable)
    gs = torch.autograd.grad(loss, [trainable[k] for k in names], allow_unused=True)
    grads = {k: (g if g is not None else torch.zeros_like(trainable[k]))
             for k, g in zip(names, gs)}
    for v in trainable.values():
        v.requires_grad_(False)
    if opt is not None:
        opt.step(trainable, grads)
    return loss.detach(), [f.detach() for f in flows], grads


def to_torch_params(np_params, dtype=torch.float32):
    return {k: torch.tensor(v, dtype=dtype) for k, v in np_params.items()}
