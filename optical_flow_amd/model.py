"""MI355X-native mirror of the reference ``model.py`` (xianlopez/optical_flow).

Same public names and argument meaning as ``/root/reference/model.py``:

* ``reset18_encoder(height, width, name)``                       (model.py:10-26)
* ``create_cost_volume(features1, features2, max_disp)``          (model.py:29-42)
* ``warp_features(flow_1_to_2, features2)``                       (model.py:55-73)
* ``upscale_flow(flow)``                                          (model.py:76-77)
* ``flow_module(features1, features2, previous_flow, max_disp)``  (model.py:80-116)
* ``build_flow_net(height, width, pretrained_weights_path, max_disp=3)`` (model.py:119-143)
* ``resnet_layer_simple(x, nblocks, downsample, idx)`` (the un-vendored ``resnet`` submodule's
  stage, model.py:2,18,20,22; assumed basic blocks)

Tensors are torch NHWC float32 on the GPU; every op runs as HIP kernels (``ops.py``).  The
returned ``FlowNet`` keeps the Keras ``Model`` surface the driver uses: ``__call__`` ->
``[flow3, flow2, flow1, flow0]`` (fine -> coarse), ``trainable_weights``, ``summary()``,
``save_weights(path)``, ``load_weights(path)``.

Parameters live in one flat device arena (``ParamStore``) with a matching gradient arena, so
the optimizer is a single fused launch and the data-parallel all-reduce works on contiguous
buckets.  The arena is ordered by backward completion (finest flow head first, encoder
stem last) so buckets become ready in order during the backward pass.
"""
from __future__ import annotations

import ctypes as C
import os
from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np
import torch

from . import ops
from ._lib import ACT_LEAKY, ACT_NONE, ACT_RELU, call
from .params import (ENC_CHANNELS, HEAD_WIDTHS, blocks_spec, encoder_blocks, encoder_spec,
                     flow_net_spec, head_cin, head_spec, init_params, stage_blocks)


# =================================================================== parameter arena ====
class ParamStore:
    """Flat fp32 device arenas for the trainable weights, their gradients, and the
    non-trainable BN moving statistics.  ``params[name]`` are leaf views (HWIO kernels)."""

    def __init__(self, spec, values: Optional[Dict[str, np.ndarray]] = None, device="cuda",
                 order: Optional[List[str]] = None, seed: int = 0):
        if values is None:
            values = init_params(spec, seed)
        self.spec = OrderedDict((p.name, p) for p in spec)
        train = [p for p in spec if p.trainable]
        if order is not None:
            rank = {n: i for i, n in enumerate(order)}
            train = sorted(train, key=lambda p: rank.get(p.name, len(rank)))
        self.arena_order = [p.name for p in train]
        self.offsets = OrderedDict()
        off = 0
        for p in train:
            self.offsets[p.name] = off
            off += (p.size + 3) // 4 * 4          # 16-byte aligned views
        self.numel = max(off, 4)
        self.arena = torch.zeros(self.numel, device=device)
        self.grad_arena = torch.zeros(self.numel, device=device)
        bufs = [p for p in spec if not p.trainable]
        self.buf_offsets = OrderedDict()
        off = 0
        for p in bufs:
            self.buf_offsets[p.name] = off
            off += (p.size + 3) // 4 * 4
        self.buffers = torch.zeros(max(off, 4), device=device)
        self.params: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        for p in spec:
            if p.trainable:
                o = self.offsets[p.name]
                v = self.arena[o:o + p.size].view(p.shape)
                v.requires_grad_(True)
                g = self.grad_arena[o:o + p.size].view(p.shape)
                v._of_grad = g
                v.grad = g
            else:
                o = self.buf_offsets[p.name]
                v = self.buffers[o:o + p.size].view(p.shape)
            self.params[p.name] = v
        self.version = 0
        self.bn_guard = None        # ops.BNZGuard, made by the model on its first forward
        self.load(values)

    def __getitem__(self, name) -> torch.Tensor:
        return self.params[name]

    def trainable(self) -> List[torch.Tensor]:
        return [self.params[n] for n, p in self.spec.items() if p.trainable]

    @torch.no_grad()
    def load(self, values: Dict[str, np.ndarray], strict: bool = True):
        missing = [n for n in self.spec if n not in values]
        if strict and missing:
            raise KeyError("missing weights: %s" % missing[:5])
        for n, v in values.items():
            if n not in self.params:
                if strict:
                    raise KeyError("unexpected weight %s" % n)
                continue
            t = torch.as_tensor(np.asarray(v, np.float32))
            assert tuple(t.shape) == tuple(self.spec[n].shape), (n, t.shape, self.spec[n].shape)
            self.params[n].copy_(t.to(self.params[n].device))
        self.version += 1
        if self.bn_guard is not None:        # new gammas: check them before the next step
            self.bn_guard.check_now()

    def state(self) -> "OrderedDict[str, np.ndarray]":
        return OrderedDict((n, self.params[n].detach().cpu().numpy()) for n in self.spec)

    def zero_grad(self):
        call("of_fill", C.c_void_p(self.grad_arena.data_ptr()), 0.0, self.numel, ops._stream())

    def grads(self) -> "OrderedDict[str, torch.Tensor]":
        return OrderedDict((n, self.params[n]._of_grad) for n, p in self.spec.items()
                           if p.trainable)


def backward_order(max_disp=3, levels=4) -> List[str]:
    """Arena order = gradient completion order of the backward pass."""
    names = []
    for level in reversed(range(levels)):
        names += [p.name for p in head_spec(level, max_disp, levels) if p.trainable]
    names += [p.name for p in reversed(encoder_spec(levels)) if p.trainable]
    return names


# ========================================================================= encoder ======
# OFLOW_PER_LAYER_BLOCKS=1: run the residual blocks as separate conv nodes (A/B timing only)
_PER_LAYER_BLOCKS = os.environ.get("OFLOW_PER_LAYER_BLOCKS", "0") == "1"

class Encoder:
    """reset18_encoder (model.py:10-26): conv1 7x7/2 + BN + ReLU -> out0 (H/2, 64);
    max-pool; three resnet_layer_simple stages -> H/4 x64, H/8 x128, H/16 x256.
    The stage body is the assumed standard basic block (params.py)."""

    def __init__(self, store: ParamStore, name="ResNet18", levels=4, bn_mode="inference"):
        self.store = store
        self.name = name
        self.levels = levels
        P = store.params
        stem_bn = tuple(P["ResNet18/layer1_bn/" + k]
                        for k in ("gamma", "beta", "moving_mean", "moving_variance"))
        self.conv1 = ops.ConvLayer(P["ResNet18/conv1/kernel"], P["ResNet18/conv1/bias"], stride=2,
                                   act=ACT_RELU, bn=stem_bn, cin_p=4,
                                   version_of=lambda: store.version, name="conv1")
        self.blocks = block_layers(store, encoder_blocks(levels))
        self.set_bn_mode(bn_mode)

    def bn_layers(self):
        out = [self.conv1]
        for a, b, p in self.blocks:
            out += [a, b] + ([p] if p is not None else [])
        return out

    def set_bn_mode(self, bn_mode):
        """"inference" (the reference's train.py:51: moving statistics, the default) or
        "training" (old/train.py:59: batch statistics, moving statistics updated; P5)."""
        assert bn_mode in ("inference", "training"), bn_mode
        self.bn_mode = bn_mode
        for L in self.bn_layers():
            L.bn_train = bn_mode == "training"
            L._pack_key = None

    def forward4(self, x4, groups=1):
        """x4: (N, H, W, 4) images with a zero 4th channel -> 4 feature maps.  groups: the
        number of separate encoder calls x4 stacks (the FlowNet's image1s / image2s: 2), each
        with its own batch statistics in bn_mode "training"."""
        if self.bn_mode == "training":
            return ops.encoder_forward_train(x4, self.conv1, self.blocks, groups)
        if not _PER_LAYER_BLOCKS:
            return ops.encoder_forward(x4, self.conv1, self.blocks)
        x = self.conv1(x4)
        outs = [x]
        x = ops.maxpool2(x)
        for i, (a, b, p) in enumerate(self.blocks):
            if _PER_LAYER_BLOCKS:       # A/B switch: one autograd node per conv
                y = a(x)
                x = b(y, residual=p(x) if p is not None else x)
            else:
                x = ops.res_block(x, a, b, p)
            if i % 2 == 1:
                outs.append(x)
        return outs

    def __call__(self, images):
        """images: (N, H, W, 3) -> [H/2 x64, H/4 x64, H/8 x128, H/16 x256]."""
        return self.forward4(ops._pad_channels(images, 4))


def block_layers(store: ParamStore, blocks):
    """(conv_a, conv_b, proj or None) ConvLayers of residual blocks whose weights live in
    ``store`` under the block prefixes of params.encoder_blocks / params.stage_blocks."""
    P = store.params
    ver = lambda: store.version

    def bn(prefix):
        return (P[prefix + "/gamma"], P[prefix + "/beta"], P[prefix + "/moving_mean"],
                P[prefix + "/moving_variance"])

    out = []
    for prefix, cin, cout, stride, proj in blocks:
        a = ops.ConvLayer(P[prefix + "/conv_a/kernel"], P[prefix + "/conv_a/bias"],
                          stride=stride, act=ACT_RELU, bn=bn(prefix + "/bn_a"),
                          version_of=ver, name=prefix + "/conv_a")
        b = ops.ConvLayer(P[prefix + "/conv_b/kernel"], P[prefix + "/conv_b/bias"], stride=1,
                          act=ACT_RELU, bn=bn(prefix + "/bn_b"), version_of=ver,
                          name=prefix + "/conv_b")
        p = None
        if proj:
            p = ops.ConvLayer(P[prefix + "/proj/kernel"], P[prefix + "/proj/bias"],
                              stride=stride, act=ACT_NONE, bn=bn(prefix + "/bn_proj"),
                              version_of=ver, name=prefix + "/proj")
        out.append((a, b, p))
    return out


def resnet_layer_simple(x, nblocks, downsample, idx, store: Optional[ParamStore] = None,
                        seed: int = 0, precision: str = "fp32", bn_mode: str = "inference"):
    """``resnet.models.resnet_layer_simple(x, nblocks, downsample, idx)`` (model.py:2,18,20,22).
    The ``resnet`` submodule is not vendored, so this is the assumed ResNet-18 basic stage
    (parity unpinned): ``nblocks`` blocks of [conv3x3(s) + BN + ReLU,
    conv3x3 + BN] + shortcut (1x1/s conv + BN when downsampling or when the channel count
    changes) -> add -> ReLU, with 64 * 2^(idx-2) output channels; BN in inference mode (P5).

    x: (N, H, W, C) NHWC float32 on the GPU; ``precision`` "bf16" runs the block convs on the
    bf16 kernels (configs 3-5).  Like the Keras functional call, a call with no
    ``store`` creates fresh layers (Keras-default init from ``seed``; the store is kept on
    the returned tensor as ``_resnet_store``); a ``store`` holding the stage's weights under
    ``ResNet18/res{idx}_{j}/...`` (e.g. a FlowNet's) reuses them."""
    assert x.dim() == 4, "NHWC input"
    blocks = stage_blocks(idx, x.shape[-1], nblocks, downsample)
    if store is None:
        store = ParamStore(blocks_spec(blocks), seed=seed, device=x.device)
    layers = block_layers(store, blocks)
    flat = [L for blk in layers for L in blk if L is not None]
    assert bn_mode in ("inference", "training"), bn_mode
    for L in flat:                      # "bf16": the convs on bf16 MFMA (configs 3-5)
        L.precision = precision
        L.bn_train = bn_mode == "training"
    if bn_mode == "training":           # batch statistics (P5): z always kept, no guard
        for a, b, p in layers:
            ya = ops.conv_bn_train(a, x)
            sc = ops.conv_bn_train(p, x) if p is not None else x
            x = ops.conv_bn_train(b, ya, residual=sc)
        x._resnet_store = store
        return x
    if store.bn_guard is None:          # z kept for BN layers with gamma ~ 0 (ops.BNZGuard)
        store.bn_guard = ops.BNZGuard(flat)
    store.bn_guard.poll()
    store.bn_guard.mark(flat)
    for a, b, p in layers:
        x = ops.res_block(x, a, b, p)
    x._resnet_store = store
    return x


def reset18_encoder(height, width, name="ResNet18", seed=0, device="cuda"):
    """model.py:10-26.  ``height``/``width`` fix nothing here (the kernels take any size
    divisible by 16); kept for signature parity.  Owns its own parameter store."""
    store = ParamStore(encoder_spec(), seed=seed, device=device)
    enc = Encoder(store, name)
    enc.input_shape = (height, width, 3)
    return enc


# =================================================================== flow primitives ====
def create_cost_volume(features1, features2, max_disp):
    """model.py:29-42 (P8): unnormalised 49-offset correlation, zero padding."""
    assert features1.shape == features2.shape
    return ops.cost_volume(features1, features2, max_disp)


def warp_features(flow_1_to_2, features2):
    """model.py:55-73 with the reference's index convention (P1): the grid is
    meshgrid(range(h), range(w), 'ij') + flow, sampled as (x=ch0, y=ch1)."""
    _, height, width, _ = features2.shape
    assert flow_1_to_2.shape[1] == height
    assert flow_1_to_2.shape[2] == width
    assert flow_1_to_2.shape[3] == 2
    return ops.warp(features2, flow_1_to_2)


def upscale_flow(flow):
    """model.py:76-77: bilinear resize x2 (half-pixel centres) times 2.0 (P6, P7)."""
    return ops.upscale2x(flow, 2.0)


class FlowHead:
    """The six 3x3 convs a ``flow_module`` call creates (model.py:104-114): 128, 128, 96, 64,
    32 with LeakyReLU(0.3), then a linear 2-channel flow conv."""

    def __init__(self, store: ParamStore, level: int, max_disp: int = 3, levels: int = 4):
        self.level = level
        self.max_disp = max_disp
        self.cin = head_cin(level, max_disp, levels)
        # Concat row padded to a multiple of 8 channels: 115 -> 120, not 116.  A 116-float
        # (464-byte) row runs the level-3/2 c0 convs 12-15 % slower than a 120-float one in
        # both precisions (profiles/r1_conv_bench*.txt); the zero channels cost 3.5 % MACs.
        self.cp = (self.cin + 7) // 8 * 8
        P = store.params
        ver = lambda: store.version
        self.convs = []
        for i, cout in enumerate(HEAD_WIDTHS):
            pre = "flow_module_%d/conv%d" % (level, i)
            self.convs.append(ops.ConvLayer(P[pre + "/kernel"], P[pre + "/bias"], stride=1,
                                            act=ACT_LEAKY if i < 5 else ACT_NONE,
                                            cin_p=self.cp if i == 0 else None, version_of=ver,
                                            name=pre))

    def __call__(self, features1, features2, previous_flow):
        return flow_module(features1, features2, previous_flow, self.max_disp, head=self)


def flow_module(features1, features2, previous_flow, max_disp, head: Optional[FlowHead] = None):
    """model.py:80-116: [upscale + warp] -> cost volume -> concat -> 6 convs.  Keras creates
    new conv layers per call; here ``head`` carries them (a fresh randomly initialised head
    is created when omitted, mirroring that)."""
    assert features1.shape[1] == features2.shape[1]
    assert features1.shape[2] == features2.shape[2]
    assert features1.shape[3] == features2.shape[3]
    if head is None:
        c = features1.shape[3]
        level = {256: 0, 128: 1, 64: 2 if previous_flow is not None else 3}.get(c, 2)
        if previous_flow is None and c != 256:
            raise ValueError("a standalone flow_module needs an explicit head for this shape")
        store = ParamStore(head_spec(level, max_disp), device=features1.device)
        head = FlowHead(store, level, max_disp)
        head._store = store
    if previous_flow is not None:
        assert previous_flow.shape[0] == features1.shape[0]
        assert previous_flow.shape[1] * 2 == features1.shape[1]
        assert previous_flow.shape[2] * 2 == features1.shape[2]
        assert previous_flow.shape[3] == 2
        flow_up = upscale_flow(previous_flow)
        features2_warped = warp_features(flow_up, features2)
    else:
        flow_up = None
        features2_warped = features2
    x = ops.corr_concat(features1, features2_warped, flow_up, max_disp, head.cp,
                        head.convs[0].precision, layers=head.convs)
    return ops.conv_stack(x, head.convs)


# ========================================================================= flow net ======
class FlowNet:
    """The Keras ``Model`` returned by build_flow_net (model.py:119-143)."""

    def __init__(self, height, width, max_disp=3, seed=0, device="cuda", values=None,
                 precision="fp32", levels=4, bn_mode="inference"):
        """levels=5 enables the reference's commented-out 5th pyramid level (model.py:24-25,
        138, 141): encoder stage 5 (512 channels at H/32) and flow4 at H/2.  bn_mode:
        "inference" (train.py:51, the default) or "training" (old/train.py:59; P5)."""
        assert levels in (4, 5), levels
        m = 2 ** levels
        assert height % m == 0 and width % m == 0, \
            "H and W must be divisible by %d with %d levels (P17)" % (m, levels)
        self.height, self.width, self.max_disp = height, width, max_disp
        self.levels = levels
        self.store = ParamStore(flow_net_spec(max_disp, levels), values=values, device=device,
                                order=backward_order(max_disp, levels), seed=seed)
        self.encoder = Encoder(self.store, levels=levels, bn_mode=bn_mode)
        self.heads = [FlowHead(self.store, level, max_disp, levels) for level in range(levels)]
        self.name = "flow_net"
        self._packer = None
        self.set_precision(precision)

    def set_precision(self, precision):
        """"fp32" (config 2) or "bf16" (configs 3-5: conv fwd / dgrad on bf16 MFMA, fp32
        accumulation, fp32 activations, weights, gradients and Adam state)."""
        assert precision in ("fp32", "bf16"), precision
        self.precision = precision
        for L in self.conv_layers():
            L.precision = precision
            L._bf16 = None
            L._wf = L._wd = None
            L._pack_key = None
        self._packer = None

    def set_bn_mode(self, bn_mode):
        """BatchNormalization "inference" (train.py:51, default) or "training" (P5)."""
        self.encoder.set_bn_mode(bn_mode)
        self._packer = None

    @property
    def bn_mode(self):
        return self.encoder.bn_mode

    def conv_layers(self):
        layers = [self.encoder.conv1]
        for a, b, p in self.encoder.blocks:
            layers += [a, b] + ([p] if p is not None else [])
        for h in self.heads:
            layers += h.convs
        return layers

    @property
    def trainable_weights(self) -> List[torch.Tensor]:
        return self.store.trainable()

    @property
    def weight_names(self) -> List[str]:
        return [n for n, p in self.store.spec.items() if p.trainable]

    def __call__(self, batch_imgs):
        """(B, H, W, 6) -> [flow3 (H/2), flow2 (H/4), flow1 (H/8), flow0 (H/16)] (levels=4;
        levels=5 prepends flow4 at H/2, so flow0 is at H/32)."""
        assert batch_imgs.shape[1] == self.height and batch_imgs.shape[2] == self.width
        assert batch_imgs.shape[3] == 6
        if self._packer is None:
            self._packer = ops.ConvPacker(self.conv_layers(), lambda: self.store.version)
        if self.encoder.bn_mode == "inference":
            if self.store.bn_guard is None:          # z kept for BN layers with gamma ~ 0
                self.store.bn_guard = ops.BNZGuard(self.conv_layers())
            self.store.bn_guard.poll()
        self._packer.ensure()                        # all conv weights packed in one launch
        imgs = ops.split_pair(batch_imgs)            # image1s then image2s (model.py:122-123)
        # shared encoder, both images (P12); training-mode BN: two calls' statistics
        feats = self.encoder.forward4(imgs, groups=2)
        flows = []
        prev = None
        L = self.levels
        for level in range(L):
            f1, f2 = ops.halves(feats[L - 1 - level])
            prev = self.heads[level](f1, f2, prev)
            flows.append(prev)
        return flows[::-1]

    # ---- Keras Model surface used by train.py ------------------------------------------
    def summary(self, print_fn=print):
        total = 0
        print_fn("Model: \"%s\"" % self.name)
        for n, p in self.store.spec.items():
            total += p.size if p.trainable else 0
            print_fn("  %-44s %-18s %s" % (n, str(p.shape), "" if p.trainable else "(non-trainable)"))
        print_fn("Trainable params: %d" % total)

    def save_weights(self, path, save_format=None):
        """Keras Model.save_weights (train.py:88): a path without an .h5 / .npz suffix
        writes a TensorFlow checkpoint (prefix.index + prefix.data-00000-of-00001 + the
        directory's 'checkpoint' file) with Keras object-based keys (checkpoint.py, SURVEY.md
        §8 f row 2); '.npz' writes a numpy archive of the parameter names."""
        fmt = save_format or ("npz" if path.endswith(".npz") else
                              "h5" if path.endswith((".h5", ".keras")) else "tf")
        if fmt == "h5":
            raise NotImplementedError("HDF5 weights need h5py, which is not installed; use the "
                                      "TensorFlow checkpoint format (no suffix)")
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        if fmt == "npz":
            np.savez(path if path.endswith(".npz") else path + ".npz", **self.store.state())
        else:
            from .checkpoint import save_keras_checkpoint
            save_keras_checkpoint(path, self.store.state(), levels=self.levels)

    def load_weights(self, path, strict=True):
        """Keras Model.load_weights: a TF checkpoint prefix (or its directory) or an .npz."""
        if os.path.exists(path + ".index") or os.path.isdir(path):
            from .checkpoint import load_keras_checkpoint
            shapes = {n: p.shape for n, p in self.store.spec.items()}
            self.store.load(load_keras_checkpoint(path, levels=self.levels, expect_shapes=shapes),
                            strict=strict)
            return
        p = path if os.path.exists(path) else path + ".npz"
        with np.load(p, allow_pickle=False) as z:
            self.store.load({k: z[k] for k in z.files}, strict=strict)


def build_flow_net(height, width, pretrained_weights_path=None, max_disp=3, seed=0,
                   device="cuda", precision="fp32", levels=4, bn_mode="inference"):
    """model.py:119-143.  ``pretrained_weights_path``: the stand-alone ResNet18 encoder's
    weights, as a TF checkpoint (Keras object-based keys, checkpoint.py) or an .npz of
    encoder parameter names; like the reference (model.py:128-129) every encoder weight must
    be matched."""
    net = FlowNet(height, width, max_disp, seed=seed, device=device, precision=precision,
                  levels=levels, bn_mode=bn_mode)
    if pretrained_weights_path is not None:
        enc_names = [p.name for p in encoder_spec(levels)]
        if (os.path.exists(pretrained_weights_path + ".index")
                or os.path.isdir(pretrained_weights_path)):
            from .checkpoint import load_keras_checkpoint
            shapes = {p.name: p.shape for p in encoder_spec(levels)}
            vals = load_keras_checkpoint(pretrained_weights_path, levels=levels,
                                         encoder_only=True, expect_shapes=shapes)
        else:
            with np.load(pretrained_weights_path, allow_pickle=False) as z:
                vals = {k: z[k] for k in z.files}
        missing = [n for n in enc_names if n not in vals]
        assert not missing, "pretrained encoder weights missing: %s" % missing[:5]
        net.store.load({n: vals[n] for n in enc_names}, strict=False)
    return net


class TwoLayerHead:
    """Config-1 plumbing model (BASELINE.json configs[0]; build-defined, not in the
    reference): conv3x3/2 6->32 + LeakyReLU(0.3) -> conv3x3 32->2, one flow at H/2, fed to
    LossLayer([flow]).  Same HIP kernels as the full net."""

    def __init__(self, height, width, seed=0, device="cuda", values=None):
        from .params import two_layer_head_spec
        self.height, self.width = height, width
        self.store = ParamStore(two_layer_head_spec(), values=values, device=device, seed=seed)
        P = self.store.params
        ver = lambda: self.store.version
        self.convs = [
            ops.ConvLayer(P["head2/conv0/kernel"], P["head2/conv0/bias"], stride=2,
                          act=ACT_LEAKY, cin_p=8, version_of=ver, name="head2/conv0"),
            ops.ConvLayer(P["head2/conv1/kernel"], P["head2/conv1/bias"], stride=1,
                          act=ACT_NONE, version_of=ver, name="head2/conv1")]

    @property
    def trainable_weights(self):
        return self.store.trainable()

    @property
    def weight_names(self):
        return [n for n, p in self.store.spec.items() if p.trainable]

    def __call__(self, batch_imgs):
        x = ops._pad_channels(batch_imgs, 8)      # (B,H,W,6) -> 8 zero-padded channels
        return [ops.conv_stack(x, self.convs)]
