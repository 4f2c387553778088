"""Parameter specification and deterministic initialisation of the flow network.

Names and shapes follow the Keras graph the reference builds:

* encoder ``reset18_encoder`` -- ``/root/reference/model.py:10-26``: conv1 7x7/2 (+bias,
  ``kernel_regularizer`` ignored by the custom loop, P11), ``layer1_bn``, ReLU, max-pool,
  then three ``resnet_layer_simple`` stages (``model.py:18,20,22``).  The ``resnet``
  submodule that defines those stages is not vendored (``/root/reference/.gitmodules``),
  so the stage body is the standard ResNet-18 basic block (parity
  unpinned): ``[conv3x3(s)+BN+ReLU, conv3x3+BN] + shortcut(1x1/s conv + BN when
  downsampling) -> add -> ReLU``.  Keras ``Conv2D`` defaults apply (``use_bias=True``).
* decoder ``flow_module`` -- ``model.py:80-116``: six 3x3 convs (128,128,96,64,32,2) per
  pyramid level; new layers per call, so four independent heads (P12).

Kernels are HWIO (Keras layout, P14).  Init = Keras defaults: glorot-uniform kernels,
zero biases, BN gamma=1 / beta=0 / moving_mean=0 / moving_variance=1.  Values are drawn
from ``numpy.random.default_rng(seed)`` in spec order, so any machine regenerates the
same weights without shipping a checkpoint (SURVEY.md §8 d).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

HEAD_WIDTHS = (128, 128, 96, 64, 32, 2)          # model.py:104-114
# model.py:18-23; the 5th entry is the commented-out stage 5 (model.py:24-25), enabled by
# levels=5 (SURVEY.md §8 f row 3: flow4 at H/2 and a 512-channel encoder output at H/32)
ENC_STAGES = ((2, False, 64), (3, True, 128), (4, True, 256), (5, True, 512))
ENC_CHANNELS = (64, 64, 128, 256, 512)           # outputs at H/2, H/4, H/8, H/16, H/32
LEVELS = (4, 5)


@dataclass(frozen=True)
class PSpec:
    name: str
    shape: Tuple[int, ...]
    kind: str            # 'kernel' | 'bias' | 'gamma' | 'beta' | 'mean' | 'var'

    @property
    def trainable(self) -> bool:
        return self.kind in ("kernel", "bias", "gamma", "beta")

    @property
    def size(self) -> int:
        return int(np.prod(self.shape))


def _conv(prefix, k, cin, cout):
    return [PSpec(prefix + "/kernel", (k, k, cin, cout), "kernel"),
            PSpec(prefix + "/bias", (cout,), "bias")]


def _bn(prefix, c):
    return [PSpec(prefix + "/gamma", (c,), "gamma"), PSpec(prefix + "/beta", (c,), "beta"),
            PSpec(prefix + "/moving_mean", (c,), "mean"),
            PSpec(prefix + "/moving_variance", (c,), "var")]


def encoder_blocks(levels: int = 4):
    """Yield (prefix, cin, cout, stride, has_proj) for every residual block, in order."""
    assert levels in LEVELS, levels
    cin = 64
    for idx, down, cout in ENC_STAGES[:levels - 1]:
        for blk in stage_blocks(idx, cin, 2, down):
            yield blk
        cin = cout


def stage_blocks(idx: int, cin: int, nblocks: int = 2, downsample: bool = False):
    """The blocks one ``resnet_layer_simple(x, nblocks, downsample, idx)`` call creates
    (model.py:18,20,22; assumed basic stage): output channels 64 * 2^(idx-2)
    (the shape comments of model.py:19,21,23), the first block strided by 2 when downsampling
    and projected when downsampling or when the channel count changes."""
    cout = 64 << (idx - 2)
    out = []
    for j in range(nblocks):
        stride = 2 if (downsample and j == 0) else 1
        proj = j == 0 and (downsample or cin != cout)
        out.append(("ResNet18/res%d_%d" % (idx, j), cin, cout, stride, proj))
        cin = cout
    return out


def blocks_spec(blocks) -> List[PSpec]:
    s = []
    for prefix, cin, cout, stride, proj in blocks:
        s += _conv(prefix + "/conv_a", 3, cin, cout) + _bn(prefix + "/bn_a", cout)
        s += _conv(prefix + "/conv_b", 3, cout, cout) + _bn(prefix + "/bn_b", cout)
        if proj:
            s += _conv(prefix + "/proj", 1, cin, cout) + _bn(prefix + "/bn_proj", cout)
    return s


def encoder_spec(levels: int = 4) -> List[PSpec]:
    return (_conv("ResNet18/conv1", 7, 3, 64) + _bn("ResNet18/layer1_bn", 64) +
            blocks_spec(encoder_blocks(levels)))


def head_cin(level: int, max_disp: int = 3, levels: int = 4) -> int:
    """Input channels of the first head conv at pyramid level (0 = coarsest, H/2^levels)."""
    c = ENC_CHANNELS[levels - 1 - level]
    ncv = (2 * max_disp + 1) ** 2
    return c + ncv + (2 if level > 0 else 0)      # model.py:100-102 (P9)


def head_spec(level: int, max_disp: int = 3, levels: int = 4) -> List[PSpec]:
    s = []
    cin = head_cin(level, max_disp, levels)
    for i, cout in enumerate(HEAD_WIDTHS):
        s += _conv("flow_module_%d/conv%d" % (level, i), 3, cin, cout)
        cin = cout
    return s


def flow_net_spec(max_disp: int = 3, levels: int = 4) -> List[PSpec]:
    s = encoder_spec(levels)
    for level in range(levels):
        s += head_spec(level, max_disp, levels)
    return s


def two_layer_head_spec() -> List[PSpec]:
    """Config-1 plumbing head (BASELINE.json configs[0]; SURVEY.md §8 d): build-defined,
    not in the reference: conv3x3/2 6->32 + LeakyReLU(0.3) -> conv3x3 32->2."""
    return _conv("head2/conv0", 3, 6, 32) + _conv("head2/conv1", 3, 32, 2)


def init_params(spec: List[PSpec], seed: int = 0) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.default_rng(seed)
    out = OrderedDict()
    for p in spec:
        if p.kind == "kernel":
            kh, kw, cin, cout = p.shape
            limit = np.sqrt(6.0 / (kh * kw * cin + kh * kw * cout))
            out[p.name] = rng.uniform(-limit, limit, size=p.shape).astype(np.float32)
        elif p.kind in ("bias", "beta", "mean"):
            out[p.name] = np.zeros(p.shape, np.float32)
        else:  # gamma, var
            out[p.name] = np.ones(p.shape, np.float32)
    return out


def perturb_params(params, seed: int = 1, scale: float = 0.05):
    """Give biases / BN affine / moving stats non-trivial values (test helper: zero biases
    and identity BN would leave those code paths unexercised)."""
    rng = np.random.default_rng(seed)
    out = OrderedDict()
    for k, v in params.items():
        if k.endswith("/bias") or k.endswith("/beta") or k.endswith("/moving_mean"):
            v = (rng.standard_normal(v.shape) * scale).astype(np.float32)
        elif k.endswith("/gamma") or k.endswith("/moving_variance"):
            v = (1.0 + rng.uniform(-0.2, 0.2, v.shape)).astype(np.float32)
        out[k] = v
    return out
