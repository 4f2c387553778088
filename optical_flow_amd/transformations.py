"""Mirror of the reference ``transformations.py`` sampler (the only part of that file the
training path imports, model.py:5).  The SE(3) helpers (concat_images, Backproject/Project/
WarpLayer, transform3d, rotation helpers) are unused by the path and out of scope
(SURVEY.md §2.1)."""
from __future__ import annotations

import torch

from . import ops


def bilinear_interpolation(input_tensor, sampling_points):
    """transformations.py:85-129: input (B,h,w,C), sampling_points (B,h,w,2) absolute (x, y)
    = (column, row); x0/x1/y0/y1 clipped to the border, weights from the clipped x1/y1 and
    the unclipped point (P2).  One fused HIP kernel (fwd) / scatter + point-grad kernel (bwd)."""
    assert sampling_points.dtype == torch.float32
    return ops.bilinear(input_tensor, sampling_points)


def evaluate_tensor_on_xy_grid(input_tensor, x, y):
    """transformations.py:70-81: gather_nd(input, stack([b, y, x])).  Not on the hot path
    (the fused sampler never materialises it); kept for API parity as device indexing."""
    bsz = input_tensor.shape[0]
    bidx = torch.arange(bsz, device=input_tensor.device).view(bsz, 1, 1).expand_as(x)
    return input_tensor[bidx, y.long(), x.long()]
