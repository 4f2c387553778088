"""Mirror of the reference ``loss.py`` (LossLayer, loss.py:5-32)."""
from __future__ import annotations

from . import ops


class LossLayer:
    """Multi-scale photometric L1: for scale s, resize the (B,H,W,6) pairs to H/2^(s+1),
    warp image2 by flows[s] with ``warp_features``' convention, mean |image1 - warped| over
    B*h*w*3, averaged over scales (P10).  HIP: one pyramid kernel per level, one fused
    warp+|diff|+reduce kernel per scale, and a d(flow) kernel per scale for the backward."""

    def __call__(self, batch_imgs, flows):
        num_scales = len(flows)
        H, W = batch_imgs.shape[1], batch_imgs.shape[2]
        for scale_idx in range(num_scales):
            scaled_height = int(H / (2.0 ** (scale_idx + 1)))
            scaled_width = int(W / (2.0 ** (scale_idx + 1)))
            assert flows[scale_idx].shape[1] == scaled_height
            assert flows[scale_idx].shape[2] == scaled_width
        assert batch_imgs.shape[3] == 6
        return ops.photometric_loss(batch_imgs, list(flows))
