"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

A second, independent restatement of the reference warp in numpy, written as the literal
TF op sequence (meshgrid 'ij' -> stack -> tile -> cast -> add -> floor/clip -> 4x gather_nd ->
weights -> accumulate_n) of ``/root/reference/model.py:65-72`` and
``/root/reference/transformations.py:70-129``.  Used to cross-check ``ref_flow.warp_features``
(forward only).  PARITY UNPINNED (no TensorFlow in the image).
"""
import numpy as np


def gather_nd(params, indices):
    """tf.gather_nd with indices[..., 3] = (b, row, col) into a (B,H,W,C) tensor."""
    return params[indices[..., 0], indices[..., 1], indices[..., 2]]


def warp_features_np(flow, f2):
    bsz, h, w, _ = f2.shape
    ii, jj = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")      # model.py:65
    ij = np.stack([ii, jj], -1)[None]                                    # model.py:66-67
    ij = np.tile(ij, (bsz, 1, 1, 1)).astype(np.float32) + flow          # model.py:68-71
    x = ij[..., 0]                                                       # transformations.py:93
    y = ij[..., 1]                                                       # transformations.py:94
    x0 = np.floor(x).astype(np.int32); x1 = x0 + 1                       # :98-99
    y0 = np.floor(y).astype(np.int32); y1 = y0 + 1                       # :100-101
    x0 = np.clip(x0, 0, w - 1); x1 = np.clip(x1, 0, w - 1)               # :104-105
    y0 = np.clip(y0, 0, h - 1); y1 = np.clip(y1, 0, h - 1)               # :106-107
    bidx = np.tile(np.arange(bsz).reshape(bsz, 1, 1), (1, h, w))         # :76-78

    def ev(xx, yy):
        return gather_nd(f2, np.stack([bidx, yy, xx], -1))               # :79-80

    v00, v01, v10, v11 = ev(x0, y0), ev(x0, y1), ev(x1, y0), ev(x1, y1)  # :110-113
    a = x1.astype(np.float32) - x                                        # :116-120
    b = y1.astype(np.float32) - y                                        # :121
    w00 = (a * b)[..., None]; w01 = (a * (1.0 - b))[..., None]
    w10 = ((1.0 - a) * b)[..., None]; w11 = ((1.0 - a) * (1.0 - b))[..., None]
    return w00 * v00 + w01 * v01 + w10 * v10 + w11 * v11                 # :128-129
