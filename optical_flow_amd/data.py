"""Synthetic image pairs with the reference's value contract.

``data_reader.py:7-9,53-63`` (P15): BGR / 255 - [123,117,104]/255, pairs packed NHWC as
``(B, H, W, 6)`` with ``[..., :3]`` = image1 and ``[..., 3:]`` = image2 (``data_reader.py:36-41``,
P16).  There is no dataset on the box, so (SURVEY.md §8 d): image1 ~ U[0,1) - mean, image2 =
image1 shifted by a random integer (dx, dy) in [-4, 4]^2 (edge-replicated) plus N(0, 0.01)
noise.  Seeds: ``default_rng(seed + rank)``.
"""
import numpy as np

IMAGE_MEANS = np.array([123.0, 117.0, 104.0], np.float32) / 255.0


def synthetic_batch(batch_size, height, width, seed=1234, rank=0):
    rng = np.random.default_rng(seed + rank)
    img1 = rng.random((batch_size, height, width, 3), dtype=np.float32)
    out = np.empty((batch_size, height, width, 6), np.float32)
    for b in range(batch_size):
        dy, dx = rng.integers(-4, 5, size=2)
        p = np.pad(img1[b], ((4, 4), (4, 4), (0, 0)), mode="edge")
        img2 = p[4 + dy:4 + dy + height, 4 + dx:4 + dx + width]
        img2 = img2 + rng.normal(0.0, 0.01, img2.shape).astype(np.float32)
        out[b, :, :, :3] = img1[b] - IMAGE_MEANS
        out[b, :, :, 3:] = img2 - IMAGE_MEANS
    return out
