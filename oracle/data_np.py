"""TEST INFRASTRUCTURE ONLY -- CPU restatement (numpy) of the reference's data path and flow
pictures, used by tests/ as the checker of the HIP kernels in image_ops.hip.  Nothing in the
product imports this module.

Rows of SURVEY.md §8 f:
  row 1  read_item (data_reader.py:45-64): cv2.imread -> cv2.resize(img, (W, H)) ->
         float32 / 255 -> - image_means (float64) -> stored into the float32 batch (:36-41);
  row 4  draw_optical_flow_color / draw_optical_flow_intensity (drawing.py:37-53).

cv2 is not installed in this image, so neither restatement is pinned against OpenCV itself
("parity unpinned" for cv2; SURVEY.md §8 c).  What is restated is OpenCV 4.x's published
algorithm, step by step in the same IEEE single / integer arithmetic:
  - resize, 8-bit, INTER_LINEAR (imgproc/resize.cpp): coordinates, 11-bit fixed-point weights,
    horizontal border columns, the 128-bit universal-intrinsic vertical pass
    ((S >> 4) * beta >> 16, + 2 >> 2), the dsize == ssize copy and the exact-2x INTER_AREA
    switch.  An IPP-dispatched OpenCV build may differ by 1 LSB.
  - cartToPolar (fastAtan32f polynomial), NORM_MINMAX normalize, HSV2BGR on 8 bits.  OpenCV's
    AVX2 dispatch of the atan polynomial uses FMA; this restates the unfused form.
PNG decoding is checked against PIL (an independent decoder; decoding is lossless, so any
correct decoder agrees bit for bit).
"""
from __future__ import annotations

import numpy as np

IMAGE_MEANS = (np.array([123.0, 117.0, 104.0]) / 255.0).reshape(1, 1, 3)   # data_reader.py:7-9
F32 = np.float32


def _coords(dsize: int, ssize: int):
    """fx = (float)((d + 0.5) * scale - 0.5), s = floor(fx), fx -= s (resize.cpp)."""
    inv = np.float64(dsize) / np.float64(ssize)
    scale = 1.0 / inv
    d = np.arange(dsize, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(F32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(F32)).astype(F32)
    return s, f


def _weights(f):
    """saturate_cast<short>({1 - f, f} * INTER_RESIZE_COEF_SCALE): cvRound (half to even)."""
    w0 = np.rint((F32(1.0) - f) * F32(2048.0)).astype(np.int64)
    w1 = np.rint(f * F32(2048.0)).astype(np.int64)
    return w0, w1


def resize_linear_u8(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """cv2.resize(img, (out_w, out_h)) for an 8-bit (h, w, c) image (INTER_LINEAR default)."""
    assert img.dtype == np.uint8 and img.ndim == 3
    sh, sw, _ = img.shape
    if (sh, sw) == (out_h, out_w):
        return img.copy()
    src = img.astype(np.int64)
    if sw == 2 * out_w and sh == 2 * out_h:                     # INTER_AREA fast path
        s = src[0::2, 0::2] + src[0::2, 1::2] + src[1::2, 0::2] + src[1::2, 1::2]
        return ((s + 2) >> 2).astype(np.uint8)
    # horizontal: clamped coordinates, border columns S[s] * 2048
    sx, fx = _coords(out_w, sw)
    neg = sx < 0
    fx = np.where(neg, F32(0), fx).astype(F32)
    sx = np.where(neg, 0, sx)
    border = sx + 1 >= sw
    right = sx >= sw - 1
    fx = np.where(right, F32(0), fx).astype(F32)
    sx = np.where(right, sw - 1, sx)
    a0, a1 = _weights(fx)
    sx1 = np.minimum(sx + 1, sw - 1)
    hr = src[:, sx, :] * a0[None, :, None] + src[:, sx1, :] * a1[None, :, None]
    hr = np.where(border[None, :, None], src[:, sx, :] * 2048, hr)
    # vertical: unclamped weights, clipped rows, SIMD rounding
    sy, fy = _coords(out_h, sh)
    b0, b1 = _weights(fy)
    r0 = np.clip(sy, 0, sh - 1)
    r1 = np.clip(sy + 1, 0, sh - 1)
    v = (((hr[r0] >> 4) * b0[:, None, None]) >> 16) + (((hr[r1] >> 4) * b1[:, None, None]) >> 16)
    v = (v + 2) >> 2
    return np.clip(v, 0, 255).astype(np.uint8)


def normalise(img_u8: np.ndarray) -> np.ndarray:
    """data_reader.py:59-63 followed by the float32 store of :40-41."""
    x = img_u8.astype(F32) / F32(255.0)
    return (x - IMAGE_MEANS).astype(F32)


def preprocess_pairs(frames, out_h: int, out_w: int) -> np.ndarray:
    """frames: [(img1_bgr_u8, img2_bgr_u8), ...] with swaps applied -> (B, H, W, 6) float32."""
    out = np.zeros((len(frames), out_h, out_w, 6), F32)
    for i, (a, b) in enumerate(frames):
        out[i, :, :, :3] = normalise(resize_linear_u8(a, out_h, out_w))
        out[i, :, :, 3:] = normalise(resize_linear_u8(b, out_h, out_w))
    return out


# ------------------------------------------------------------------- drawing.py (row 4) ----
_D = 180.0 / np.pi
P1, P3 = F32(0.9997878412794807) * F32(_D), F32(-0.3258083974640975) * F32(_D)
P5, P7 = F32(0.1555786518463281) * F32(_D), F32(-0.04432655554792128) * F32(_D)


def fast_atan_deg(y, x):
    """OpenCV fastAtan32f (atan_f32), degrees in [0, 360)."""
    y, x = y.astype(F32), x.astype(F32)
    ax, ay = np.abs(x), np.abs(y)
    eps = F32(2.220446049250313e-16)
    big = ax >= ay
    with np.errstate(invalid="ignore", divide="ignore"):
        c = np.where(big, ay / (ax + eps), ax / (ay + eps)).astype(F32)
    c2 = c * c
    p = (((P7 * c2 + P5) * c2 + P3) * c2 + P1) * c
    a = np.where(big, p, F32(90.0) - p).astype(F32)
    a = np.where(x < 0, F32(180.0) - a, a).astype(F32)
    a = np.where(y < 0, F32(360.0) - a, a).astype(F32)
    return a


def flow_color(flow: np.ndarray) -> np.ndarray:
    """draw_optical_flow_color (drawing.py:45-53) for one (h, w, 2) float32 flow -> BGR u8."""
    u, v = flow[..., 0].astype(F32), flow[..., 1].astype(F32)
    mag = np.sqrt(u * u + v * v).astype(F32)
    ang = (fast_atan_deg(v, u) * F32(np.pi / 180.0)).astype(F32)
    hue = (((ang * F32(180.0)) / F32(np.pi)) / F32(2.0)).astype(np.uint8)
    smin, smax = float(mag.min()), float(mag.max())
    scale = 255.0 * (1.0 / (smax - smin) if smax - smin > 2.220446049250313e-16 else 0.0)
    shift = 0.0 - smin * scale
    val = (mag * F32(scale) + F32(shift)).astype(F32)
    V = np.clip(val, 0, 255).astype(np.uint8)
    # HSV2RGB_b
    h = hue.astype(F32) * F32(6.0 / 180.0)
    s = F32(255.0) * F32(1.0 / 255.0)
    vv = V.astype(F32) * F32(1.0 / 255.0)
    sector = np.floor(h).astype(np.int64)
    h = (h - sector.astype(F32)).astype(F32)
    bad = (sector < 0) | (sector >= 6)
    sector = np.where(bad, 0, sector)
    h = np.where(bad, F32(0), h).astype(F32)
    tab = np.stack([vv, vv * (F32(1) - s), vv * (F32(1) - s * h), vv * (F32(1) - s * (F32(1) - h))])
    sd = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])
    out = np.empty(flow.shape[:2] + (3,), np.uint8)
    for ch in range(3):
        idx = sd[sector, ch]
        val_c = np.take_along_axis(tab, idx[None], 0)[0] * F32(255.0)
        out[..., ch] = np.clip(np.rint(val_c), 0, 255).astype(np.uint8)
    if s == 0:                                                   # not reached: S = 255
        out[...] = np.clip(np.rint(vv * F32(255.0)), 0, 255).astype(np.uint8)[..., None]
    return out


def flow_intensity(flow: np.ndarray) -> np.ndarray:
    """draw_optical_flow_intensity (drawing.py:37-42); channel 0 squared twice, as written."""
    u = flow[..., 0].astype(F32)
    m = np.sqrt(u * u + u * u).astype(F32)
    return np.minimum(m / F32(20.0), F32(1.0)).astype(F32)
