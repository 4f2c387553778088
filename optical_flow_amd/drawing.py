"""Flow pictures (SURVEY.md §8 f row 4): the reference ``drawing.py`` with the same names, for
offline use -- ``display_training`` writes PNG files instead of opening a cv2 window.

``draw_optical_flow_color`` / ``draw_optical_flow_intensity`` run as HIP kernels on the flow
tensor the network produced (``of_flow_color`` / ``of_flow_intensity``, image_ops.hip); the
arrow overlay is host-side drawing on one small picture (as in the reference), rasterised
here without cv2: arrowedLine's geometry (tip length 0.1 of the shaft, +-45 degree barbs)
with a 2-pixel-wide brush.  cv2 is absent from this image, so pixel parity of the arrows
with cv2's anti-aliasing-free thick-line rasteriser is unpinned.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np
import torch

from ._lib import call
from .data_reader import imwrite


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def draw_optical_flow_color(optical_flow) -> np.ndarray:
    """drawing.py:45-53.  optical_flow: (h, w, 2) or (n, h, w, 2) float32 (CUDA tensor or
    numpy) -> (h, w, 3) / (n, h, w, 3) uint8 BGR (HSV coding: hue = direction, value =
    magnitude min-max normalised per picture)."""
    f = torch.as_tensor(optical_flow, dtype=torch.float32)
    single = f.dim() == 3
    f = (f[None] if single else f).cuda().contiguous()
    n, h, w, c = f.shape
    assert c == 2
    out = torch.empty((n, h, w, 3), dtype=torch.uint8, device=f.device)
    ws = torch.empty(2 * n, device=f.device)
    call("of_flow_color", C.c_void_p(f.data_ptr()), n, h, w, C.c_void_p(out.data_ptr()),
         C.c_void_p(ws.data_ptr()), _stream())
    out = out.cpu().numpy()
    return out[0] if single else out


def draw_optical_flow_intensity(optical_flow) -> np.ndarray:
    """drawing.py:37-42: min(|flow| / 20, 1) -- as written there, sqrt(u^2 + u^2)."""
    f = torch.as_tensor(optical_flow, dtype=torch.float32).cuda().contiguous()
    assert f.shape[-1] == 2
    out = torch.empty(f.shape[:-1], device=f.device)
    call("of_flow_intensity", C.c_void_p(f.data_ptr()), out.numel(), C.c_void_p(out.data_ptr()),
         _stream())
    return out.cpu().numpy()


def _stamp(image, x, y, color):
    """A 2x2 brush (thickness=2) at integer (x, y), clipped to the picture."""
    h, w, _ = image.shape
    for dy in (0, 1):
        for dx in (0, 1):
            xx, yy = x + dx - 1, y + dy - 1
            if 0 <= xx < w and 0 <= yy < h:
                image[yy, xx] = color


def _line(image, p0, p1, color):
    """8-connected Bresenham line from p0 to p1 with the 2-pixel brush."""
    x0, y0 = int(p0[0]), int(p0[1])
    x1, y1 = int(p1[0]), int(p1[1])
    dx, dy = abs(x1 - x0), -abs(y1 - y0)
    sx, sy = (1 if x0 < x1 else -1), (1 if y0 < y1 else -1)
    err = dx + dy
    while True:
        _stamp(image, x0, y0, color)
        if x0 == x1 and y0 == y1:
            break
        e2 = 2 * err
        if e2 >= dy:
            err += dy
            x0 += sx
        if e2 <= dx:
            err += dx
            y0 += sy


def arrowed_line(image, start, end, color, tip_length=0.1):
    """cv2.arrowedLine geometry: the shaft plus two barbs of tip_length * |shaft| at +-45
    degrees around the reversed direction."""
    _line(image, start, end, color)
    ang = math.atan2(start[1] - end[1], start[0] - end[0])
    tip = tip_length * math.hypot(end[0] - start[0], end[1] - start[1])
    for da in (math.pi / 4, -math.pi / 4):
        p = (int(round(end[0] + tip * math.cos(ang + da))), int(round(end[1] + tip * math.sin(ang + da))))
        _line(image, p, end, color)


ARROW_COLOR = (1.0, 0.0, 0.0)      # blue in BGR (drawing.py:14)
ARROW_GRID = (8, 15)               # arrow rows x columns (drawing.py:26-27)


def _arrow_end(x, y, flow, width, height):
    """Tip of the arrow at (x, y): the displaced point rounded half-to-even (np.round) and
    clamped into the picture."""
    tip = np.rint(np.asarray([x, y], np.float64) + np.asarray(flow, np.float64))
    return (int(min(max(tip[0], 0), width - 1)), int(min(max(tip[1], 0), height - 1)))


def draw_arrow(image, x, y, optical_flow):
    """The arrow of drawing.py:5-14: from (x, y) to (x, y) + flow, tip rounded and clipped
    to the picture, drawn in place."""
    h, w = image.shape[:2]
    arrowed_line(image, (int(x), int(y)), _arrow_end(x, y, optical_flow, w, h), ARROW_COLOR)


def _arrow_anchors(height, width):
    """Arrow origins of drawing.py:28-32: every height//8-th row and width//15-th column."""
    rows, cols = ARROW_GRID
    return [(x, y) for y in range(0, height, height // rows) for x in range(0, width, width // cols)]


def draw_all_arrows(img1, img2, optical_flow):
    """drawing.py:17-34: the mean of the two pictures (values <= 1) with the flow drawn as an
    8 x 15 grid of arrows; returns the new picture."""
    assert img1.shape == img2.shape and img1.max() <= 1 and img2.max() <= 1
    height, width = img1.shape[:2]
    assert tuple(optical_flow.shape) == (height, width, 2)
    picture = 0.5 * (img1 + img2)
    for x, y in _arrow_anchors(height, width):
        draw_arrow(picture, x, y, optical_flow[y, x])
    return picture


def resize_linear(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """cv2.resize(img, (out_w, out_h)) on a float image (INTER_LINEAR, float weights,
    half-pixel centres, border-clamped): the display-side resizes of drawing.py:61-64."""
    sh, sw = img.shape[:2]

    def axis(dsize, ssize):
        f = ((np.arange(dsize) + 0.5) * (ssize / dsize) - 0.5).astype(np.float32)
        s = np.floor(f).astype(np.int64)
        f = f - s
        f = np.where(s < 0, 0, f)
        s = np.clip(s, 0, ssize - 1)
        f = np.where(s >= ssize - 1, 0, f).astype(np.float32)
        return s, np.minimum(s + 1, ssize - 1), f

    y0, y1, fy = axis(out_h, sh)
    x0, x1, fx = axis(out_w, sw)
    fx = fx[None, :, None]
    rows0 = img[y0][:, x0] * (1 - fx) + img[y0][:, x1] * fx
    rows1 = img[y1][:, x0] * (1 - fx) + img[y1][:, x1] * fx
    fy = fy[:, None, None]
    return (rows0 * (1 - fy) + rows1 * fy).astype(img.dtype)


def display_training(batch_imgs, flows, out_dir=None, step=0):
    """drawing.py:56-66 without a window: the finest flow of batch element 0 drawn as arrows
    over the blended pair (x4 upscaled, like the reference) and as the HSV colour picture,
    written to ``out_dir`` as PNGs.  Returns the two pictures (float BGR, uint8 BGR)."""
    imgs = batch_imgs.detach().float().cpu().numpy() if torch.is_tensor(batch_imgs) else batch_imgs
    img1 = imgs[0, :, :, :3]
    img2 = imgs[1 if imgs.shape[0] > 1 else 0, :, :, 3:]   # drawing.py:59 reads element 1
    f0 = flows[0][0]
    flow = f0.detach().float().cpu().numpy() if torch.is_tensor(f0) else np.asarray(f0)
    img1_down = resize_linear(img1, flow.shape[0], flow.shape[1])
    img2_down = resize_linear(img2, flow.shape[0], flow.shape[1])
    blended_image = draw_all_arrows(img1_down, img2_down, flow)
    img_to_show = resize_linear(blended_image, flow.shape[0] * 4, flow.shape[1] * 4)
    color = draw_optical_flow_color(f0.detach() if torch.is_tensor(f0) else flow)
    if out_dir is not None:
        os.makedirs(out_dir, exist_ok=True)
        imwrite(os.path.join(out_dir, "flow_arrows_%06d.png" % step),
                np.clip(np.rint(img_to_show * 255.0), 0, 255).astype(np.uint8))
        imwrite(os.path.join(out_dir, "flow_color_%06d.png" % step), color)
    return img_to_show, color
