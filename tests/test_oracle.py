"""The CPU oracle (oracle/ref_flow.py) pinned by hand-derived known-answer tests of the
TensorFlow op semantics the reference relies on, and by a second
numpy restatement of the warp.  Parity unpinned against TF itself (not installed)."""
import numpy as np
import pytest
import torch

from oracle import ref_flow as R
from oracle.warp_np import warp_features_np


def test_same_pads_tf_rule():
    # P3: stride 2 on even n -> total pad max(k-2, 0), floor before / ceil after
    assert R.same_pads(384, 7, 2) == (2, 3)
    assert R.same_pads(96, 3, 2) == (0, 1)
    assert R.same_pads(96, 1, 2) == (0, 0)
    assert R.same_pads(48, 3, 1) == (1, 1)
    assert R.same_pads(7, 3, 2) == (1, 1)      # odd input: ceil(7/2)=4 -> total 2


def test_conv_same_matches_explicit_loop():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((1, 6, 7, 2))
    w = rng.standard_normal((3, 3, 2, 3))
    b = rng.standard_normal(3)
    y = R.conv2d_same(torch.tensor(x), torch.tensor(w), torch.tensor(b), 2).numpy()
    pt, _ = R.same_pads(6, 3, 2)
    pl, _ = R.same_pads(7, 3, 2)
    ho, wo = 3, 4
    ref = np.zeros((1, ho, wo, 3))
    for oy in range(ho):
        for ox in range(wo):
            for r in range(3):
                for s in range(3):
                    iy, ix = oy * 2 - pt + r, ox * 2 - pl + s
                    if 0 <= iy < 6 and 0 <= ix < 7:
                        ref[0, oy, ox] += x[0, iy, ix] @ w[r, s]
    ref += b
    np.testing.assert_allclose(y, ref, rtol=1e-12, atol=1e-12)


def test_zero_flow_warp_is_transpose_and_clamp():
    # F6 / P1: warp(x)[i, j] = x[clip(j, H-1), clip(i, W-1)] with zero flow
    h, w = 3, 5
    x = torch.arange(h * w * 2, dtype=torch.float64).reshape(1, h, w, 2)
    out = R.warp_features(torch.zeros(1, h, w, 2, dtype=torch.float64), x)
    for i in range(h):
        for j in range(w):
            assert torch.equal(out[0, i, j], x[0, min(j, h - 1), min(i, w - 1)])


def test_warp_numpy_restatement_agrees():
    rng = np.random.default_rng(1)
    f2 = rng.standard_normal((2, 9, 13, 4)).astype(np.float32)
    flow = (rng.standard_normal((2, 9, 13, 2)) * 4).astype(np.float32)
    a = warp_features_np(flow, f2)
    b = R.warp_features(torch.tensor(flow), torch.tensor(f2)).numpy()
    np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6)


def test_warp_out_of_range_weights_use_clipped_corners():
    # P2: x = -2.5 -> x0 = x1 = 0 (clipped), a = x1 - x = 2.5, weights still sum to 1
    inp = torch.tensor([[[[1.0], [2.0]], [[3.0], [4.0]]]], dtype=torch.float64)   # 2x2
    pts = torch.tensor([[[[-2.5, 0.0]]]], dtype=torch.float64)                     # x, y
    out = R.bilinear_interpolation(inp[:, :1, :1], pts)
    assert out.item() == pytest.approx(1.0)
    pts = torch.tensor([[[[5.25, 0.5]]]], dtype=torch.float64).requires_grad_(True)
    out = R.bilinear_interpolation(inp, pts)
    # x clipped to column 1 -> d/dx = 0 (x0c == x1c); y interpolates rows 0/1 of column 1
    assert out.item() == pytest.approx(3.0)
    out.backward()
    assert pts.grad[0, 0, 0, 0].item() == 0.0
    assert pts.grad[0, 0, 0, 1].item() == pytest.approx(2.0)


def test_cost_volume_one_hot():
    # P8: a one-hot feature at (y, x) in f2 appears in channel i*7+j of pixel (y-i+3, x-j+3)
    h, w, c = 9, 9, 3
    f1 = torch.ones(1, h, w, c, dtype=torch.float64)
    f2 = torch.zeros(1, h, w, c, dtype=torch.float64)
    f2[0, 4, 4, 1] = 1.0
    cv = R.create_cost_volume(f1, f2, 3)
    nz = torch.nonzero(cv[0])
    assert len(nz) == 49
    for y, x, k in nz.tolist():
        i, j = divmod(k, 7)
        assert (y + i - 3, x + j - 3) == (4, 4)


@pytest.mark.parametrize("s", [1, 2, 3, 4])
def test_resize_down_is_two_tap_average(s):
    # P6: half-pixel resize by 2^s = mean of rows/cols f*y + f/2 - 1 and + f/2
    f = 2 ** s
    H, W = 32, 48
    x = torch.tensor(np.random.default_rng(2).standard_normal((1, H, W, 6)))
    y = R.resize_bilinear(x, H // f, W // f)
    r0 = np.arange(H // f) * f + f // 2 - 1
    c0 = np.arange(W // f) * f + f // 2 - 1
    xn = x.numpy()[0]
    ref = 0.25 * (xn[r0][:, c0] + xn[r0 + 1][:, c0] + xn[r0][:, c0 + 1] + xn[r0 + 1][:, c0 + 1])
    np.testing.assert_allclose(y.numpy()[0], ref, rtol=1e-12, atol=1e-12)


def test_upscale_times_two_and_half_pixel():
    # P7: resize x2 (half-pixel, edge-clamped) then *2.0 on both channels
    x = torch.tensor([[[[1.0, 10.0], [3.0, 30.0]]]], dtype=torch.float64)   # (1,1,2,2)
    y = R.upscale_flow(x)
    assert y.shape == (1, 2, 4, 2)
    # columns 0..3 sample 0, 0.25, 0.75, 1 of the way from pixel 0 to 1 -> *2
    np.testing.assert_allclose(y[0, 0, :, 0].numpy(), 2 * np.array([1.0, 1.5, 2.5, 3.0]))
    np.testing.assert_allclose(y[0, 1, :, 1].numpy(), 2 * np.array([10.0, 15.0, 25.0, 30.0]))


def test_leaky_relu_slope():
    x = torch.tensor([-2.0, 0.0, 3.0], dtype=torch.float64)
    assert R.leaky_relu(x).tolist() == pytest.approx([-0.6, 0.0, 3.0])


def test_keras_adam_first_step_closed_form():
    # P13: first step m = 0.1 g, v = 0.001 g^2, lr_t = lr*sqrt(1-b2)/(1-b1)
    # -> delta = lr*sqrt(.001)/.1 * .1 g / (sqrt(.001)|g| + eps) ~= lr*sign(g)
    opt = R.KerasAdam(lr=1e-3)
    p = {"w": torch.tensor([1.0, -2.0], dtype=torch.float64)}
    g = {"w": torch.tensor([0.5, -4.0], dtype=torch.float64)}
    opt.step(p, g)
    lr_t = 1e-3 * np.sqrt(1 - 0.999) / (1 - 0.9)
    ref = np.array([1.0, -2.0]) - lr_t * (0.1 * np.array([0.5, -4.0])) / (
        np.sqrt(0.001 * np.array([0.25, 16.0])) + 1e-7)
    np.testing.assert_allclose(p["w"].numpy(), ref, rtol=1e-14)


def test_bn_inference_uses_moving_stats():
    p = {"b/gamma": torch.tensor([2.0]), "b/beta": torch.tensor([0.5]),
         "b/moving_mean": torch.tensor([1.0]), "b/moving_variance": torch.tensor([3.999])}
    y = R.batchnorm_inference(torch.tensor([[3.0]]), p, "b")
    assert y.item() == pytest.approx((3.0 - 1.0) * 2.0 / 2.0 + 0.5)


def test_bn_training_batch_stats_and_moving_update():
    """batchnorm_training (P5, old/train.py:59): a hand-computed case.  One channel, values
    1, 2, 3, 6: mean 3, biased variance 3.5 (normalisation), unbiased 14/3 (moving variance);
    moving = 0.99 moving + 0.01 stat (Keras momentum 0.99)."""
    p = {"b/gamma": torch.tensor([2.0], dtype=torch.float64),
         "b/beta": torch.tensor([0.5], dtype=torch.float64),
         "b/moving_mean": torch.tensor([1.0], dtype=torch.float64),
         "b/moving_variance": torch.tensor([2.0], dtype=torch.float64)}
    x = torch.tensor([1.0, 2.0, 3.0, 6.0], dtype=torch.float64).view(1, 2, 2, 1)
    y = R.batchnorm_training(x, p, "b")
    want = (x - 3.0) / np.sqrt(3.5 + R.BN_EPS) * 2.0 + 0.5
    assert torch.allclose(y, want, rtol=1e-14, atol=1e-14)
    assert p["b/moving_mean"].item() == pytest.approx(0.99 * 1.0 + 0.01 * 3.0, rel=1e-14)
    assert p["b/moving_variance"].item() == pytest.approx(0.99 * 2.0 + 0.01 * 14.0 / 3.0,
                                                          rel=1e-14)
    # FusedBatchNormGradV3: gradients through the batch statistics (gradcheck, fresh stats)
    xg = torch.tensor(np.random.default_rng(9).standard_normal((2, 3, 3, 2)),
                      requires_grad=True)
    gg = torch.tensor([1.3, -0.7], dtype=torch.float64, requires_grad=True)
    q = {"b/gamma": gg, "b/beta": torch.tensor([0.1, 0.2], dtype=torch.float64),
         "b/moving_mean": torch.zeros(2, dtype=torch.float64),
         "b/moving_variance": torch.ones(2, dtype=torch.float64)}
    assert torch.autograd.gradcheck(lambda a, g_: R.batchnorm_training(a, dict(q, **{"b/gamma": g_}),
                                                                      "b"), (xg, gg))
    # dL/dz sums to 0 per channel (the mean is subtracted), so the conv bias gets ~0
    xg.grad = None
    R.batchnorm_training(xg, q, "b").pow(3).sum().backward()
    assert xg.grad.sum(dim=(0, 1, 2)).abs().max().item() < 1e-12


def test_photometric_loss_zero_for_identity_pairs():
    # image2 == transposed image1 and zero flows give the reference warp (transpose) ...
    # so use square images where the transpose of a symmetric image is itself
    n, H = 1, 32
    a = np.random.default_rng(3).standard_normal((H, H, 3))
    a = a + a.transpose(1, 0, 2)
    batch = np.concatenate([a, a], -1)[None]
    flows = [torch.zeros(n, H >> (s + 1), H >> (s + 1), 2, dtype=torch.float64) for s in range(4)]
    loss = R.photometric_loss(torch.tensor(batch), flows)
    assert loss.item() < 1e-12


@pytest.mark.parametrize("fn", ["warp", "corr", "upscale"])
def test_oracle_gradcheck(fn):
    rng = np.random.default_rng(4)
    if fn == "warp":
        # the sampler itself in float64 (warp_features rounds its coordinates to float32
        # like the reference, which finite differences at eps=1e-6 cannot resolve)
        f2 = torch.tensor(rng.standard_normal((1, 4, 5, 2)), requires_grad=True)
        pts = torch.tensor(rng.uniform(-1.3, 5.3, (1, 4, 5, 2)) + 0.31, requires_grad=True)
        assert torch.autograd.gradcheck(R.bilinear_interpolation, (f2, pts))
    elif fn == "corr":
        a = torch.tensor(rng.standard_normal((1, 5, 6, 3)), requires_grad=True)
        b = torch.tensor(rng.standard_normal((1, 5, 6, 3)), requires_grad=True)
        assert torch.autograd.gradcheck(lambda x, y: R.create_cost_volume(x, y, 3), (a, b))
    else:
        a = torch.tensor(rng.standard_normal((1, 3, 4, 2)), requires_grad=True)
        assert torch.autograd.gradcheck(R.upscale_flow, (a,))
