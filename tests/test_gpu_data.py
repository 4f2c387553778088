"""GPU parity of SURVEY.md §8 f rows 1 and 4 through the C ABI: the preprocess kernel
(cv2-style resize + normalise + pair packing) and the native AsyncReader's get_batch against
the numpy restatement (oracle/data_np.py), bit for bit; the flow colour / intensity kernels
against the same oracle, bit for bit."""
import os

import numpy as np
import pytest
import torch

from oracle import data_np as D

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def lib():
    from optical_flow_amd import _lib
    assert torch.cuda.is_available()
    return _lib.load()


SIZES = [((375, 1242), (384, 512)),    # KITTI 2011_09_26 frame -> the bench shape
         ((376, 1241), (192, 640)),    # KITTI 2011_09_28 frame -> train.py's default shape
         ((370, 1224), (96, 320)),
         ((64, 96), (64, 96)),         # cv::resize copy
         ((64, 96), (32, 48)),         # exact 2x: INTER_AREA switch
         ((17, 29), (40, 70)),         # upscale both axes
         ((1, 1), (3, 5))]


def test_preprocess_pairs_bit_exact():
    from optical_flow_amd.data_reader import preprocess_frames
    rng = np.random.default_rng(0)
    for (sh, sw), (oh, ow) in SIZES:
        frames = []
        for _ in range(2):
            a = rng.integers(0, 256, (sh, sw, 3)).astype(np.uint8)
            b = rng.integers(0, 256, (sh + 1, sw + 2, 3)).astype(np.uint8)   # ragged in a batch
            frames.append((a, b))
        got = preprocess_frames(frames, oh, ow).cpu().numpy()
        exp = D.preprocess_pairs(frames, oh, ow)
        np.testing.assert_array_equal(got, exp, err_msg="%s -> %s" % ((sh, sw), (oh, ow)))


def test_async_reader_get_batch_bit_exact(tmp_path):
    from test_data_path import make_kitti
    from optical_flow_amd.data_reader import AsyncReader, ReaderOpts
    content = make_kitti(str(tmp_path), frames=5, size=(37, 61))
    opts = ReaderOpts(str(tmp_path), 4, 48, 64, 4, seed=3, nslots=2)
    with AsyncReader(opts) as r:
        assert r.pinned
        for _ in range(2 * r.nbatches + 1):                    # crosses two epoch wraps
            batch = r.get_batch()
            frames = []
            for pi, sw in zip(r.last_pairs, r.last_swapped):
                p1, p2 = r.data_info[pi]
                if sw:
                    p1, p2 = p2, p1
                frames.append((content[p1], content[p2]))
            torch.cuda.synchronize()
            np.testing.assert_array_equal(batch.cpu().numpy(), D.preprocess_pairs(frames, 48, 64))


def test_read_item_and_batch(tmp_path):
    from test_data_path import make_kitti
    from optical_flow_amd.data_reader import ReaderOpts, read_batch, read_item
    content = make_kitti(str(tmp_path), days=(("d", 1),), frames=3)
    paths = sorted(content)
    opts = ReaderOpts(None, 3, 16, 24, 1)
    a, b = read_item([paths[0], paths[1]], opts, swap=True)
    exp = D.preprocess_pairs([(content[paths[1]], content[paths[0]])], 16, 24)[0]
    np.testing.assert_array_equal(a.cpu().numpy(), exp[..., :3])
    np.testing.assert_array_equal(b.cpu().numpy(), exp[..., 3:])
    out = read_batch([[paths[0], paths[1]], [paths[2], paths[3]]], opts, swaps=[False, True])
    exp = D.preprocess_pairs([(content[paths[0]], content[paths[1]]),
                              (content[paths[3]], content[paths[2]])], 16, 24)
    np.testing.assert_array_equal(out[:2].cpu().numpy(), exp)
    assert out[2].abs().sum().item() == 0                       # read_batch zero-fills


def _flows(rng, n, h, w, scale):
    f = (rng.standard_normal((n, h, w, 2)) * scale).astype(np.float32)
    f[:, 0, :4] = [[0, 0], [1, 0], [0, -1], [-2, 0]]            # atan branch edges
    f[:, 1, :4] = [[3, 3], [-3, 3], [-3, -3], [3, -3]]
    return f


def test_flow_color_bit_exact():
    from optical_flow_amd.drawing import draw_optical_flow_color
    rng = np.random.default_rng(1)
    for n, h, w, scale in [(1, 24, 32, 1.0), (3, 96, 128, 8.0), (2, 192, 256, 0.05)]:
        f = _flows(rng, n, h, w, scale)
        got = draw_optical_flow_color(torch.from_numpy(f).cuda())
        for i in range(n):
            np.testing.assert_array_equal(got[i], D.flow_color(f[i]))
    zero = np.zeros((8, 8, 2), np.float32)                      # max == min: value 0
    np.testing.assert_array_equal(draw_optical_flow_color(zero), D.flow_color(zero))


def test_flow_intensity_bit_exact():
    from optical_flow_amd.drawing import draw_optical_flow_intensity
    rng = np.random.default_rng(2)
    f = _flows(rng, 2, 40, 50, 15.0)
    np.testing.assert_array_equal(draw_optical_flow_intensity(torch.from_numpy(f).cuda()),
                                  D.flow_intensity(f))


def test_display_training_writes_pngs(tmp_path):
    from PIL import Image
    from optical_flow_amd.data import synthetic_batch
    from optical_flow_amd.drawing import display_training
    batch = torch.from_numpy(synthetic_batch(2, 64, 128, seed=5)).cuda()
    rng = np.random.default_rng(3)
    flows = [torch.from_numpy(_flows(rng, 2, 32, 64, 3.0)).cuda()]
    arrows, color = display_training(batch, flows, out_dir=str(tmp_path), step=7)
    assert arrows.shape == (128, 256, 3) and color.shape == (32, 64, 3)
    a = np.asarray(Image.open(tmp_path / "flow_arrows_000007.png"))
    c = np.asarray(Image.open(tmp_path / "flow_color_000007.png"))[..., ::-1]
    assert a.shape == (128, 256, 3)
    np.testing.assert_array_equal(c, color)


def test_train_driver_on_kitti_tree(tmp_path):
    """train.py's loop shape on a KITTI-shaped tree: AsyncReader batches -> train_step ->
    display pictures every 10 batches (train.py:64-82)."""
    from test_data_path import make_kitti
    from optical_flow_amd.train import main
    root = tmp_path / "kitti"
    make_kitti(str(root), days=(("2011_09_26", 2),), frames=6, size=(40, 130))
    disp = tmp_path / "disp"
    log = tmp_path / "log.jsonl"
    main(["--kitti", str(root), "--height", "32", "--width", "64", "--batch", "2",
          "--epochs", "1", "--nworkers", "2", "--display-dir", str(disp), "--log", str(log)])
    lines = [l for l in open(log).read().splitlines() if l]
    assert len(lines) == (2 * (5 + 6)) // 2                     # nbatches = 22 pairs // 2
    import json
    assert all(np.isfinite(json.loads(l)["loss"]) for l in lines)
    assert sorted(os.listdir(disp)) == ["flow_arrows_000009.png", "flow_color_000009.png"]
