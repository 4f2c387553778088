"""SURVEY.md §8 f row 1 (data_reader.py) on the CPU: the native PNG codec against PIL (an
independent decoder), the numpy restatement of cv2.resize / normalisation (oracle/data_np.py)
against hand-derived values and torch's bilinear resize, and the native AsyncReader's batch
bookkeeping (host hand-out, no GPU).  GPU parity of the preprocess kernel: test_gpu_data.py."""
import os
import struct
import zlib

import numpy as np
import pytest
import torch

from oracle import data_np as D

PIL = pytest.importorskip("PIL.Image")


@pytest.fixture(scope="module")
def lib():
    from optical_flow_amd import _lib, build
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    return _lib.load()


def _chunk(t, body):
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body))


def png_bytes(samples, depth, ctype, interlace=False, plte=None):
    """Minimal PNG writer for decoder coverage: filter 0 rows, optional Adam7, sub-byte depths.
    samples: (h, w, channels) integer array of raw sample values."""
    h, w, ch = samples.shape

    def rows(img):
        out = b""
        for r in img:
            flat = r.reshape(-1).astype(np.int64)
            if depth == 16:
                line = b"".join(struct.pack(">H", int(v)) for v in flat)
            elif depth == 8:
                line = bytes(int(v) for v in flat)
            else:
                bits = "".join(format(int(v), "0%db" % depth) for v in flat)
                bits += "0" * (-len(bits) % 8)
                line = bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8))
            out += b"\x00" + line
        return out

    if interlace:
        raw = b""
        for x0, y0, dx, dy in [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4),
                               (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]:
            sub = samples[y0::dy, x0::dx]
            if sub.size:
                raw += rows(sub)
    else:
        raw = rows(samples)
    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 1 if interlace else 0)
    body = _chunk(b"IHDR", ihdr)
    if plte is not None:
        body += _chunk(b"PLTE", bytes(plte.reshape(-1).tolist()))
    return b"\x89PNG\r\n\x1a\n" + body + _chunk(b"IDAT", zlib.compress(raw)) + _chunk(b"IEND", b"")


def _read(path):
    from optical_flow_amd.data_reader import imread_bgr
    return imread_bgr(str(path))


def _pil_bgr(path):
    return np.asarray(PIL.open(str(path)).convert("RGB"))[..., ::-1]


# ------------------------------------------------------------------------------ PNG codec --
@pytest.mark.parametrize("mode", ["RGB", "RGBA", "L", "LA", "P", "1"])
def test_png_decode_matches_pil(lib, tmp_path, mode):
    rng = np.random.default_rng(1)
    rgb = rng.integers(0, 256, (37, 53, 3)).astype(np.uint8)
    im = {"RGB": lambda: PIL.fromarray(rgb),
          "RGBA": lambda: PIL.fromarray(np.dstack([rgb, rgb[..., 0]])),
          "L": lambda: PIL.fromarray(rgb[..., 1]),
          "LA": lambda: PIL.fromarray(np.dstack([rgb[..., 1], rgb[..., 2]]), "LA"),
          "P": lambda: PIL.fromarray(rgb).convert("P"),
          "1": lambda: PIL.fromarray(rgb[..., 0] > 128)}[mode]()
    p = tmp_path / "x.png"
    im.save(p)
    np.testing.assert_array_equal(_read(p), _pil_bgr(p))


def test_png_decode_16bit_takes_high_byte(lib, tmp_path):
    rng = np.random.default_rng(2)
    v = rng.integers(0, 65536, (9, 11, 3))
    p = tmp_path / "x16.png"
    p.write_bytes(png_bytes(v, 16, 2))
    np.testing.assert_array_equal(_read(p), (v >> 8).astype(np.uint8)[..., ::-1])


@pytest.mark.parametrize("depth", [1, 2, 4])
def test_png_decode_subbyte_gray_scaled(lib, tmp_path, depth):
    rng = np.random.default_rng(depth)
    v = rng.integers(0, 1 << depth, (7, 13, 1))
    p = tmp_path / "g.png"
    p.write_bytes(png_bytes(v, depth, 0))
    exp = (v[..., 0] * (255 // ((1 << depth) - 1))).astype(np.uint8)
    np.testing.assert_array_equal(_read(p), np.repeat(exp[..., None], 3, 2))
    np.testing.assert_array_equal(_read(p), _pil_bgr(p))


@pytest.mark.parametrize("shape", [(1, 1), (5, 3), (17, 23), (8, 8)])
def test_png_decode_adam7(lib, tmp_path, shape):
    rng = np.random.default_rng(3)
    v = rng.integers(0, 256, shape + (3,))
    p = tmp_path / "i.png"
    p.write_bytes(png_bytes(v, 8, 2, interlace=True))
    np.testing.assert_array_equal(_read(p), v.astype(np.uint8)[..., ::-1])
    np.testing.assert_array_equal(_read(p), _pil_bgr(p))


def test_png_decode_palette_subbyte(lib, tmp_path):
    rng = np.random.default_rng(4)
    plte = rng.integers(0, 256, (16, 3))
    idx = rng.integers(0, 16, (6, 9, 1))
    p = tmp_path / "p4.png"
    p.write_bytes(png_bytes(idx, 4, 3, plte=plte))
    np.testing.assert_array_equal(_read(p), plte[idx[..., 0]].astype(np.uint8)[..., ::-1])


@pytest.mark.parametrize("filt", range(7))
def test_png_write_roundtrip(lib, tmp_path, filt):
    from optical_flow_amd.data_reader import imwrite
    rng = np.random.default_rng(filt)
    img = rng.integers(0, 256, (19, 31, 3)).astype(np.uint8)
    p = tmp_path / "w.png"
    imwrite(str(p), img, filt=filt)
    np.testing.assert_array_equal(_pil_bgr(p), img)           # PIL reads what we wrote
    np.testing.assert_array_equal(_read(p), img)
    g = img[..., 0]
    imwrite(str(p), g, filt=filt)
    np.testing.assert_array_equal(np.asarray(PIL.open(str(p))), g)


def test_png_errors(lib, tmp_path):
    from optical_flow_amd.data_reader import imwrite
    img = np.zeros((4, 4, 3), np.uint8)
    p = tmp_path / "ok.png"
    imwrite(str(p), img)
    data = p.read_bytes()
    bad = tmp_path / "bad.png"
    bad.write_bytes(data[:-20])                                 # truncated
    with pytest.raises(AssertionError, match="PNG"):
        _read(bad)
    flip = bytearray(data)
    flip[40] ^= 0xFF                                            # inside IDAT -> CRC mismatch
    bad.write_bytes(bytes(flip))
    with pytest.raises(AssertionError, match="CRC"):
        _read(bad)
    bad.write_bytes(b"GIF89a" + b"\0" * 64)
    with pytest.raises(AssertionError, match="not a PNG"):
        _read(bad)
    with pytest.raises(AssertionError, match="cannot open"):
        _read(tmp_path / "missing.png")


# ------------------------------------------------------------------ oracle: cv2.resize ----
def test_resize_kat_fixed_point():
    """Hand-derived: 1 x 3 -> 1 x 2 (scale 1.5): dst0 at f=0.25 from s=0, dst1 at f=0.75 from
    s=1; weights (1536, 512) and (512, 1536); the vertical pass with beta (2048, 0) computes
    ((S >> 4) * 2048 >> 16 + 2) >> 2."""
    img = np.array([[[10], [200], [90]]], np.uint8)
    out = D.resize_linear_u8(img, 1, 2)
    h0 = 10 * 1536 + 200 * 512
    h1 = 200 * 512 + 90 * 1536
    exp = [(((h >> 4) * 2048 >> 16) + 2) >> 2 for h in (h0, h1)]
    assert out[0, :, 0].tolist() == exp == [58, 118]


def test_resize_special_cases():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (6, 8, 3)).astype(np.uint8)
    np.testing.assert_array_equal(D.resize_linear_u8(img, 6, 8), img)        # copy
    i = img.astype(int)
    area = (i[0::2, 0::2] + i[0::2, 1::2] + i[1::2, 0::2] + i[1::2, 1::2] + 2) >> 2
    np.testing.assert_array_equal(D.resize_linear_u8(img, 3, 4), area)      # INTER_AREA


@pytest.mark.parametrize("src,dst", [((375, 1242), (384, 512)), ((376, 1241), (192, 640)),
                                     ((40, 70), (97, 33)), ((13, 9), (13, 27))])
def test_resize_close_to_float_bilinear(src, dst):
    """cv2's fixed point stays within 1 LSB of exact half-pixel bilinear (same coordinates;
    torch F.interpolate(bilinear, align_corners=False) without antialias)."""
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, src + (3,)).astype(np.uint8)
    ours = D.resize_linear_u8(img, *dst).astype(np.int64)
    t = torch.from_numpy(img).permute(2, 0, 1)[None].double()
    ref = torch.nn.functional.interpolate(t, size=dst, mode="bilinear", align_corners=False)
    ref = ref[0].permute(1, 2, 0).numpy()
    assert np.abs(ours - ref).max() <= 1.0


def test_normalise_value_contract():
    """P15: float32(u8)/255 - mean(float64), stored as float32."""
    u = np.arange(256, dtype=np.uint8).reshape(1, 256, 1).repeat(3, 2)
    out = D.normalise(u)
    exp = (u.astype(np.float32) / np.float32(255.0)).astype(np.float64) - D.IMAGE_MEANS
    np.testing.assert_array_equal(out, exp.astype(np.float32))
    assert out.dtype == np.float32
    assert abs(out[0, 123, 0]) < 1e-7 and abs(out[0, 104, 2]) < 1e-7


# --------------------------------------------------------------------- reader bookkeeping --
def make_kitti(root, days=(("2011_09_26", 2), ("2011_09_28", 1)), frames=4, size=(20, 30),
               seed=0):
    """A KITTI-raw-shaped tree: <day>/<day>_drive_000k_sync/image_0{2,3}/data/NNNNNNNNNN.png
    plus the per-day calib .txt files read_kitti skips."""
    from optical_flow_amd.data_reader import imwrite
    rng = np.random.default_rng(seed)
    content = {}
    for day, ndrives in days:
        os.makedirs(os.path.join(root, day), exist_ok=True)
        open(os.path.join(root, day, "calib_cam_to_cam.txt"), "w").close()
        for k in range(ndrives):
            drive = "%s_drive_%04d_sync" % (day, k + 1)
            for cam in ("image_02", "image_03"):
                d = os.path.join(root, day, drive, cam, "data")
                os.makedirs(d, exist_ok=True)
                for f in range(frames):
                    h, w = size[0] + (k + f) % 3, size[1] + f % 2      # ragged frame sizes
                    img = rng.integers(0, 256, (h, w, 3)).astype(np.uint8)
                    p = os.path.join(d, "%010d.png" % f)
                    imwrite(p, img)
                    content[p] = img
    return content


def test_read_kitti_listing(lib, tmp_path):
    from optical_flow_amd.data_reader import read_kitti
    make_kitti(str(tmp_path))
    pairs = read_kitti(str(tmp_path))
    # per drive: (frames - 1) temporal + frames stereo pairs; 3 drives of 4 frames
    assert len(pairs) == 3 * (3 + 4)
    drive_of = lambda p: p.split(os.sep)[-4]
    for p1, p2 in pairs:
        assert drive_of(p1) == drive_of(p2) and "image_02" in p1
    first = [p for p in pairs if drive_of(p[0]).endswith("2011_09_28_drive_0001_sync")]
    assert [os.path.basename(a) + os.path.basename(b) for a, b in first[:3]] == [
        "0000000000.png0000000001.png", "0000000001.png0000000002.png",
        "0000000002.png0000000003.png"]
    assert all("image_03" in b for _, b in first[3:])


def _reader(tmp_path, batch=4, seed=7, nworkers=3, nslots=2, content=None):
    """An AsyncReader over tmp_path's KITTI tree, written first unless ``content`` (the tree's
    frames, already on disk) is given: a reader's worker threads start decoding at once, so a
    second reader must not rewrite the files under the first one."""
    from optical_flow_amd.data_reader import AsyncReader, ReaderOpts
    if content is None:
        content = make_kitti(str(tmp_path))
    opts = ReaderOpts(str(tmp_path), batch, 16, 24, nworkers, seed=seed, nslots=nslots)
    return AsyncReader(opts, pinned=False), content


def test_async_reader_epochs_and_swaps(lib, tmp_path):
    from optical_flow_amd.data_reader import split_raw
    r, content = _reader(tmp_path)
    with r:
        n = len(r.data_info)
        assert r.nbatches == n // 4 == 5
        assert r.max_h == 22 and r.max_w == 31                      # scanned from headers
        for epoch in range(3):
            seen = []
            for _ in range(r.nbatches):
                raw = r.next_raw()
                frames = split_raw(raw, 4)
                for (a, b), pi, sw in zip(frames, r.last_pairs, r.last_swapped):
                    p1, p2 = r.data_info[pi]
                    if sw:
                        p1, p2 = p2, p1
                    np.testing.assert_array_equal(a, content[p1])
                    np.testing.assert_array_equal(b, content[p2])
                    seen.append(int(pi))
            # each epoch draws nbatches*batch distinct pairs (the remainder is dropped)
            assert len(set(seen)) == len(seen) == 20
        swaps = np.concatenate([r.last_swapped])
        assert set(swaps.tolist()) <= {0, 1}


def test_async_reader_is_deterministic(lib, tmp_path):
    a, content = _reader(tmp_path, seed=11)
    b, _ = _reader(tmp_path, seed=11, content=content)
    c, _ = _reader(tmp_path, seed=12, content=content)
    order = {}
    for name, r in (("a", a), ("b", b), ("c", c)):
        with r:
            seq = []
            for _ in range(6):
                raw = r.next_raw()
                seq.append((r.last_pairs.tolist(), r.last_swapped.tolist(), raw.sum()))
            order[name] = seq
    assert order["a"] == order["b"]
    assert order["a"] != order["c"]
    flags = [s for batch in order["a"] for s in batch[1]]
    assert 0 < sum(flags) < len(flags)                               # both orders occur


def test_async_reader_reports_bad_file(lib, tmp_path):
    from optical_flow_amd.data_reader import AsyncReader, ReaderOpts
    content = make_kitti(str(tmp_path), days=(("d", 1),), frames=3)
    pairs = [[p, p] for p in sorted(content)][:4]
    bad = str(tmp_path / "corrupt.png")
    open(bad, "wb").write(open(pairs[0][0], "rb").read()[:50])
    pairs[1] = [bad, pairs[1][1]]
    opts = ReaderOpts(None, 4, 8, 8, 2, seed=0, nslots=1, pairs=pairs, max_h=64, max_w=64)
    with AsyncReader(opts, pinned=False) as r:
        with pytest.raises(AssertionError, match="corrupt.png"):
            r.next_raw()
        with pytest.raises(AssertionError, match="corrupt.png"):     # every epoch
            r.next_raw()


def test_reader_rejects_oversized_frames(lib, tmp_path):
    from optical_flow_amd.data_reader import AsyncReader, ReaderOpts
    content = make_kitti(str(tmp_path), days=(("d", 1),), frames=2)
    pairs = [[p, p] for p in sorted(content)]
    opts = ReaderOpts(None, 2, 8, 8, 1, pairs=pairs, max_h=10, max_w=10)
    with AsyncReader(opts, pinned=False) as r:
        with pytest.raises(AssertionError, match="larger than the reader's max"):
            r.next_raw()
    with pytest.raises(AssertionError, match="fewer pairs than one batch"):
        AsyncReader(ReaderOpts(None, 8, 8, 8, 1, pairs=pairs, max_h=64, max_w=64), pinned=False)
