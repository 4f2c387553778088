"""SURVEY.md §8 f row 2: TensorFlow checkpoint (tensor bundle) writer / reader on the CPU.
TensorFlow is not installed and the reference ships no checkpoint, so the format is checked
against its published structure (known-answer CRC32C, footer, header entry, entry fields)
and by round trips; parity with files TF itself wrote is unpinned."""
import os
import struct

import numpy as np
import pytest

from optical_flow_amd import checkpoint as K


@pytest.fixture(scope="module", autouse=True)
def lib():
    from optical_flow_amd import _lib, build
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    return _lib.load()


def test_crc32c_and_mask_kat():
    assert K.crc32c(b"123456789") == 0xE3069283            # CRC-32C check value
    assert K.crc32c(b"") == 0
    data = bytes(range(256)) * 5
    assert K.crc32c(data[300:], K.crc32c(data[:300])) == K.crc32c(data)
    assert K.crc32c(np.frombuffer(data, np.uint8)) == K.crc32c(data)
    for v in (0, 1, 0xE3069283, 0xFFFFFFFF):
        assert K.unmask(K.mask(v)) == v
    assert K.mask(0) == 0xA282EAD8


def test_varint_and_protobuf():
    for n in (0, 1, 127, 128, 300, 2 ** 32, 2 ** 63 + 5):
        assert K._get_varint(K._varint(n), 0) == (n, len(K._varint(n)))
    assert K._varint(300) == b"\xac\x02"                   # protobuf encoding example
    msg = K._pb_varint(1, 7) + K._pb_bytes(2, b"abc") + K._pb_fixed32(6, 0xDEADBEEF)
    assert K._pb_parse(msg) == {1: [7], 2: [b"abc"], 6: [0xDEADBEEF]}


def test_table_roundtrip_multiblock(tmp_path, monkeypatch):
    monkeypatch.setattr(K, "BLOCK_SIZE", 512)              # force many data blocks
    items = sorted((("layer_with_weights-%d/kernel/x%03d" % (i % 7, i)).encode(), bytes([i % 251]) * (i % 37))
                   for i in range(300))
    p = str(tmp_path / "t.index")
    K.write_table(p, items)
    assert K.read_table(p) == items
    raw = open(p, "rb").read()
    assert struct.unpack("<Q", raw[-8:])[0] == 0xDB4775248B80FB57
    bad = bytearray(raw)
    bad[10] ^= 1
    open(p, "wb").write(bytes(bad))
    with pytest.raises(ValueError, match="CRC"):
        K.read_table(p)


def test_bundle_roundtrip_and_layout(tmp_path):
    rng = np.random.default_rng(0)
    t = {"b/kernel": rng.standard_normal((3, 3, 4, 5)).astype(np.float32),
         "a/bias": np.arange(5, dtype=np.float32),
         "c/step": np.array(7, np.int64),
         "d/double": rng.standard_normal(4),
         K.OBJECT_GRAPH_KEY: b"\x0a\x00graph bytes"}
    prefix = str(tmp_path / "ck" / "weights")
    K.write_bundle(prefix, t)
    back = K.read_bundle(prefix)
    assert list(back) == sorted(t)                         # keys sorted bytewise
    for k, v in t.items():
        if isinstance(v, bytes):
            assert back[k] == v
        else:
            assert back[k].dtype == v.dtype and back[k].shape == v.shape
            np.testing.assert_array_equal(back[k], v)
    # header entry (key "") first: 1 shard, little endian, version producer 1
    items = K.read_table(prefix + ".index")
    assert items[0][0] == b""
    hdr = K._pb_parse(items[0][1])
    assert hdr[1] == [1] and 2 not in hdr and K._pb_parse(hdr[3][0]) == {1: [1]}
    # an entry: DT_FLOAT, shape dims, offset/size into the data file, masked CRC32C
    e = K._pb_parse(dict(items)[b"b/kernel"])
    assert e[1] == [K.DT_FLOAT]
    dims = [K._pb_parse(d)[1][0] for d in K._pb_parse(e[2][0])[2]]
    assert dims == [3, 3, 4, 5]
    data = open(prefix + K.DATA_SUFFIX, "rb").read()
    off, size = e.get(4, [0])[0], e[5][0]
    assert size == 3 * 3 * 4 * 5 * 4
    assert data[off:off + size] == t["b/kernel"].tobytes()
    assert K.unmask(e[6][0]) == K.crc32c(t["b/kernel"].tobytes())
    # corrupt the tensor bytes -> CRC mismatch
    bad = bytearray(data)
    bad[off] ^= 0x40
    open(prefix + K.DATA_SUFFIX, "wb").write(bytes(bad))
    with pytest.raises(ValueError, match="CRC"):
        K.read_bundle(prefix)


def test_keras_object_paths():
    from optical_flow_amd.params import encoder_spec, flow_net_spec
    for levels in (4, 5):
        paths = K.keras_object_paths(levels)
        spec = flow_net_spec(levels=levels)
        assert list(paths) == [p.name for p in spec]
        assert len(set(paths.values())) == len(paths)
        assert paths["ResNet18/conv1/kernel"] == "layer_with_weights-0/layer_with_weights-0/kernel"
        assert paths["ResNet18/layer1_bn/moving_variance"] == \
            "layer_with_weights-0/layer_with_weights-1/moving_variance"
        assert paths["flow_module_0/conv0/kernel"] == "layer_with_weights-1/kernel"
        assert paths["flow_module_%d/conv5/bias" % (levels - 1)] == \
            "layer_with_weights-%d/bias" % (6 * levels)
        enc = K.keras_object_paths(levels, encoder_only=True)
        assert list(enc) == [p.name for p in encoder_spec(levels)]
        assert enc["ResNet18/conv1/kernel"] == "layer_with_weights-0/kernel"


def test_keras_checkpoint_roundtrip(tmp_path):
    from optical_flow_amd.params import encoder_spec, flow_net_spec, init_params
    vals = init_params(flow_net_spec(), 3)
    prefix = str(tmp_path / "flow_net_0" / "weights")
    K.save_keras_checkpoint(prefix, vals)
    assert open(str(tmp_path / "flow_net_0" / "checkpoint")).read().startswith(
        'model_checkpoint_path: "weights"')
    raw = K.read_bundle(prefix)
    assert "layer_with_weights-3/kernel" + K.VAR_SUFFIX in raw
    back = K.load_keras_checkpoint(str(tmp_path / "flow_net_0"))    # directory -> latest
    assert list(back) == list(vals)
    for k in vals:
        np.testing.assert_array_equal(back[k], vals[k])
    # object graph: root's children are the weighted layers, variables carry checkpoint keys
    g = K._pb_parse(raw[K.OBJECT_GRAPH_KEY])[1]
    root = K._pb_parse(g[0])
    names = [K._pb_parse(c)[2][0].decode() for c in root[1]]
    assert names[:2] == ["layer_with_weights-0", "layer_with_weights-1"]
    keys = set()
    for node in g:
        for a in K._pb_parse(node).get(2, []):
            keys.add(K._pb_parse(a)[3][0].decode())
    assert keys == {k for k in raw if k != K.OBJECT_GRAPH_KEY}
    # encoder-only checkpoint (build_flow_net's pretrained_weights_path)
    enc = {p.name: vals[p.name] for p in encoder_spec()}
    K.save_keras_checkpoint(str(tmp_path / "enc" / "ckpt"), enc, encoder_only=True)
    got = K.load_keras_checkpoint(str(tmp_path / "enc" / "ckpt"), encoder_only=True)
    assert list(got) == list(enc)
    # a model weight absent from the file is an error (assert_existing_objects_matched)
    with pytest.raises(AssertionError, match="does not hold"):
        K.load_keras_checkpoint(str(tmp_path / "enc" / "ckpt"))
    shapes = {p.name: p.shape for p in encoder_spec()}
    shapes["ResNet18/conv1/kernel"] = (3, 3, 3, 64)
    with pytest.raises(AssertionError, match="shape mismatch"):
        K.load_keras_checkpoint(str(tmp_path / "enc" / "ckpt"), encoder_only=True,
                                expect_shapes=shapes)
