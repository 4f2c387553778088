"""TensorFlow checkpoint interop (SURVEY.md §8 f row 2): ``save_weights`` / ``load_weights`` in
the TF "tensor bundle" format that Keras writes for a path without an ``.h5`` suffix
(``train.py:88``: ``flow_net.save_weights(os.path.join(save_dir, 'flow_net_<epoch>',
'weights'))``; ``model.py:127-129``: ``encoder.load_weights(pretrained)`` +
``assert_existing_objects_matched()``).

On disk (TensorFlow's published tensor-bundle V2 layout, restated here -- TensorFlow is not
installed, so none of this is pinned against files TF itself wrote; "parity unpinned"):
  <prefix>.data-00000-of-00001   the tensors' raw little-endian bytes, back to back;
  <prefix>.index                 a LevelDB-format table (sorted keys, prefix-compressed
                                 blocks with restart points, masked-CRC32C block trailers,
                                 index block, 48-byte footer with magic 0xdb4775248b80fb57)
                                 mapping "" -> BundleHeaderProto and each tensor key ->
                                 BundleEntryProto (dtype, shape, offset, size, masked CRC32C);
  <dir>/checkpoint               the text CheckpointState naming the latest prefix.
The protobuf messages are encoded by hand (field numbers from tensor_bundle.proto,
tensor_shape.proto, versions.proto, trackable_object_graph.proto).  CRC32C is native
(of_crc32c in liboflow.so).

Keys.  Keras writes object-based keys: ``<path>/.ATTRIBUTES/VARIABLE_VALUE`` where <path>
walks ``layer_with_weights-<k>`` children (a functional model numbers the layers that own
weights, in ``model.layers`` order) down to the variable's attribute name, plus a
``_CHECKPOINTABLE_OBJECT_GRAPH`` string tensor describing that object graph.  For the
reference graph ``model.layers`` is depth-ordered: the ResNet18 encoder sub-model is
``layer_with_weights-0`` and the 24 flow-module convs follow in level / conv order
(``model.py:134-137``, each head a chain).  Inside the encoder the order is conv1,
layer1_bn, then per residual block conv_a, bn_a, conv_b, bn_b, proj, bn_proj -- the block
layers come from the absent ``resnet`` submodule, so that order is assumption a3 (SURVEY.md
§8 a3), like the block itself.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _lib

MAGIC = 0xDB4775248B80FB57
MASK_DELTA = 0xA282EAD8
VAR_SUFFIX = "/.ATTRIBUTES/VARIABLE_VALUE"
OBJECT_GRAPH_KEY = "_CHECKPOINTABLE_OBJECT_GRAPH"
DATA_SUFFIX = ".data-00000-of-00001"
BLOCK_SIZE = 262144            # TF table::Options default
RESTART_INTERVAL = 16

# tensorflow/core/framework/types.proto
DT_FLOAT, DT_DOUBLE, DT_INT32, DT_STRING, DT_INT64, DT_BOOL, DT_HALF = 1, 2, 3, 7, 9, 10, 19
NP_OF_DT = {DT_FLOAT: np.float32, DT_DOUBLE: np.float64, DT_INT32: np.int32,
            DT_INT64: np.int64, DT_BOOL: np.bool_, DT_HALF: np.float16}
DT_OF_NP = {np.dtype(v): k for k, v in NP_OF_DT.items()}


# ------------------------------------------------------------------------------ CRC32C ----
def crc32c(data, crc: int = 0) -> int:
    """CRC32C of bytes / a numpy array, continuing from crc (native of_crc32c)."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        return _lib.lib().of_crc32c(C.c_void_p(a.ctypes.data), a.nbytes, crc) if a.nbytes else crc
    b = bytes(data)
    return _lib.lib().of_crc32c(C.c_char_p(b), len(b), crc) if b else crc


def mask(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + MASK_DELTA) & 0xFFFFFFFF


def unmask(m: int) -> int:
    rot = (m - MASK_DELTA) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---------------------------------------------------------------------- protobuf wire ----
def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _get_varint(buf, pos: int) -> Tuple[int, int]:
    shift = val = 0
    while True:
        b = buf[pos]
        pos += 1
        val |= (b & 0x7F) << shift
        if not b & 0x80:
            return val, pos
        shift += 7
        if shift > 63:
            raise ValueError("checkpoint: malformed varint")


def _pb_varint(field: int, v: int) -> bytes:
    return _varint(field << 3) + _varint(v) if v else b""


def _pb_bytes(field: int, b: bytes, always: bool = False) -> bytes:
    return _varint(field << 3 | 2) + _varint(len(b)) + b if (b or always) else b""


def _pb_fixed32(field: int, v: int) -> bytes:
    return _varint(field << 3 | 5) + struct.pack("<I", v)


def _pb_parse(buf: bytes) -> Dict[int, list]:
    out: Dict[int, list] = {}
    pos = 0
    while pos < len(buf):
        key, pos = _get_varint(buf, pos)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _get_varint(buf, pos)
        elif wt == 2:
            ln, pos = _get_varint(buf, pos)
            v = bytes(buf[pos:pos + ln])
            pos += ln
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        else:
            raise ValueError("checkpoint: unsupported protobuf wire type %d" % wt)
        out.setdefault(field, []).append(v)
    return out


# ------------------------------------------------------------------ LevelDB-format table --
def _block(entries: List[Tuple[bytes, bytes]], restart_interval: int) -> bytes:
    out = bytearray()
    restarts = []
    prev = b""
    for i, (k, v) in enumerate(entries):
        if i % restart_interval == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        prev = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def _handle(offset: int, size: int) -> bytes:
    return _varint(offset) + _varint(size)


def write_table(path: str, items: List[Tuple[bytes, bytes]]):
    """A LevelDB/TF table with keys in byte order (no compression)."""
    keys = [k for k, _ in items]
    assert keys == sorted(keys) and len(set(keys)) == len(keys), "table keys must be sorted, unique"
    f = bytearray()

    def emit(contents: bytes) -> bytes:
        off = len(f)
        f.extend(contents)
        f.append(0)                                      # kNoCompression
        f.extend(struct.pack("<I", mask(crc32c(contents + b"\x00"))))
        return _handle(off, len(contents))

    index = []
    cur: List[Tuple[bytes, bytes]] = []
    cur_bytes = 0
    for k, v in items:
        cur.append((k, v))
        cur_bytes += len(k) + len(v) + 8
        if cur_bytes >= BLOCK_SIZE:
            index.append((cur[-1][0], emit(_block(cur, RESTART_INTERVAL))))
            cur, cur_bytes = [], 0
    if cur:
        index.append((cur[-1][0], emit(_block(cur, RESTART_INTERVAL))))
    meta = emit(_block([], 1))
    idx = emit(_block(index, 1))
    footer = (meta + idx).ljust(40, b"\x00") + struct.pack("<Q", MAGIC)
    f.extend(footer)
    with open(path, "wb") as fh:
        fh.write(bytes(f))


def _read_block(data: bytes, handle: bytes, verify: bool = True) -> List[Tuple[bytes, bytes]]:
    off, p = _get_varint(handle, 0)
    size, _ = _get_varint(handle, p)
    if off + size + 5 > len(data):
        raise ValueError("checkpoint index: block past end of file")
    contents = data[off:off + size]
    if data[off + size] != 0:
        raise ValueError("checkpoint index: compressed blocks are not supported")
    if verify:
        stored = struct.unpack_from("<I", data, off + size + 1)[0]
        if unmask(stored) != crc32c(contents + b"\x00"):
            raise ValueError("checkpoint index: block CRC mismatch")
    nres = struct.unpack_from("<I", contents, size - 4)[0]
    end = size - 4 - 4 * nres
    out = []
    pos = 0
    prev = b""
    while pos < end:
        shared, pos = _get_varint(contents, pos)
        nonshared, pos = _get_varint(contents, pos)
        vlen, pos = _get_varint(contents, pos)
        key = prev[:shared] + contents[pos:pos + nonshared]
        pos += nonshared
        out.append((key, contents[pos:pos + vlen]))
        pos += vlen
        prev = key
    return out


def read_table(path: str, verify: bool = True) -> List[Tuple[bytes, bytes]]:
    with open(path, "rb") as fh:
        data = fh.read()
    if len(data) < 48 or struct.unpack_from("<Q", data, len(data) - 8)[0] != MAGIC:
        raise ValueError("%s: not a TensorFlow table (bad footer magic)" % path)
    footer = data[len(data) - 48:len(data) - 8]
    _, p = _get_varint(footer, 0)
    _, p = _get_varint(footer, p)                        # metaindex handle (unused)
    idx_handle = footer[p:]
    items = []
    for _, h in _read_block(data, idx_handle, verify):
        items += _read_block(data, h, verify)
    return items


# ------------------------------------------------------------------------ tensor bundle ----
def _shape_proto(shape) -> bytes:
    return b"".join(_pb_bytes(2, _pb_varint(1, int(d)), always=True) for d in shape)


def _entry_proto(dtype: int, shape, offset: int, size: int, crc: int) -> bytes:
    return (_pb_varint(1, dtype) + _pb_bytes(2, _shape_proto(shape), always=True) +
            _pb_varint(4, offset) + _pb_varint(5, size) + _pb_fixed32(6, mask(crc)))


def _string_tensor_bytes(strings: List[bytes]) -> Tuple[bytes, int]:
    """tensor_bundle's string layout: varint64 lengths, masked CRC32C of the lengths (as
    uint64), the bytes; returns (bytes, entry crc)."""
    lens = b"".join(_varint(len(s)) for s in strings)
    crc = 0
    for s in strings:
        crc = crc32c(struct.pack("<Q", len(s)), crc)
    lc = struct.pack("<I", mask(crc))
    crc = crc32c(lc, crc)
    for s in strings:
        crc = crc32c(s, crc)
    return lens + lc + b"".join(strings), crc


def write_bundle(prefix: str, tensors: "OrderedDict[str, object]"):
    """tensors: key -> numpy array, or -> bytes for a scalar DT_STRING tensor."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    entries = []
    off = 0
    with open(prefix + DATA_SUFFIX, "wb") as fh:
        for key in sorted(tensors, key=lambda k: k.encode()):
            v = tensors[key]
            if isinstance(v, (bytes, bytearray)):
                raw, crc = _string_tensor_bytes([bytes(v)])
                dtype, shape = DT_STRING, ()
            else:
                a = np.asarray(v)                # (ascontiguousarray would make 0-d 1-d)
                if not a.flags.c_contiguous:
                    a = a.copy(order="C")
                if a.dtype not in DT_OF_NP:
                    raise TypeError("checkpoint: unsupported dtype %s for %s" % (a.dtype, key))
                a = a.astype(a.dtype.newbyteorder("<"), copy=False)
                raw = a.tobytes()
                crc = crc32c(raw)
                dtype, shape = DT_OF_NP[a.dtype], a.shape
            fh.write(raw)
            entries.append((key.encode(), _entry_proto(dtype, shape, off, len(raw), crc)))
            off += len(raw)
    header = _pb_varint(1, 1) + _pb_bytes(3, _pb_varint(1, 1), always=True)  # 1 shard, v1
    write_table(prefix + ".index", [(b"", header)] + entries)


def read_bundle(prefix: str, verify: bool = True) -> "OrderedDict[str, object]":
    """key -> numpy array (DT_STRING scalars -> bytes)."""
    items = read_table(prefix + ".index", verify)
    if not items or items[0][0] != b"":
        raise ValueError("%s.index: bundle header missing" % prefix)
    hdr = _pb_parse(items[0][1])
    if hdr.get(1, [1])[0] != 1:
        raise ValueError("%s: multi-shard bundles are not supported" % prefix)
    if hdr.get(2, [0])[0] != 0:
        raise ValueError("%s: big-endian bundles are not supported" % prefix)
    with open(prefix + DATA_SUFFIX, "rb") as fh:
        data = fh.read()
    out = OrderedDict()
    for key, val in items[1:]:
        e = _pb_parse(val)
        if 7 in e:
            raise ValueError("%s: sliced (partitioned) variables are not supported" % key)
        dtype = e.get(1, [0])[0]
        shape = tuple(_pb_parse(dm).get(1, [0])[0] for dm in _pb_parse(e.get(2, [b""])[0]).get(2, []))
        off, size = e.get(4, [0])[0], e.get(5, [0])[0]
        raw = data[off:off + size]
        if len(raw) != size:
            raise ValueError("%s: tensor bytes past the end of the data file" % key.decode())
        name = key.decode()
        if dtype == DT_STRING:
            n = int(np.prod(shape)) if shape else 1
            lens, pos = [], 0
            for _ in range(n):
                ln, pos = _get_varint(raw, pos)
                lens.append(ln)
            crc = 0
            for ln in lens:
                crc = crc32c(struct.pack("<Q", ln), crc)
            crc = crc32c(raw[pos:pos + 4], crc)
            pos += 4
            strs = []
            for ln in lens:
                strs.append(raw[pos:pos + ln])
                crc = crc32c(raw[pos:pos + ln], crc)
                pos += ln
            value = strs[0] if not shape else strs
        else:
            if dtype not in NP_OF_DT:
                raise ValueError("%s: unsupported dtype %d" % (name, dtype))
            value = np.frombuffer(raw, dtype=np.dtype(NP_OF_DT[dtype]).newbyteorder("<")) \
                .astype(NP_OF_DT[dtype]).reshape(shape)
            crc = crc32c(raw)
        if verify and 6 in e and unmask(e[6][0]) != crc:
            raise ValueError("%s: tensor CRC mismatch" % name)
        out[name] = value
    return out


def write_checkpoint_state(prefix: str):
    """The <dir>/checkpoint text file (CheckpointState) naming prefix as the latest."""
    d, base = os.path.split(prefix)
    with open(os.path.join(d or ".", "checkpoint"), "w") as fh:
        fh.write('model_checkpoint_path: "%s"\nall_model_checkpoint_paths: "%s"\n' % (base, base))


def latest_checkpoint(directory: str) -> Optional[str]:
    p = os.path.join(directory, "checkpoint")
    if not os.path.exists(p):
        return None
    for line in open(p):
        if line.startswith("model_checkpoint_path:"):
            name = line.split(":", 1)[1].strip().strip('"')
            return name if os.path.isabs(name) else os.path.join(directory, name)
    return None


# ------------------------------------------------------------ Keras object-based keys ----
_KERAS_ATTR = {"kernel": "kernel", "bias": "bias", "gamma": "gamma", "beta": "beta",
               "moving_mean": "moving_mean", "moving_variance": "moving_variance"}


def _encoder_layer_order(levels: int) -> List[str]:
    from .params import encoder_blocks
    order = ["ResNet18/conv1", "ResNet18/layer1_bn"]
    for prefix, cin, cout, stride, proj in encoder_blocks(levels):
        order += [prefix + "/conv_a", prefix + "/bn_a", prefix + "/conv_b", prefix + "/bn_b"]
        if proj:
            order += [prefix + "/proj", prefix + "/bn_proj"]
    return order


def keras_object_paths(levels: int = 4, encoder_only: bool = False) -> "OrderedDict[str, str]":
    """our parameter name -> Keras object path (without VAR_SUFFIX) for the reference
    flow_net (or, encoder_only, for the stand-alone ResNet18 encoder model that
    build_flow_net's pretrained_weights_path holds)."""
    from .params import HEAD_WIDTHS, flow_net_spec
    names = [p.name for p in flow_net_spec(levels=levels)]
    layer_path = {}
    enc_prefix = "" if encoder_only else "layer_with_weights-0/"
    for k, layer in enumerate(_encoder_layer_order(levels)):
        layer_path[layer] = "%slayer_with_weights-%d" % (enc_prefix, k)
    if not encoder_only:
        k = 1
        for level in range(levels):
            for i in range(len(HEAD_WIDTHS)):
                layer_path["flow_module_%d/conv%d" % (level, i)] = "layer_with_weights-%d" % k
                k += 1
    out = OrderedDict()
    for n in names:
        layer, attr = n.rsplit("/", 1)
        if layer in layer_path:
            out[n] = layer_path[layer] + "/" + _KERAS_ATTR[attr]
    return out


def _object_graph(paths: List[str]) -> bytes:
    """A TrackableObjectGraph for the given variable paths: node 0 is the root; every path
    component is a node; a variable node carries one VARIABLE_VALUE SerializedTensor whose
    checkpoint_key is path + VAR_SUFFIX (trackable_object_graph.proto)."""
    children: List[List[Tuple[int, str]]] = [[]]
    attrs: List[Optional[Tuple[str, str]]] = [None]
    index = {"": 0}
    for path in paths:
        parent = ""
        for comp in path.split("/"):
            node = parent + "/" + comp if parent else comp
            if node not in index:
                index[node] = len(children)
                children.append([])
                attrs.append(None)
                children[index[parent]].append((index[node], comp))
            parent = node
        attrs[index[path]] = (path, path + VAR_SUFFIX)
    nodes = b""
    for ch, at in zip(children, attrs):
        body = b"".join(_pb_bytes(1, _pb_varint(1, nid) + _pb_bytes(2, nm.encode()), always=True)
                        for nid, nm in ch)
        if at is not None:
            st = (_pb_bytes(1, b"VARIABLE_VALUE") + _pb_bytes(2, at[0].encode()) +
                  _pb_bytes(3, at[1].encode()))
            body += _pb_bytes(2, st, always=True)
        nodes += _pb_bytes(1, body, always=True)
    return nodes


def save_keras_checkpoint(prefix: str, values: Dict[str, np.ndarray], levels: int = 4,
                          encoder_only: bool = False):
    """Write values (our names) as a Keras object-based TF checkpoint at prefix."""
    paths = keras_object_paths(levels, encoder_only)
    tensors = OrderedDict()
    for name, path in paths.items():
        tensors[path + VAR_SUFFIX] = np.asarray(values[name], np.float32)
    tensors[OBJECT_GRAPH_KEY] = _object_graph(list(paths.values()))
    write_bundle(prefix, tensors)
    write_checkpoint_state(prefix)


def load_keras_checkpoint(prefix: str, levels: int = 4, encoder_only: bool = False,
                          expect_shapes: Optional[Dict[str, tuple]] = None
                          ) -> "OrderedDict[str, np.ndarray]":
    """Read a TF checkpoint written for the reference graph: object-based keys (Keras
    save_weights) or, failing those, our own parameter names used as keys.  Returns our
    names -> arrays; raises AssertionError when a weight of the model is not in the file or
    has another shape (assert_existing_objects_matched, model.py:129)."""
    if os.path.isdir(prefix):
        latest = latest_checkpoint(prefix)
        assert latest is not None, "%s: no 'checkpoint' state file" % prefix
        prefix = latest
    t = read_bundle(prefix)
    paths = keras_object_paths(levels, encoder_only)
    out = OrderedDict()
    missing = []
    for name, path in paths.items():
        key = path + VAR_SUFFIX
        if key in t:
            out[name] = t[key]
        elif name in t:
            out[name] = t[name]
        else:
            missing.append(name)
    assert not missing, "checkpoint %s does not hold %d model weights, e.g. %s" % (
        prefix, len(missing), missing[:3])
    if expect_shapes:
        bad = [(n, out[n].shape, s) for n, s in expect_shapes.items()
               if n in out and tuple(out[n].shape) != tuple(s)]
        assert not bad, "checkpoint shape mismatch: %s" % bad[:3]
    return out
