"""The C-ABI library (liboflow.so) loads, exports every symbol include/oflow.h declares, and
its host-only entry points behave -- no GPU compute is launched here."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from optical_flow_amd import _lib, build
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    return _lib.load()


def declared():
    src = open(os.path.join(ROOT, "include", "oflow.h")).read()
    return sorted(set(re.findall(r"\b(of_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol(lib):
    from optical_flow_amd._lib import PROTOTYPES
    names = declared()
    assert len(names) >= 40
    for n in names:
        assert hasattr(lib, n), "liboflow.so does not export %s" % n
        assert n in PROTOTYPES, "ctypes binding missing for %s" % n
    assert set(PROTOTYPES) == set(names), "bindings for undeclared symbols"


def test_abi_version_and_errors(lib):
    assert lib.of_abi_version() == 1
    st = lib.of_same_pads(0, 3, 1, None, None, None)
    assert st == 1                                   # OF_EINVAL, no exception across the ABI
    assert b"same_pads" in lib.of_last_error()


def test_same_pads_tf_rule(lib):
    b, a, o = C.c_int(), C.c_int(), C.c_int()
    for n, k, s, exp in [(384, 7, 2, (2, 3, 192)), (96, 3, 2, (0, 1, 48)), (96, 1, 2, (0, 0, 48)),
                         (48, 3, 1, (1, 1, 48)), (7, 3, 2, (1, 1, 4))]:
        assert lib.of_same_pads(n, k, s, C.byref(b), C.byref(a), C.byref(o)) == 0
        assert (b.value, a.value, o.value) == exp


def test_packed_sizes_and_workspaces(lib):
    from optical_flow_amd._lib import ConvDesc
    d = ConvDesc(8, 192, 256, 115, 116, 128, 3, 3, 1, 1, 1, 192, 256)
    assert lib.of_conv_wfwd_elems(C.byref(d)) == 1056 * 128    # 9*116 -> 1044 -> 1056 rows
    assert lib.of_conv_wbwd_elems(C.byref(d)) == 9 * 128 * 116
    assert lib.of_conv2d_fwd_workspace(C.byref(d)) == 0          # big grid: no split-K
    assert lib.of_conv2d_wgrad_workspace(C.byref(d)) > 0
    small = ConvDesc(8, 24, 32, 305, 308, 128, 3, 3, 1, 1, 1, 24, 32)
    assert lib.of_conv2d_fwd_workspace(C.byref(small)) > 0       # 48 tiles: split-K
    s2 = ConvDesc(16, 96, 128, 64, 64, 128, 3, 3, 2, 0, 0, 48, 64)
    # stride-2 input grad: 4 phase groups with 4/2/2/1 taps, each padded to 16 rows
    assert lib.of_conv_wbwd_elems(C.byref(s2)) == (4 + 2 + 2 + 1) * 128 * 64
    bad = ConvDesc(1, 8, 8, 3, 3, 8, 3, 3, 1, 1, 1, 8, 8)        # cin_p not a multiple of 4
    assert lib.of_conv_wfwd_elems(C.byref(bad)) == -1


def test_pack_table_host_side(lib):
    from optical_flow_amd._lib import ConvDesc
    n = 2
    descs = (ConvDesc * n)(ConvDesc(1, 16, 16, 3, 4, 64, 7, 7, 2, 2, 2, 8, 8),
                           ConvDesc(1, 16, 16, 64, 64, 64, 3, 3, 1, 1, 1, 16, 16))
    ptrs = [(C.c_void_p * n)(16, 32) for _ in range(3)]
    buf = (C.c_char * lib.of_conv_pack_table_bytes(n))()
    assert lib.of_conv_pack_table(n, descs, *ptrs, buf) == 0
    total = C.c_int64.from_buffer(buf, 8).value
    e0 = lib.of_conv_wfwd_elems(C.byref(descs[0])) + lib.of_conv_wbwd_elems(C.byref(descs[0]))
    e1 = lib.of_conv_wfwd_elems(C.byref(descs[1])) + lib.of_conv_wbwd_elems(C.byref(descs[1]))
    assert total == e0 + e1


def test_photo_partials(lib):
    assert lib.of_photo_l1_partials(8, 192, 256) == (8 * 192 * 256 + 1023) // 1024


def test_product_path_refuses_cpu_tensors(lib):
    import torch
    from optical_flow_amd import ops
    with pytest.raises(RuntimeError, match="GPU only"):
        ops.warp(torch.zeros(1, 4, 4, 8), torch.zeros(1, 4, 4, 2))
