"""ctypes binding of liboflow.so (include/oflow.h).

This is the only place the product touches the native library.  There is NO fallback: if
the .so is missing or a call fails, an exception is raised (a silent CPU/torch path would
void every parity claim).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# OFLOW_LIB: an alternative build of the same library (A/B experiments with tools/ab_build.sh)
LIB_PATH = os.environ.get("OFLOW_LIB") or os.path.join(HERE, "liboflow.so")

OF_OK, OF_EINVAL, OF_EHIP, OF_EUNSUPPORTED, OF_ETIMEOUT = 0, 1, 2, 3, 4
OF_REDUCE_SUM, OF_REDUCE_AVG = 0, 1         # of_comm_allreduce_ex_async op
ACT_NONE, ACT_RELU, ACT_LEAKY = 0, 1, 2


class B16iIO(C.Structure):
    """of_b16i_io (include/oflow.h): the ends of one conv_halo_b16 launch."""
    _fields_ = [("a16", C.c_void_p), ("lda16", C.c_int), ("y", C.c_void_p), ("ldy", C.c_int),
                ("y16", C.c_void_p), ("ldy16", C.c_int), ("aux", C.c_void_p), ("ldr", C.c_int),
                ("act_src", C.c_void_p), ("ld_act", C.c_int), ("act16", C.c_void_p),
                ("ld_act16", C.c_int), ("col_part", C.c_void_p), ("mask_out", C.c_void_p),
                ("mask_in", C.c_void_p)]


class ConvDesc(C.Structure):
    _fields_ = [(n, C.c_int32) for n in
                ("n", "h", "w", "cin", "cin_p", "cout", "kh", "kw", "stride", "pad_top",
                 "pad_left", "ho", "wo")]


P = C.c_void_p
I = C.c_int
I64 = C.c_int64
F = C.c_float
SZ = C.c_size_t
PD = C.POINTER(ConvDesc)

# name -> (restype, argtypes); must match include/oflow.h
PROTOTYPES = {
    "of_abi_version": (I, []),
    "of_last_error": (C.c_char_p, []),
    "of_same_pads": (I, [I, I, I, C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "of_conv_wfwd_elems": (I64, [PD]),
    "of_conv_wbwd_elems": (I64, [PD]),
    "of_conv_pack_weights": (I, [PD, P, P, P, P]),
    "of_conv_pack_table_bytes": (SZ, [I]),
    "of_conv_pack_table": (I, [I, PD, C.POINTER(P), C.POINTER(P), C.POINTER(P), P]),
    "of_conv_pack_many": (I, [P, I64, P]),
    "of_conv2d_fwd_workspace": (SZ, [PD]),
    "of_conv2d_fwd": (I, [PD, P, I, P, P, P, P, P, P, F, P, I, I, F, P, I, P, I, P, SZ, P]),
    "of_conv2d_dgrad_workspace": (SZ, [PD]),
    "of_conv2d_dgrad": (I, [PD, P, I, P, P, I, I, F, P, I, P, SZ, P]),
    "of_conv2d_wgrad_workspace": (SZ, [PD]),
    "of_conv2d_wgrad": (I, [PD, P, I, P, I, P, P, I, P, SZ, P]),
    "of_conv_path": (I, [PD]),
    "of_conv_wfwd16_elems": (I64, [PD]),
    "of_conv_wbwd16_elems": (I64, [PD]),
    "of_conv_pack_weights_bf16": (I, [PD, P, P, P, P]),
    "of_conv_pack_table_ex": (I, [I, PD, C.POINTER(P), C.POINTER(P), C.POINTER(P),
                                  C.POINTER(I), P]),
    "of_conv2d_fwd_bf16_workspace": (SZ, [PD]),
    "of_conv2d_fwd_bf16": (I, [PD, P, I, P, P, P, P, P, P, F, P, I, I, F, P, I, P, I, P, SZ, P]),
    "of_conv2d_wgrad_bf16_workspace": (SZ, [PD]),
    "of_conv2d_wgrad_bf16": (I, [PD, P, I, P, I, P, P, I, P, SZ, P]),
    "of_conv2d_dgrad_bf16_workspace": (SZ, [PD]),
    "of_conv2d_dgrad_bf16": (I, [PD, P, I, P, P, I, I, F, P, I, P, SZ, P]),
    "of_conv2d_dgrad_add": (I, [PD, P, I, P, P, I, P, I, P, SZ, P]),
    "of_conv2d_dgrad_add_bf16": (I, [PD, P, I, P, P, I, P, I, P, SZ, P]),
    "of_conv_pack_weights_x3": (I, [PD, P, P, P, P]),
    "of_conv2d_fwd_x3_workspace": (SZ, [PD]),
    "of_conv2d_dgrad_x3_workspace": (SZ, [PD]),
    "of_conv2d_fwd_x3": (I, [PD, P, I, P, P, P, P, P, P, F, P, I, I, F, P, I, P, I, P, SZ, P]),
    "of_conv2d_dgrad_x3": (I, [PD, P, I, P, P, I, I, F, P, I, P, SZ, P]),
    "of_conv2d_dgrad_add_x3": (I, [PD, P, I, P, P, I, P, I, P, SZ, P]),
    "of_conv2d_wgrad_x3_workspace": (SZ, [PD]),
    "of_conv2d_wgrad_x3": (I, [PD, P, I, P, I, P, P, I, P, SZ, P]),
    "of_act_bwd": (I, [P, P, I, F, P, I64, P]),
    "of_colsum_workspace": (SZ, [I64, I]),
    "of_colsum": (I, [P, I64, I, I, P, I, P, P]),
    "of_bn_act_bwd_workspace": (SZ, [I64, I]),
    "of_bn_act_bwd": (I, [I64, I, I, P, P, P, P, P, P, F, P, P, P, P, P, I, P, P]),
    "of_min_abs_segments": (I, [P, P, I, P, P]),
    "of_maxpool_bn_act_bwd_workspace": (SZ, [I, I, I, I]),
    "of_maxpool_bn_act_bwd": (I, [I, I, I, I, P, P, P, P, P, P, P, F, P, P, P, P, I, P, P]),
    "of_maxpool2_fwd": (I, [P, I, I, I, I, P, P]),
    "of_maxpool2_bwd": (I, [P, P, I, I, I, I, P, P]),
    "of_corr_fwd_workspace": (SZ, [I, I, I, I, I]),
    "of_corr_fwd": (I, [P, I, P, I, I, I, I, I, I, P, I, P, SZ, P]),
    "of_corr_bwd": (I, [P, I, P, I, P, I, I, I, I, I, I, P, I, I, P, I, I, P]),
    "of_corr_concat_fwd": (I, [P, P, P, I, I, I, I, I, P, I, P, SZ, P]),
    "of_corr_concat_bwd": (I, [P, I, P, P, I, I, I, I, I, P, P, P, P]),
    "of_corr_concat_fwd16": (I, [P, P, P, I, I, I, I, I, P, I, P]),
    "of_corr_concat_fwd16_ok": (I, [I, I, I, I]),
    "of_warp_fwd": (I, [P, I, I, I, I, P, P, P]),
    "of_warp_bwd": (I, [P, P, I, I, I, I, P, P, P, P]),
    "of_warp_bwd_add": (I, [P, P, I, I, I, I, P, P, P, P, I, P]),
    "of_bilinear_fwd": (I, [P, I, I, I, I, P, P, P]),
    "of_bilinear_bwd": (I, [P, P, I, I, I, I, P, P, P, P]),
    "of_to_bf16_image": (I, [P, I64, I, I, P, I, P]),
    "of_conv2d_b16i_tiles": (I, [I, PD]),
    "of_conv2d_b16i_mask_bytes": (SZ, [PD]),
    "of_conv2d_b16i": (I, [I, PD, P, P, P, P, P, P, P, F, I, F, P]),
    "of_col_part_reduce": (I, [P, I, I, P, I, P]),
    "of_conv2d_wgrad_b16i_workspace": (SZ, [PD]),
    "of_conv2d_wgrad_b16i": (I, [PD, P, I, P, I, P, I, P, P, F, P, SZ, P]),
    "of_warp_bwd_det_workspace": (SZ, [I, I, I, I]),
    "of_warp_bwd_det_header": (SZ, [I, I, I, I]),
    "of_warp_bwd_det": (I, [P, P, I, I, I, I, P, I, P, P, P, I, P, SZ, P]),
    "of_upscale2x_fwd": (I, [P, I, I, I, I, F, P, I, P]),
    "of_upscale2x_bwd": (I, [P, I, I, I, I, I, F, P, I, P]),
    "of_upscale2x_bwd_ld": (I, [P, I, I, I, I, I, F, P, I, I, P]),
    "of_pyramid6": (I, [P, I, I, I, I, C.POINTER(P), P]),
    "of_split_pair": (I, [P, I, I, I, P, P]),
    "of_photo_l1_partials": (I, [I, I, I]),
    "of_photo_l1_fwd": (I, [P, P, I, I, I, P, P]),
    "of_photo_l1_bwd": (I, [P, P, I, I, I, F, P, P, P]),
    "of_photo_l1_bwd_ld": (I, [P, P, I, I, I, F, P, P, I, P]),
    "of_sum_partials": (I, [C.POINTER(P), C.POINTER(I), C.POINTER(F), I, P, P]),
    "of_adam_keras": (I, [P, P, P, P, I64, F, F, F, F, F, P]),
    "of_adam_keras_dev": (I, [P, P, P, P, I64, P, P, F, F, F, F, P]),
    "of_add_inplace": (I, [P, P, I64, P]),
    "of_copy_strided": (I, [P, I, P, I, I64, I, P]),
    "of_fill": (I, [P, F, I64, P]),
    "of_stream_wait": (I, [P, P]),
    "of_timing_enable": (I, [I]),
    "of_set_tuning": (I, [I, I]),
    "of_timing_read": (I, [I, C.POINTER(I), C.POINTER(C.c_double), C.POINTER(F)]),
    # data path (SURVEY §8 f row 1) and flow pictures (row 4)
    "of_png_info": (I, [C.c_char_p, C.POINTER(I), C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "of_png_read_bgr": (I, [C.c_char_p, P, I64, C.POINTER(I), C.POINTER(I)]),
    "of_png_write": (I, [C.c_char_p, P, I, I, I, I]),
    "of_png_scan": (I, [I, C.POINTER(C.c_char_p), I, C.POINTER(I), C.POINTER(I)]),
    "of_reader_create": (I, [I, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), I, I, I, I, I,
                             C.c_uint64, I, C.POINTER(P)]),
    "of_reader_raw_bytes": (I64, [P]),
    "of_reader_nbatches": (I, [P]),
    "of_reader_next": (I, [P, P, I64, P, I, I, C.POINTER(C.c_int32), C.POINTER(C.c_int32), P]),
    "of_reader_next_host": (I, [P, P, I64, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "of_reader_destroy": (I, [P]),
    "of_preprocess_pairs": (I, [P, I, I, I, P, P]),
    "of_flow_color": (I, [P, I, I, I, P, P, P]),
    "of_flow_intensity": (I, [P, I64, P, P]),
    "of_crc32c": (C.c_uint32, [P, I64, C.c_uint32]),   # checkpoint bundles (row 2)
    # inference BN folded into the backward
    "of_conv_pack_weights_bn": (I, [PD, I, P, P, P, P, P, F, P]),
    "of_conv_pack_table_bn": (I, [I, PD, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(I),
                                  C.POINTER(P), C.POINTER(P), F, P]),
    "of_conv2d_wgrad_bn_workspace": (SZ, [PD, I]),
    "of_conv2d_wgrad_bn": (I, [PD, I, P, I, P, I, P, I, P, P, F, P, SZ, P]),
    "of_conv2d_dgrad_add_act": (I, [PD, I, P, I, P, P, I, P, I, I, F, P, I, P, SZ, P]),
    "of_conv2d_dgrad_bnp_bytes": (SZ, [PD]),
    "of_conv2d_dgrad_add_act_bnp": (I, [PD, I, P, I, P, P, I, P, I, I, F, P, I, P, P, P, I, P,
                                        SZ, P, P, SZ, P]),
    "of_bn_bwd_final": (I, [P, I, I, P, P, F, P, P, P, I, P]),
    "of_bn_bwd_reduce": (I, [I64, I, I, P, P, P, P, P, P, F, P, P, P, P, I, P, P]),
    "of_maxpool_bn_relu_bwd": (I, [I, I, I, I, P, P, P, P, P, P, F, P, P, P, P, I, P, P]),
    "of_conv2d_fwd_pool": (I, [PD, I, P, I, P, P, P, P, P, P, F, I, F, P, I, P, I, P, P, SZ, P]),
    "of_photo_l1_fwd_multi": (I, [C.POINTER(P), C.POINTER(P), I, C.POINTER(I), C.POINTER(I), I, P,
                                  P]),
    "of_photo_l1_bwd_multi": (I, [C.POINTER(P), C.POINTER(P), I, C.POINTER(I), C.POINTER(I), I,
                                  C.POINTER(F), P, C.POINTER(P), C.POINTER(I), P]),
    "of_stem_bwd_fused_workspace": (SZ, [PD, I]),
    "of_stem_bwd_fused": (I, [PD, I, P, I, P, P, P, P, P, P, F, P, P, P, P, I, P, SZ, P]),
    # BatchNormalization in training mode (bn_mode="training")
    "of_bn_train_workspace": (SZ, [I64, I, I]),
    "of_bn_train_stats": (I, [I64, I, I, P, F, F, P, P, P, P, P, P]),
    "of_bn_train_apply": (I, [I64, I, I, P, P, P, P, P, P, I, P, P]),
    "of_bn_train_bwd": (I, [I64, I, I, I, P, P, P, P, P, P, P, P, P, P, I, P, P]),
    # gradient all-reduce over RCCL (SURVEY §8 b / e)
    "of_comm_id_bytes": (I, []),
    "of_comm_get_unique_id": (I, [P]),
    "of_comm_probe": (I, []),
    "of_comm_init": (I, [C.POINTER(P), P, I, I]),
    "of_comm_init_timeout": (I, [C.POINTER(P), P, I, I, C.c_double]),
    "of_comm_info": (I, [P, C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "of_comm_allreduce_async": (I, [P, P, P, I64, P]),
    "of_comm_allreduce_ex_async": (I, [P, P, P, I64, I, P]),
    "of_comm_async_error": (I, [P]),
    "of_comm_abort": (I, [P]),
    "of_comm_destroy": (I, [P, I]),
}


class OflowError(RuntimeError):
    pass


class OflowTimeout(OflowError):
    """OF_ETIMEOUT: a collective setup or wait passed its deadline (and was aborted)."""


_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """Load liboflow.so; raises if it is absent (build it with optical_flow_amd.build)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise OflowError("liboflow.so not found at %s: run `python -m optical_flow_amd.build` "
                             "(the HIP path has no fallback)" % path)
        lib = C.CDLL(path)
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.of_abi_version() != 1:
            raise OflowError("liboflow ABI mismatch")
        # OFLOW_TUNE="key=value,...": of_set_tuning switches for A/B runs (include/oflow.h)
        for kv in filter(None, os.environ.get("OFLOW_TUNE", "").split(",")):
            k, v = kv.split("=")
            if lib.of_set_tuning(int(k), int(v)) != OF_OK:
                raise OflowError("OFLOW_TUNE: " + lib.of_last_error().decode(errors="replace"))
        _lib = lib
        return lib


def lib():
    return _lib if _lib is not None else load()


def check(status: int, what: str = ""):
    if status != OF_OK:
        msg = lib().of_last_error().decode(errors="replace")
        if status == OF_EINVAL:
            raise AssertionError("%s: %s" % (what, msg))
        if status == OF_ETIMEOUT:
            raise OflowTimeout("%s timed out: %s" % (what, msg))
        raise OflowError("%s failed (%d): %s" % (what, status, msg))


def call(name: str, *args):
    st = getattr(lib(), name)(*args)
    check(st, name)
    return st
