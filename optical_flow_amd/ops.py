"""Autograd glue over liboflow: every forward and backward below is one or more HIP kernels
launched through the C ABI on torch's current HIP stream.  torch only allocates the tensors.

Tensors are NHWC float32 on the GPU.  Each Function cites the reference op it replaces.
"""
from __future__ import annotations

import contextlib
import os
import ctypes as C
from typing import Optional

import torch

from . import _lib
from ._lib import ACT_LEAKY, ACT_NONE, ACT_RELU, ConvDesc, call

LEAKY_ALPHA = 0.3      # keras LeakyReLU() default (model.py:105)
BN_EPS = 1e-3          # keras BatchNormalization default (model.py:14)


# Bench instrumentation: when TIMING_TAGS is a list, every conv launch appends
# (layer name, kind) in launch order, matching the hipEvent records of of_timing_read().
# With TIMING_ONLY a set of (layer name, kind), only those launches are timed (one-shot
# of_timing_enable(2) per launch) and tagged: the bench times the dominant kernel's launches
# in the timed region without event pairs around the other ~250 launches of the step.
TIMING_TAGS = None
TIMING_ONLY = None
_oneshot_armed = False


def _tag(layer, kind):
    global _oneshot_armed
    if TIMING_ONLY is not None:
        if (layer.name, kind) not in TIMING_ONLY:
            # a one-shot armed for a selected launch whose C entry returned before its
            # timing_end (e.g. an empty grid) must not time this launch instead
            if _oneshot_armed:
                _lib.lib().of_timing_enable(0)
                _oneshot_armed = False
            return
        _lib.lib().of_timing_enable(2)
        _oneshot_armed = True
    if TIMING_TAGS is not None:
        TIMING_TAGS.append((layer.name, kind))


# Deterministic mode: the feature-warp backward -- the only kernel of the step
# that adds with float atomics (the scatter-add gradient of the gathers of
# transformations.py:110-113,128) -- runs as a fixed-order window gather, or an exact int64
# fixed-point sum where no window covers the field (of_warp_bwd_det), so a train step is
# bitwise reproducible run to run, eager or replayed from a graph.  Every other reduction of
# the step is fixed-order already.  ON by default since round 5 (DESIGN.md §3 gives its cost
# against the float-atomic form); OFLOW_DETERMINISTIC=0 or set_deterministic(False) selects
# the atomic warp_bwd_gather.
DETERMINISTIC = os.environ.get("OFLOW_DETERMINISTIC", "1") == "1"


def set_deterministic(on: bool = True) -> bool:
    """Select the deterministic warp backward; returns the previous setting."""
    global DETERMINISTIC
    prev, DETERMINISTIC = DETERMINISTIC, bool(on)
    return prev


@contextlib.contextmanager
def deterministic(on: bool = True):
    prev = set_deterministic(on)
    try:
        yield
    finally:
        set_deterministic(prev)


def _workspace(nbytes: int, device):
    """Scratch for one launch: (tensor keeping it alive, pointer, bytes).  The caching
    allocator is stream-ordered, so the block is only reused after this stream's kernel."""
    if nbytes <= 0:
        return None, None, 0
    t = torch.empty((nbytes + 15) // 4, device=device)
    return t, C.c_void_p(t.data_ptr()), nbytes


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check_dev(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("optical_flow_amd ops run on the GPU only (got a %s tensor): the "
                               "HIP path has no CPU fallback" % t.device)
        if t.dtype != torch.float32:
            raise TypeError("expected float32, got %s" % t.dtype)


def _c4(c):
    return (c + 3) // 4 * 4


def same_pads(n, k, s):
    b, a, o = C.c_int(), C.c_int(), C.c_int()
    call("of_same_pads", n, k, s, C.byref(b), C.byref(a), C.byref(o))
    return b.value, a.value, o.value


# ------------------------------------------------------------------- gradient arenas ----
_GRAD_READY_HOOK = None


def set_grad_ready_hook(fn):
    """fn(param) is called once a Function has enqueued all kernels writing param's gradient
    (used by dist.GradBucketReducer to start bucket all-reduces during the backward)."""
    global _GRAD_READY_HOOK
    _GRAD_READY_HOOK = fn


def _grad_ready(*params):
    if _GRAD_READY_HOOK is not None:
        for p in params:
            if p is not None:
                _GRAD_READY_HOOK(p)


# ------------------------------------------------------- weight-gradient side stream ----
# The weight gradient of a conv is off the backward's critical path (nothing downstream reads
# it until the optimizer / all-reduce), so wgrad launches whose target is the gradient arena
# run on a second HIP stream, ordered after the kernel that produced their dy.  Small-grid
# layers (coarse flow levels, encoder stages 3-4) and the tail waves of large ones then share
# the chip with the input-gradient chain.  The current stream joins the side stream at the
# end of the autograd backward (engine callback), so .backward() returning still means every
# gradient kernel is ordered before whatever the caller enqueues next.
SIDE_STREAM_WGRAD = True
# Only layers with at most this many output pixels put their wgrad on the side stream: the
# overlap pays where grids underfill the chip (coarse flow levels, encoder stages 3-4, the
# H/8 flow level); a large layer's dgrad already fills it, and sharing the CUs would only
# stretch both kernels.  Measured A/B (tools/gpu_abenv.sh, one box, 2 rounds): fp32 B=8
# 65536 -> 131072 (adds the 96x128 level) +1.0 %, every wgrad on the side +0.6 %; bf16 B=32
# 65536 -> 524288 (the same layers at 4x the batch) +2-4 %, 131072 +0.6 %.  Per precision
# by default (the bf16 kernels are ~2.5x faster per FLOP, so the same layer underfills the
# chip at 4x the pixels); OFLOW_SIDE_MAX_PIX overrides both.
_SIDE_ENV = os.environ.get("OFLOW_SIDE_MAX_PIX")
SIDE_STREAM_MAX_PIX = int(_SIDE_ENV) if _SIDE_ENV else None
SIDE_MAX_PIX_DEFAULT = {"fp32": 131072, "bf16": 524288}


def _side_max_pix(layer) -> int:
    if SIDE_STREAM_MAX_PIX is not None:
        return SIDE_STREAM_MAX_PIX
    return SIDE_MAX_PIX_DEFAULT[layer.precision]
_SIDE = {}
_side_armed = False
# The BN reduction of a layer whose t = dL/dz the input-gradient kernel already produced
# (of_bn_bwd_reduce without t_out: dgamma, dbeta and the bias gradient only) runs on the side
# stream too; OFLOW_BN_SIDE=0 keeps it on the current stream for A/B.
BN_REDUCE_SIDE = os.environ.get("OFLOW_BN_SIDE", "1") == "1"
# Launch order inside a conv's backward.  Weight gradient first (default): a side-stream
# weight gradient then forks before the input gradient is enqueued and overlaps it.  Input
# gradient first (OFLOW_DGRAD_FIRST=1, the critical path queued earlier where the host is
# slower than the GPU) measured 2 % slower (A/B, one box: 590-593 vs 602-606 pairs/s): the
# side stream's fork then waits for the dgrad.
DGRAD_FIRST = os.environ.get("OFLOW_DGRAD_FIRST", "0") == "1"
# The stride-2 / 1x1 implicit GEMMs (res3_0 / res4_0 conv_a and proj, model.py:20,22) share
# the chip with the side stream's weight gradients in the step (half their
# alone rate).  S2_WGRAD_MAIN: their own weight gradients on the current stream; S2_JOIN: the
# current stream waits for the side stream before their input gradient.  Measured (fp32 B=8,
# two interleaved rounds, one box, gpurun_out/abs2): 651.5 / 653.6 pairs/s -> main 655.0 /
# 650.9, join 642.0 / 641.6, both 647.9 / 649.3: off (the side stream's work does not go away,
# it only moves).
S2_WGRAD_MAIN = os.environ.get("OFLOW_S2_WGRAD_MAIN", "0") == "1"
S2_JOIN = os.environ.get("OFLOW_S2_JOIN", "0") == "1"


def _gemm_layer(layer) -> bool:
    return layer.stride != 1 or (layer.kh == 1 and layer.kw == 1)


# Cross-stream waits through of_stream_wait (device-scope event fences) instead of torch's
# Stream.wait_stream (a default event: system-scope release / acquire).  OFLOW_STREAM_WAIT=torch
# keeps torch's for A/B.
NATIVE_STREAM_WAIT = os.environ.get("OFLOW_STREAM_WAIT", "native") != "torch"


def stream_wait(waiter, signaller):
    """Order stream ``waiter`` after the work enqueued so far on ``signaller``."""
    if NATIVE_STREAM_WAIT:
        call("of_stream_wait", C.c_void_p(waiter.cuda_stream), C.c_void_p(signaller.cuda_stream))
    else:
        waiter.wait_stream(signaller)


def _side_join():
    global _side_armed
    _side_armed = False
    side_join_now()
    # buffers read by side-stream kernels of this backward go back to their pools only now,
    # after the current stream has been ordered behind those streams (FlowGrad.release)
    while _DEFERRED_RELEASE:
        key, buf = _DEFERRED_RELEASE.pop()
        FlowGrad._pool.setdefault(key, []).append(buf)


_DEFERRED_RELEASE = []


def side_join_now():
    """Order each device's current stream after everything enqueued so far on its side
    streams (the end-of-backward join, also used after work launched outside a backward)."""
    if SINGLE_STREAM:
        return                       # nothing was forked (single_stream())
    for dev, s in list(_SIDE.items()) + list(_CORR_SIDE.items()) + list(_COMM.items()):
        stream_wait(torch.cuda.current_stream(dev), s)


# Single-stream mode (single_stream()): every fork point above and below keeps its work on the
# current stream -- the same kernels in the same per-stream order, which an eager step must
# reproduce bitwise (tools/eager_order_probe.py: it does, every step).  A diagnostic: a HIP
# graph CAPTURED this way replays its first launch like the eager step and diverges from the
# second on, so Trainer.graphed captures with the side streams.
SINGLE_STREAM = False


@contextlib.contextmanager
def single_stream(on: bool = True):
    """Keep every kernel of the enclosed work on the current stream (no side-stream forks)."""
    global SINGLE_STREAM, SIDE_STREAM_WGRAD, PROJ_SIDE, CORR_DF1_SIDE
    saved = (SINGLE_STREAM, SIDE_STREAM_WGRAD, PROJ_SIDE, CORR_DF1_SIDE)
    if on:
        SINGLE_STREAM, SIDE_STREAM_WGRAD, PROJ_SIDE, CORR_DF1_SIDE = True, False, False, False
    try:
        yield
    finally:
        SINGLE_STREAM, SIDE_STREAM_WGRAD, PROJ_SIDE, CORR_DF1_SIDE = saved


# The data-parallel collectives' own stream (dist.GradBucketReducer): a bucket's all-reduce
# waits for the work enqueued so far on the current stream and on the wgrad side stream (the
# kernels that wrote the bucket), and nothing but the end-of-backward join waits for it -- a
# slow peer's collective then holds back neither this rank's remaining weight gradients (side
# stream) nor its input-gradient chain (current stream).
_COMM = {}


def comm_stream(*tensors, in_backward: bool = True):
    """The collective stream of the current device, ordered after all work enqueued so far on
    the current and weight-gradient side streams.  Every collective of the communicator goes
    here -- during the backward and after it (``in_backward=False``: dist.GradBucketReducer
    .finish, whose caller joins it with side_join_now) -- so one communicator is only ever
    used on one stream (RCCL's operations on a communicator must be serialised in the same
    order on every rank; a communicator used on two streams also preceded the graph-replay
    host fault of DESIGN.md §1, round 5)."""
    global _side_armed
    cur = torch.cuda.current_stream()
    s = _COMM.get(cur.device)
    if s is None:
        s = _COMM[cur.device] = torch.cuda.Stream(cur.device)
    stream_wait(s, cur)
    side = _SIDE.get(cur.device)
    if side is not None:
        stream_wait(s, side)
    for t in tensors:
        if t is not None:
            t.record_stream(s)
    if in_backward and not _side_armed:
        _side_armed = True
        torch.autograd.Variable._execution_engine.queue_callback(_side_join)
    return s


def side_stream(*tensors):
    """The wgrad side stream of the current device, ordered after all work enqueued so far on
    the current stream; ``tensors`` (read by the side stream's kernels) are marked in use by
    it for the caching allocator."""
    global _side_armed
    cur = torch.cuda.current_stream()
    s = _SIDE.get(cur.device)
    if s is None:
        s = _SIDE[cur.device] = torch.cuda.Stream(cur.device)
    stream_wait(s, cur)
    for t in tensors:
        if t is not None:
            t.record_stream(s)
    if not _side_armed:
        _side_armed = True
        torch.autograd.Variable._execution_engine.queue_callback(_side_join)
    return s


# The cost volume's gradient w.r.t. features1 (of_corr_concat_bwd's df1) is read only by the
# encoder's backward, which runs after every flow module's: with CORR_DF1_SIDE it runs on a
# stream of its own beside the decoder's input-gradient chain (df2 -> warp backward -> the
# coarser level), and the encoder backward waits for that stream (corr_side_wait).
# Measured A/B (one box): fp32 B=8 587-589 -> 581-586 pairs/s (the main chain's convs already
# fill the chip; the memory-bound df1 only slows them), bf16 B=32 1353 -> 1363 (round 2) and
# 1422.7 / 1426.9 -> 1430.9 / 1435.9 (round 3, tools/gpu_r3q.sh).  Round 4 fused both
# gradients into one kernel (corr_bwd_fused, main stream): bf16 B=32 side 1745.8 / 1745.3 ->
# fused 1748.5 / 1750.8 (profiles/r4_late/step_ab.txt), and with the H/8 heads on images 1703.9 -> 1716.4
# (misc5, a slower box): off for both precisions.  CORR_DF1_SIDE (env OFLOW_CORR_DF1_SIDE =
# 0 / 1) forces it either way.
_DF1_ENV = os.environ.get("OFLOW_CORR_DF1_SIDE")
CORR_DF1_SIDE = None if _DF1_ENV is None else _DF1_ENV == "1"
CORR_DF1_SIDE_DEFAULT = {"fp32": False, "bf16": False}


def corr_df1_side(precision):
    return CORR_DF1_SIDE if CORR_DF1_SIDE is not None else CORR_DF1_SIDE_DEFAULT[precision]
_CORR_SIDE = {}


def corr_side_stream(*tensors):
    """The df1 stream of the current device, ordered after the current stream's work so far;
    ``tensors`` are marked in use by it for the caching allocator."""
    global _side_armed
    cur = torch.cuda.current_stream()
    s = _CORR_SIDE.get(cur.device)
    if s is None:
        s = _CORR_SIDE[cur.device] = torch.cuda.Stream(cur.device)
    stream_wait(s, cur)
    for t in tensors:
        if t is not None:
            t.record_stream(s)
    if not _side_armed:
        _side_armed = True
        torch.autograd.Variable._execution_engine.queue_callback(_side_join)
    return s


def corr_side_wait(device):
    """Order the current stream after the df1 stream (before anything reads a df1)."""
    s = _CORR_SIDE.get(torch.device(device))
    if s is not None:
        stream_wait(torch.cuda.current_stream(device), s)


def grad_target(param: torch.Tensor):
    """Where a Function writes the gradient of ``param``: straight into the parameter's
    gradient-arena view (accumulating, returns None to autograd) when the model installed
    one, else a fresh tensor that is returned to autograd."""
    g = getattr(param, "_of_grad", None)
    if g is not None:
        return g, 1, None
    t = torch.empty_like(param)
    return t, 0, t


# ====================================================================== convolution ====
# fp32 3x3 stride-1 fwd / dgrad on the split-bf16 halo-tile kernels (of_conv2d_*_x3: exact
# three-term operand split, per-product error of one fp32 rounding; tools/x3_accuracy.py and
# tests/test_gpu_kernels.py::test_conv_x3_accuracy measure it against fp64).
# OFLOW_F32_SPLIT=0 keeps every fp32 layer on the fp32 MFMA kernels.
F32_SPLIT = os.environ.get("OFLOW_F32_SPLIT", "1") == "1"
# With F32_SPLIT, the other GEMM-path fp32 layers with >= 16 input channels (the stride-2
# block convs and the 1x1 projections) take the split-bf16 implicit GEMMs (conv_gemm_x3,
# conv_wgrad_x3) too: 10-25 % faster per pass than the fp32 MFMA GEMM.  The stem (3 input
# channels, K = 49 taps x 4) measured 9 % / 37 % slower there (fwd / wgrad); its forward has a
# kernel of its own (conv_stem_x3, STEM_X3) and its weight gradient stays on the fp32 GEMM.
# OFLOW_X3_GEMM=0 keeps them all on the fp32 MFMA kernels.
X3_GEMM = os.environ.get("OFLOW_X3_GEMM", "1") == "1"
X3_GEMM_MIN_CIN = 16
STEM_X3 = os.environ.get("OFLOW_STEM_X3", "1") == "1"


def _stem_x3(layer) -> bool:
    """The shape conv_stem_x3 covers (of its stem_x3_ok): 7x7 stride 2, 4 padded input
    channels, 64 outputs."""
    return (STEM_X3 and layer.kh == 7 and layer.kw == 7 and layer.stride == 2 and
            layer.cin_p == 4 and layer.cout == 64)

class ConvLayer:
    """One ``layers.Conv2D(filters, k, strides, padding='same')`` (model.py:12,104-114) with an
    optional inference BatchNorm (model.py:14) and activation, holding references to its
    parameters (HWIO kernel, bias, BN vectors) and its per-step packed weights."""

    def __init__(self, kernel, bias, stride=1, act=ACT_NONE, alpha=LEAKY_ALPHA, bn=None,
                 cin_p=None, version_of=None, name="", precision="fp32", f32_split=None):
        self.kernel, self.bias = kernel, bias
        kh, kw, cin, cout = kernel.shape
        self.kh, self.kw, self.cin, self.cout = kh, kw, cin, cout
        self.cin_p = cin_p if cin_p is not None else _c4(cin)
        self.stride, self.act, self.alpha = stride, act, alpha
        self.bn = bn                      # (gamma, beta, moving_mean, moving_variance) or None
        self.version_of = version_of      # callable -> int, bumps when the weights change
        self.name = name
        assert precision in ("fp32", "bf16"), precision
        self.precision = precision        # "bf16": fwd / dgrad on bf16 MFMA (configs 3-5)
        self._pack_key = None
        self._wf = self._wd = None
        self._descs = {}
        self._bf16 = None
        self._mode = None
        self.f32_split = F32_SPLIT if f32_split is None else bool(f32_split)
        self.store_z = False              # BN layers: keep z for the backward (BNZGuard)
        self.bn_train = False             # BN in training mode (bn_mode="training", P5)

    def desc(self, n, h, w) -> ConvDesc:
        key = (n, h, w)
        d = self._descs.get(key)
        if d is None:
            pt, _, ho = same_pads(h, self.kh, self.stride)
            pl, _, wo = same_pads(w, self.kw, self.stride)
            d = ConvDesc(n, h, w, self.cin, self.cin_p, self.cout, self.kh, self.kw, self.stride,
                         pt, pl, ho, wo)
            self._descs[key] = d
        return d

    def bf16(self, d: ConvDesc = None) -> bool:
        """True when fwd/dgrad run the bf16 MFMA kernels (bf16 precision, GEMM-path layer)."""
        if self._bf16 is None:
            d = d or self.desc(1, 16, 16)
            self._bf16 = (self.precision == "bf16" and
                          _lib.lib().of_conv_path(C.byref(d)) == 0)
        return self._bf16

    def mode(self, d: ConvDesc = None) -> int:
        """Kernel family of fwd/dgrad: 0 fp32 MFMA, 1 bf16 MFMA, 2 fp32 on the split-bf16
        kernels (fp32 precision, GEMM-path layers, F32_SPLIT on: the halo tiles for 3x3
        stride 1, the implicit GEMM conv_gemm_x3 for the other shapes when X3_GEMM)."""
        if self._mode is None:
            tile = self.kh == 3 and self.kw == 3 and self.stride == 1
            self._mode = (1 if self.bf16(d) else
                          2 if (self.f32_split and self.precision == "fp32" and
                                (tile or _stem_x3(self) or
                                 (X3_GEMM and self.cin_p >= X3_GEMM_MIN_CIN)) and
                                _lib.lib().of_conv_path(C.byref(d or self.desc(1, 16, 16))) == 0)
                          else 0)
        return self._mode

    def alloc_packed(self, d: ConvDesc):
        lib = _lib.lib()
        dev = self.kernel.device
        m = self.mode(d)
        if m:
            planes = 3 if m == 2 else 1
            self._wf = torch.empty(planes * lib.of_conv_wfwd16_elems(C.byref(d)), device=dev,
                                   dtype=torch.bfloat16)
            self._wd = torch.empty(planes * lib.of_conv_wbwd16_elems(C.byref(d)), device=dev,
                                   dtype=torch.bfloat16)
        else:
            self._wf = torch.empty(lib.of_conv_wfwd_elems(C.byref(d)), device=dev)
            self._wd = torch.empty(lib.of_conv_wbwd_elems(C.byref(d)), device=dev)

    def packed(self, d: ConvDesc):
        key = (self.kernel.data_ptr(), self.version_of() if self.version_of else None)
        if self._wf is None:
            self.alloc_packed(d)
        if key != self._pack_key or self.version_of is None:
            if self.bn is not None and not self.bn_train:   # BN scale folded (_conv_backward)
                call("of_conv_pack_weights_bn", C.byref(d), self.mode(d), _ptr(self.kernel),
                     _ptr(self._wf), _ptr(self._wd), _ptr(self.bn[0]), _ptr(self.bn[3]),
                     BN_EPS, _stream())
            else:
                call(("of_conv_pack_weights", "of_conv_pack_weights_bf16",
                      "of_conv_pack_weights_x3")[self.mode(d)],
                     C.byref(d), _ptr(self.kernel), _ptr(self._wf), _ptr(self._wd), _stream())
            self._pack_key = key
        return self._wf, self._wd

    def fwd_entry(self, d):
        """(C entry point, workspace bytes) of the forward conv for this layer's precision."""
        lib = _lib.lib()
        if self.bf16(d):
            return "of_conv2d_fwd_bf16", lib.of_conv2d_fwd_bf16_workspace(C.byref(d))
        if self.mode(d) == 2:
            return "of_conv2d_fwd_x3", lib.of_conv2d_fwd_x3_workspace(C.byref(d))
        return "of_conv2d_fwd", lib.of_conv2d_fwd_workspace(C.byref(d))

    def wgrad_entry(self, d):
        lib = _lib.lib()
        if self.bf16(d):
            return "of_conv2d_wgrad_bf16", lib.of_conv2d_wgrad_bf16_workspace(C.byref(d))
        if self.mode(d) == 2 and not _stem_x3(self):
            return "of_conv2d_wgrad_x3", lib.of_conv2d_wgrad_x3_workspace(C.byref(d))
        return "of_conv2d_wgrad", lib.of_conv2d_wgrad_workspace(C.byref(d))

    def dgrad_add_entry(self, d):
        """(C entry point, workspace bytes) of the input gradient with an added gradient."""
        lib = _lib.lib()
        if self.bf16(d):
            return "of_conv2d_dgrad_add_bf16", lib.of_conv2d_dgrad_bf16_workspace(C.byref(d))
        if self.mode(d) == 2:
            return "of_conv2d_dgrad_add_x3", lib.of_conv2d_dgrad_x3_workspace(C.byref(d))
        return "of_conv2d_dgrad_add", lib.of_conv2d_dgrad_workspace(C.byref(d))

    def dgrad_entry(self, d):
        lib = _lib.lib()
        if self.bf16(d):
            return "of_conv2d_dgrad_bf16", lib.of_conv2d_dgrad_bf16_workspace(C.byref(d))
        if self.mode(d) == 2:
            return "of_conv2d_dgrad_x3", lib.of_conv2d_dgrad_x3_workspace(C.byref(d))
        return "of_conv2d_dgrad", lib.of_conv2d_dgrad_workspace(C.byref(d))

    def __call__(self, x, residual=None):
        bn = self.bn or (None, None, None, None)
        return _ConvFn.apply(x, self.kernel, self.bias, bn[0], bn[1], residual, self)


class ConvPacker:
    """Packs the GEMM-ready weights of many ConvLayers in ONE kernel launch per optimizer
    step (of_conv_pack_many over a device-resident table built once)."""

    def __init__(self, layers, version_of):
        self.layers = list(layers)
        self.version_of = version_of
        lib = _lib.lib()
        n = len(self.layers)
        descs = (ConvDesc * n)()
        wp, fp, bp = (C.c_void_p * n)(), (C.c_void_p * n)(), (C.c_void_p * n)()
        flags = (C.c_int * n)()
        for i, L in enumerate(self.layers):
            d = L.desc(1, 16, 16)
            descs[i] = d
            L.alloc_packed(d)
            flags[i] = L.mode(d)
            wp[i], fp[i], bp[i] = L.kernel.data_ptr(), L._wf.data_ptr(), L._wd.data_ptr()
        gp, vp = (C.c_void_p * n)(), (C.c_void_p * n)()
        for i, L in enumerate(self.layers):
            if L.bn is not None and not L.bn_train:      # training-mode BN: plain weights
                gp[i], vp[i] = L.bn[0].data_ptr(), L.bn[3].data_ptr()
        nbytes = lib.of_conv_pack_table_bytes(n)
        host = (C.c_char * nbytes)()
        call("of_conv_pack_table_bn", n, descs, wp, fp, bp, flags, gp, vp, BN_EPS, host)
        self.total = C.c_int64.from_buffer(host, 8).value
        self.table = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(
            self.layers[0].kernel.device)
        self._version = None

    def ensure(self):
        v = self.version_of()
        # inside a HIP-graph capture the pack is always recorded: every replay follows an
        # optimizer update that the host-side version counter does not see
        if v == self._version and not torch.cuda.is_current_stream_capturing():
            return
        call("of_conv_pack_many", C.c_void_p(self.table.data_ptr()), self.total, _stream())
        for L in self.layers:
            L._pack_key = (L.kernel.data_ptr(), v)
        self._version = v


class BNZGuard:
    """Keeps z (the pre-BN conv output) for the BN layers whose gamma came near 0.

    The inference-BN backward recovers the normalised value from the layer output,
    zhat = (y - res - beta) / gamma (of_bn_bwd_reduce): exact while |gamma| is not small, but
    its error grows like eps (|beta| + |res|) / |gamma zhat| and it is undefined at gamma = 0,
    where the reference's FusedBatchNormGrad (model.py:14, trained by train.py:55-56) still
    reads the stored z.  This guard watches min |gamma| of every BN layer on the device (one
    launch, of_min_abs_segments, every EVERY optimizer steps, read back through pinned memory
    without a sync) and switches a layer to storing z -- for good -- once it falls below the
    threshold; its backward then reads z (of_bn_act_bwd / of_maxpool_bn_act_bwd).  The
    threshold covers the lag: Keras Adam moves a weight by at most a few lr per step, and a
    check older than LAG_MAX steps is waited for.  Not active inside a HIP-graph capture (the
    mode is the one in force when the graph was captured)."""
    GAMMA_MIN = 1e-2
    EVERY = 4
    LAG_MAX = 8

    def __init__(self, layers):
        self.layers = [L for L in layers if L.bn is not None]
        self.pending = []
        self.steps = 0
        self.flagged = set()     # names of the layers that keep z
        if not self.layers:
            return
        dev = self.layers[0].kernel.device
        self.ptrs = torch.tensor([L.bn[0].data_ptr() for L in self.layers], dtype=torch.int64,
                                 device=dev)
        self.lens = torch.tensor([L.bn[0].numel() for L in self.layers], dtype=torch.int32,
                                 device=dev)
        self.out = torch.empty(len(self.layers), device=dev)
        self.check_now()

    def threshold(self, lr):
        return max(self.GAMMA_MIN, 4.0 * lr * (self.EVERY + self.LAG_MAX))

    def _launch(self):
        call("of_min_abs_segments", _ptr(self.ptrs), _ptr(self.lens), len(self.layers),
             _ptr(self.out), _stream())

    def _apply(self, mins, thr):
        for L, m in zip(self.layers, mins):
            if not m >= thr:            # (a NaN gamma is flagged too)
                L.store_z = True
                self.flagged.add(L.name)

    def mark(self, layers):
        """Apply the flags to other ConvLayer objects over the same weights (by name)."""
        for L in layers:
            if L.bn is not None and L.name in self.flagged:
                L.store_z = True

    def check_now(self, lr=1e-4):
        """Synchronous check (construction, weight loading)."""
        if not self.layers:
            return
        self._launch()
        self._apply(self.out.cpu().tolist(), self.threshold(lr))

    def after_update(self, lr):
        if not self.layers or torch.cuda.is_current_stream_capturing():
            return
        self.steps += 1
        if self.steps % self.EVERY:
            return
        self._launch()
        host = torch.empty(len(self.layers), pin_memory=True)
        host.copy_(self.out, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((self.steps, ev, host, lr))

    def poll(self):
        if torch.cuda.is_current_stream_capturing():
            return
        while self.pending:
            st, ev, host, lr = self.pending[0]
            if not ev.query():
                if self.steps - st < self.LAG_MAX:
                    return
                ev.synchronize()
            self.pending.pop(0)
            self._apply(host.tolist(), self.threshold(lr))

    def stored(self):
        return [L.name for L in self.layers if L.store_z]


def _pad_channels(t: torch.Tensor, cp: int) -> torch.Tensor:
    """Copy an NHWC tensor into a zero-padded one with cp channels (the conv ABI reads
    round_up(C,4) channels)."""
    n, h, w, c = t.shape
    if c == cp and t.is_contiguous():
        return t
    out = torch.empty((n, h, w, cp), device=t.device, dtype=t.dtype)
    if cp != c:
        call("of_fill", _ptr(out), 0.0, out.numel(), _stream())
    t = t.contiguous()
    call("of_copy_strided", _ptr(t), c, _ptr(out), cp, n * h * w, c, _stream())
    return out


def _conv_forward(layer: "ConvLayer", x, residual=None, stream=None):
    """Conv2D + BiasAdd [+ FusedBatchNorm(inference)] [+ AddV2 residual] [+ Relu/LeakyRelu]:
    one fused kernel.  Returns (y, z); z = the pre-BN conv output (BN layers only).
    stream: launch on this stream instead of the current one (the outputs are allocated on
    the current stream, which must wait for ``stream`` before reading them)."""
    _check_dev(x, residual)
    n, h, w, cx = x.shape
    assert cx == layer.cin_p, "conv %s: input has %d channels, expected %d (cin_p)" % (
        layer.name, cx, layer.cin_p)
    d = layer.desc(n, h, w)
    wf, _ = layer.packed(d)
    y = torch.empty((n, d.ho, d.wo, layer.cout), device=x.device)
    bn = layer.bn
    # BN layers: z is not stored, the backward recovers zhat from y (_conv_backward) -- unless
    # a gamma of the layer came near 0 (BNZGuard), where that recovery loses its precision
    z = torch.empty_like(y) if (bn is not None and layer.store_z) else None
    if residual is not None:
        residual = residual.contiguous()
        assert residual.shape == y.shape
    _tag(layer, 0)
    entry, wsz = layer.fwd_entry(d)
    wsk, wsp, wsb = _workspace(wsz, x.device)
    st = _stream()
    if stream is not None:
        for t in (x, y, z, wsk, residual):
            if t is not None:
                t.record_stream(stream)
        st = C.c_void_p(stream.cuda_stream)
    call(entry, C.byref(d), _ptr(x), cx, _ptr(wf), _ptr(layer.bias),
         _ptr(bn[0]) if bn else None, _ptr(bn[1]) if bn else None,
         _ptr(bn[2]) if bn else None, _ptr(bn[3]) if bn else None, BN_EPS,
         _ptr(residual), layer.cout, layer.act, layer.alpha,
         _ptr(z), layer.cout, _ptr(y), layer.cout, wsp, wsb, st)
    return y, z


# The encoder's 1x1 stride-2 projections (res3_0 / res4_0 proj, model.py:20,22) read the same
# block input as conv_a and are independent of it until conv_b adds them: their forward runs on
# a stream of its own beside conv_a (a 0.8-GFLOP conv is launch/latency-bound on its own).
# OFLOW_PROJ_SIDE=0 keeps them on the current stream.
PROJ_SIDE = os.environ.get("OFLOW_PROJ_SIDE", "1") == "1"
_FWD_SIDE = {}


def _fwd_side_stream():
    """The forward's side stream of the current device, ordered after the current stream's
    work so far (no end-of-backward join: the caller waits for it, stream_wait)."""
    cur = torch.cuda.current_stream()
    s = _FWD_SIDE.get(cur.device)
    if s is None:
        s = _FWD_SIDE[cur.device] = torch.cuda.Stream(cur.device)
    stream_wait(s, cur)
    return s


def _block_forward(a, b, p, x):
    """One residual block's forward: (ya, za, y, zb, yp, zp)."""
    yp = zp = None
    side = None
    if p is not None and PROJ_SIDE and x.is_cuda:
        # any weight packing the projection still needs is enqueued on the current stream
        # BEFORE the side stream forks from it, so the side-stream conv reads packed weights
        p.packed(p.desc(*x.shape[:3]))
        side = _fwd_side_stream()
        yp, zp = _conv_forward(p, x, stream=side)
    ya, za = _conv_forward(a, x)
    if p is not None and side is None:
        yp, zp = _conv_forward(p, x)
    if side is not None:
        stream_wait(torch.cuda.current_stream(), side)
    y, zb = _conv_forward(b, ya, residual=yp if p is not None else x)
    return ya, za, y, zb, yp, zp


def _conv_backward(layer: "ConvLayer", x, y, z, dy, has_res, needs, add=None, dx_out=None,
                   dz_given=None, t_given=False, res_src=None, in_act=None, bnp_out=None):
    """Backward of _conv_forward: BN/activation backward (with the residual gradient), weight
    and bias gradients, input gradient.  needs = (x, kernel, bias, gamma, beta, residual).
    add: a gradient summed into dx by the input-gradient kernel's epilogue (dx_out may be
    that same buffer).  dz_given: the pre-activation gradient already computed, with the BN
    and bias gradients, by a fused kernel (the stem, of_maxpool_bn_relu_bwd).

    BN layers (FusedBatchNormGrad, inference mode, P5) never form dz: with t = dy * act'(y)
    the BN scale s = gamma / sqrt(var + eps) is folded into the packed input-gradient weights
    (ConvLayer.packed, ConvPacker) and the weight-gradient reduction (of_conv2d_wgrad_bn), and
    one reduction pass (of_bn_bwd_reduce) gives dgamma, dbeta and the bias gradient, reading t
    and y (z is recovered from y; res_src = the residual added before the activation).
    t_given: dy already is t (the producing input-gradient kernel applied act' in its
    epilogue).  in_act = (act_src, act): multiply this layer's input gradient by the
    derivative of the activation that produced x (after the add, if any), so the layer before
    receives its t.  bnp_out = (L, res): L is the BN layer whose output is act_src (res its
    residual before the activation, or None): with BN_FUSE the input-gradient epilogue also
    forms L's BN partial sums (of_conv2d_dgrad_add_act_bnp) and tags dx with them
    (dx._oflow_bnp), and L's backward then runs only the final pass (of_bn_bwd_final).

    Returns (dx, d_kernel, d_bias, d_gamma, d_beta, d_residual) with None for gradients
    written straight into the gradient arena."""
    n, h, w, cx = x.shape
    d = layer.desc(n, h, w)
    _, wd = layer.packed(d)
    dy = dy.contiguous() if dy is not None else None
    s = _stream()
    need_x, need_k, need_b, need_g, need_be, need_res = needs
    ret_k = ret_b = ret_g = ret_be = dres = dx = None
    npix = n * d.ho * d.wo
    bn_fold = False
    # ---- pre-activation gradient dz -----------------------------------------------------
    if dz_given is not None:
        dz = dz_given
        bias_done = True
    elif layer.bn is not None:
        gamma, beta, mean, var = layer.bn
        tg = grad_target(gamma) if need_g else (None, 0, None)
        tb = grad_target(beta) if need_be else (None, 0, None)
        tbias = grad_target(layer.bias) if need_b else (None, 0, None)
        ret_g, ret_be, ret_b = tg[2], tb[2], tbias[2]
        acc = tg[1] if need_g else (tb[1] if need_be else tbias[1])
        # per-target accumulate flags must agree (all arena or all fresh)
        assert all(t[0] is None or t[1] == acc for t in (tg, tb, tbias))
        ws = torch.empty(_lib.lib().of_bn_act_bwd_workspace(npix, layer.cout) // 4 + 1,
                         device=dy.device)
        if t_given or layer.act == ACT_NONE:
            dz = dy                     # already t
            # only parameter gradients come out: off the critical path (BN_REDUCE_SIDE)
            side = BN_REDUCE_SIDE and SIDE_STREAM_WGRAD and acc == 1
            fused = getattr(dy, "_oflow_bnp", None)
            if fused is not None and (fused[2] is not layer or z is not None):
                fused = None
            with torch.cuda.stream(side_stream(dz, y, res_src, ws, z,
                                               fused[0] if fused else None)) if side else \
                    contextlib.nullcontext():
                if fused is not None:   # the partial sums came with t (input-grad epilogue)
                    call("of_bn_bwd_final", _ptr(fused[0]), fused[1], layer.cout, _ptr(gamma),
                         _ptr(var), BN_EPS, _ptr(tg[0]), _ptr(tb[0]), _ptr(tbias[0]), acc,
                         _stream())
                elif z is not None:     # zhat from the stored z (BNZGuard)
                    call("of_bn_act_bwd", npix, layer.cout, ACT_NONE, _ptr(dz), _ptr(y), _ptr(z),
                         _ptr(gamma), _ptr(mean), _ptr(var), BN_EPS, None, None, _ptr(tg[0]),
                         _ptr(tb[0]), _ptr(tbias[0]), acc, _ptr(ws), _stream())
                else:
                    call("of_bn_bwd_reduce", npix, layer.cout, ACT_NONE, _ptr(dz), _ptr(y),
                         _ptr(res_src), _ptr(gamma), _ptr(beta), _ptr(var), BN_EPS, None,
                         _ptr(tg[0]), _ptr(tb[0]), _ptr(tbias[0]), acc, _ptr(ws), _stream())
        else:
            dz = torch.empty_like(dy)    # t = dy * act'(y)
            if z is not None:
                call("of_bn_act_bwd", npix, layer.cout, layer.act, _ptr(dy), _ptr(y), _ptr(z),
                     _ptr(gamma), _ptr(mean), _ptr(var), BN_EPS, None, _ptr(dz), _ptr(tg[0]),
                     _ptr(tb[0]), _ptr(tbias[0]), acc, _ptr(ws), s)
            else:
                call("of_bn_bwd_reduce", npix, layer.cout, layer.act, _ptr(dy), _ptr(y),
                     _ptr(res_src), _ptr(gamma), _ptr(beta), _ptr(var), BN_EPS, _ptr(dz),
                     _ptr(tg[0]), _ptr(tb[0]), _ptr(tbias[0]), acc, _ptr(ws), s)
        if has_res and need_res:
            dres = dz                   # the residual branch's gradient is t itself
        bias_done = True
        bn_fold = True
    else:
        if layer.act != ACT_NONE:
            dz = torch.empty_like(dy)
            call("of_act_bwd", _ptr(dy), _ptr(y), layer.act, layer.alpha, _ptr(dz),
                 dy.numel(), s)
        else:
            dz = dy
        if has_res and need_res:
            dres = dz
        bias_done = False
    dzp = _pad_channels(dz, _c4(layer.cout))
    res = {"dx": None, "k": None, "b": None}

    def input_grad():
        # ---- input gradient -------------------------------------------------------------
        if need_x and S2_JOIN and SIDE_STREAM_WGRAD and _gemm_layer(layer) and \
                dz.device in _SIDE and not SINGLE_STREAM:
            stream_wait(torch.cuda.current_stream(), _SIDE[dz.device])
        if need_x:
            dx = dx_out if dx_out is not None else torch.empty((n, h, w, cx), device=dz.device)
            res["dx"] = dx
            _tag(layer, 1)
            if in_act is not None:
                src, iact = in_act
                src = src.contiguous()
                addc = add.contiguous() if add is not None else None
                if addc is not None:
                    assert addc.shape == dx.shape
                _, wsz = layer.dgrad_add_entry(d)
                wsk, wsp, wsb = _workspace(wsz, dy.device if dy is not None else dz.device)
                if not (bnp_out is not None and _dgrad_bnp(layer, d, dzp, wd, addc, src, iact,
                                                           dx, cx, bnp_out, wsp, wsb, s)):
                    call("of_conv2d_dgrad_add_act", C.byref(d), layer.mode(d), _ptr(dzp),
                         dzp.shape[-1], _ptr(wd), _ptr(addc), cx, _ptr(src), cx, iact,
                         LEAKY_ALPHA, _ptr(dx), cx, wsp, wsb, s)
            elif add is not None:
                addc = add.contiguous()
                assert addc.shape == dx.shape
                entry, wsz = layer.dgrad_add_entry(d)
                wsk, wsp, wsb = _workspace(wsz, dy.device)
                call(entry, C.byref(d), _ptr(dzp), dzp.shape[-1], _ptr(wd), _ptr(addc), cx,
                     _ptr(dx), cx, wsp, wsb, s)
            else:
                entry, wsz = layer.dgrad_entry(d)
                wsk, wsp, wsb = _workspace(wsz, dy.device)
                call(entry, C.byref(d), _ptr(dzp), dzp.shape[-1], _ptr(wd), None, 0,
                     ACT_NONE, 0.0, _ptr(dx), cx, wsp, wsb, s)

    def weight_grad():
        # ---- weight (+bias) gradient ----------------------------------------------------
        if need_k or (need_b and not bias_done):
            tk = grad_target(layer.kernel)
            tbias = grad_target(layer.bias) if (need_b and not bias_done) else (None, 0, None)
            went, wsb = layer.wgrad_entry(d)
            side = (SIDE_STREAM_WGRAD and tk[1] == 1 and (tbias[0] is None or tbias[1] == 1) and
                    d.n * d.ho * d.wo <= _side_max_pix(layer) and
                    not (S2_WGRAD_MAIN and _gemm_layer(layer)))
            with torch.cuda.stream(side_stream(x, dzp)) if side else contextlib.nullcontext():
                ss = _stream()
                if bn_fold:                 # dw = s * (x^T t): the BN scale in the reduction
                    wsb = _lib.lib().of_conv2d_wgrad_bn_workspace(C.byref(d), layer.mode(d))
                    ws = torch.empty(wsb // 4 + 1, device=dz.device)
                    gamma, _, _, var = layer.bn
                    _tag(layer, 2)
                    call("of_conv2d_wgrad_bn", C.byref(d), layer.mode(d), _ptr(x), cx, _ptr(dzp),
                         dzp.shape[-1], _ptr(tk[0]), tk[1], _ptr(gamma), _ptr(var), BN_EPS,
                         _ptr(ws), wsb, ss)
                    res["k"] = tk[2] if need_k else None
                    return
                ws = torch.empty(wsb // 4 + 1, device=dz.device)
                if tbias[0] is not None and tbias[1] != tk[1]:
                    # mixed arena / fresh targets: compute the bias into a temp, then place it
                    tmpb = torch.empty_like(layer.bias)
                    _tag(layer, 2)
                    call(went, C.byref(d), _ptr(x), cx, _ptr(dzp), dzp.shape[-1],
                         _ptr(tk[0]), _ptr(tmpb), tk[1], _ptr(ws), wsb, ss)
                    if tbias[1]:
                        call("of_add_inplace", _ptr(tbias[0]), _ptr(tmpb), tmpb.numel(), ss)
                    else:
                        tbias = (tmpb, 0, tmpb)
                else:
                    _tag(layer, 2)
                    call(went, C.byref(d), _ptr(x), cx, _ptr(dzp), dzp.shape[-1],
                         _ptr(tk[0]), _ptr(tbias[0]), tk[1], _ptr(ws), wsb, ss)
            res["k"] = tk[2] if need_k else None
            if need_b and not bias_done:
                res["b"] = tbias[2]

    def ready():
        # every gradient of this layer's parameters is enqueued: a bucket all-reduce that
        # this completes forks here, before the input gradient, so it overlaps that kernel
        _grad_ready(layer.kernel if need_k else None, layer.bias if need_b else None,
                    *(layer.bn[:2] if layer.bn is not None else ()))

    # launch order: see DGRAD_FIRST
    for f in ((input_grad, weight_grad, ready) if DGRAD_FIRST else
              (weight_grad, ready, input_grad)):
        f()
    dx, ret_k = res["dx"], res["k"]
    if res["b"] is not None or not bias_done:
        ret_b = res["b"]
    return dx, ret_k, ret_b, ret_g, ret_be, dres


# The BN backward partial sums of the layer whose output a block's input gradient carries,
# formed by that input gradient's epilogue (conv_tile_x3, one K slice: of_conv2d_dgrad_add_act_bnp)
# instead of a separate pass reading t, y and the residual again (OFLOW_BN_FUSE=0: the
# separate pass everywhere).
BN_FUSE = os.environ.get("OFLOW_BN_FUSE", "1") == "1"


def _dgrad_bnp(layer, d, dzp, wd, addc, src, iact, dx, cx, bnp_out, wsp, wsb, s):
    """of_conv2d_dgrad_add_act with bnp_out's BN partial sums; False (nothing launched) when
    the kernel form cannot carry them."""
    L, rres = bnp_out
    if not BN_FUSE or L.bn is None or L.store_z or L.cout != cx:
        return False
    lib = _lib.lib()
    pb = lib.of_conv2d_dgrad_bnp_bytes(C.byref(d))
    if pb <= 0:
        return False
    part = torch.empty(pb // 4 + 4, device=dx.device)
    nblk = C.c_int(0)
    gamma, beta = L.bn[0], L.bn[1]
    rres = rres.contiguous() if rres is not None else None
    st = lib.of_conv2d_dgrad_add_act_bnp(
        C.byref(d), layer.mode(d), _ptr(dzp), dzp.shape[-1], _ptr(wd), _ptr(addc), cx, _ptr(src),
        cx, iact, C.c_float(LEAKY_ALPHA), _ptr(dx), cx, _ptr(gamma), _ptr(beta), _ptr(rres),
        rres.shape[-1] if rres is not None else 0, _ptr(part), pb, C.byref(nblk), wsp, wsb, s)
    if st == _lib.OF_EUNSUPPORTED:
        return False
    _lib.check(st, "of_conv2d_dgrad_add_act_bnp")
    dx._oflow_bnp = (part, nblk.value, L)
    return True


class _ConvFn(torch.autograd.Function):
    """Conv2D + BiasAdd [+ FusedBatchNorm(inference)] [+ AddV2 residual] [+ Relu/LeakyRelu]
    forward; Conv2DBackpropInput / Conv2DBackpropFilter / BiasAddGrad / BN grads backward."""

    @staticmethod
    def forward(ctx, x, kernel, bias, gamma, beta, residual, layer: ConvLayer):
        _check_dev(kernel, bias)
        y, z = _conv_forward(layer, x.contiguous(), residual)
        ctx.layer = layer
        ctx.has_res = residual is not None
        ctx.save_for_backward(x.contiguous(), y, z,
                              residual.contiguous() if residual is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, z, r = ctx.saved_tensors
        out = _conv_backward(ctx.layer, x, y, z, dy, ctx.has_res, ctx.needs_input_grad[:6],
                             res_src=r)
        return (*out, None)


class _ResBlockFn(torch.autograd.Function):
    """One residual block of the encoder (resnet_layer_simple, model.py:18,20,22; assumed
    basic block): y = ReLU(BN_b(conv_b(ReLU(BN_a(conv_a(x))))) + shortcut),
    shortcut = x or BN_p(proj(x)).  One autograd node so that the input gradient's two
    branches are summed by the conv_a input-gradient epilogue (of_conv2d_dgrad_add) rather
    than by an extra elementwise pass."""

    @staticmethod
    def forward(ctx, x, *args):
        a, b, p = args[-1]
        x = x.contiguous()
        ya, za, y, zb, yp, zp = _block_forward(a, b, p, x)
        ctx.block = (a, b, p)
        ctx.save_for_backward(x, ya, za, y, zb, yp, zp)
        return y

    @staticmethod
    def backward(ctx, dy):
        dx, grads = _res_block_backward(ctx.block, ctx.saved_tensors, dy, ctx.needs_input_grad)
        return (dx, *grads, None)


def _res_block_backward(block, saved, dy, need, extra=None, t_given=False, in_act=None,
                        in_bnp=None):
    """Backward of one residual block.  need: needs_input_grad of (x, then kernel, bias,
    gamma, beta per layer a, b, p).  extra: a further gradient of the block input x (its
    other consumer) summed by the shortcut's input-gradient epilogue -- no separate add.
    t_given: dy already carries the block's output ReLU derivative (the next block's
    input-gradient epilogue applied it).  in_act = (x, ACT_RELU) when x is a ReLU output: the
    returned dx is then the previous block's t.  conv_b's input gradient always carries
    conv_a's ReLU derivative (t of conv_a).  in_bnp = (the previous block's conv_b, its
    residual): the layer whose BN partial sums conv_a's input-gradient epilogue forms
    (BN_FUSE).  Returns (dx, [param grads of a, b, p])."""
    x, ya, za, y, zb, yp, zp = saved
    a, b, p = block
    need_x = need[0]
    nb = lambda k: tuple(need[1 + 4 * k:5 + 4 * k])     # kernel, bias, gamma, beta of layer k
    sc = yp if p is not None else x                      # residual added before b's ReLU
    dya, *gb = _conv_backward(b, ya, y, zb, dy, True, (True, *nb(1), True), t_given=t_given,
                              res_src=sc, in_act=(ya, ACT_RELU), bnp_out=(a, None))
    dres = gb[-1]                                        # = t of conv_b
    gb = gb[:-1]
    if p is not None:
        dxp, *gp = _conv_backward(p, x, yp, zp, dres, False, (need_x, *nb(2), False),
                                  add=extra if need_x else None,
                                  dx_out=extra if need_x else None,   # in place: see below
                                  t_given=True)
        gp = gp[:-1]
        add, dx_out = dxp, dxp
    else:
        gp = []
        add, dx_out = dres, None
        if extra is not None and need_x:
            # (dres is also conv_b's weight-gradient input, possibly still being read on the
            # side stream: sum into a copy)
            add = dres.clone()
            call("of_add_inplace", _ptr(add), _ptr(extra.contiguous()), add.numel(), _stream())
    dx, *ga = _conv_backward(a, x, ya, za, dya, False, (need_x, *nb(0), False),
                             add=add if need_x else None, dx_out=dx_out, t_given=True,
                             in_act=in_act if need_x else None,
                             bnp_out=in_bnp if (need_x and in_act is not None) else None)
    ga = ga[:-1]
    return dx, list(ga) + list(gb) + list(gp)


class _EncoderFn(torch.autograd.Function):
    """reset18_encoder (model.py:10-26) forward and backward as ONE autograd node: conv1 +
    BN + ReLU -> out0 -> max-pool -> residual blocks -> out1..out3 (out4 with levels=5).
    Each encoder output feeds the decoder and (out0..out2) the next stage, so under plain
    autograd every such junction costs a full-size add of the two gradients; here the
    decoder's gradient of out_k is summed by the next stage's shortcut input-gradient
    epilogue (_res_block_backward extra=), and out0's by the fused stem kernel
    (of_maxpool_bn_act_bwd: max-pool backward + add + BN/ReLU backward in one pass)."""

    @staticmethod
    def forward(ctx, x4, *args):
        conv1, blocks = args[-1]
        x4 = x4.contiguous()
        y0, z0, xp = _stem_forward_pool(conv1, x4)
        x = xp
        saved = [x4, y0, z0]
        outs = [y0]
        for i, (a, b, p) in enumerate(blocks):
            ya, za, y, zb, yp, zp = _block_forward(a, b, p, x)
            saved += [x, ya, za, y, zb, yp, zp]
            x = y
            if i % 2 == 1:
                outs.append(y)
        ctx.conv1, ctx.blocks = conv1, blocks
        ctx.save_for_backward(*saved)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        corr_side_wait(gouts[0].device if gouts[0] is not None else ctx.saved_tensors[0].device)
        saved = ctx.saved_tensors
        x4, y0, z0 = saved[:3]
        conv1, blocks = ctx.conv1, ctx.blocks
        need = ctx.needs_input_grad          # x4, then per layer kernel/bias/gamma/beta
        nbk = len(blocks)
        gouts = [g.contiguous() if g is not None else None for g in gouts]
        dy = gouts[-1] if gouts[-1] is not None else torch.zeros_like(saved[3 + 7 * (nbk - 1) + 3])
        grads = []
        off = 1 + 4                          # after x4 and conv1's 4 parameters
        pos = []
        for a, b, p in blocks:
            pos.append(off)
            off += 4 * (3 if p is not None else 2)
        for i in range(nbk - 1, -1, -1):
            blk = saved[3 + 7 * i:3 + 7 * (i + 1)]
            extra = gouts[i // 2] if (i % 2 == 0 and i > 0) else None
            nd = (True,) + tuple(need[pos[i]:pos[i] + 4 * (3 if blocks[i][2] is not None else 2)])
            # block i > 0 takes a ReLU output (block i - 1's) as input: its input gradient
            # is returned as that block's t; block 0's input is the max-pooled stem output
            in_bnp = None
            if i > 0:                           # block i - 1's conv_b BN: y = blk[0]
                pa, pb_, pp = blocks[i - 1]
                pblk = saved[3 + 7 * (i - 1):3 + 7 * i]
                in_bnp = (pb_, pblk[5] if pp is not None else pblk[0])
            dy, g = _res_block_backward(blocks[i], blk, dy, nd, extra=extra,
                                        t_given=i < nbk - 1,
                                        in_act=(blk[0], ACT_RELU) if i > 0 else None,
                                        in_bnp=in_bnp)
            grads = list(g) + grads
        # stem: max-pool backward + out0's decoder gradient + BN/ReLU backward, one pass
        n, h, w, c = y0.shape
        gamma, beta, mean, var = conv1.bn
        nk, nbias, ng, nbe = need[1:5]
        tg = grad_target(gamma) if ng else (None, 0, None)
        tb = grad_target(beta) if nbe else (None, 0, None)
        tbias = grad_target(conv1.bias) if nbias else (None, 0, None)
        acc = tg[1] if ng else (tb[1] if nbe else tbias[1])
        assert all(t[0] is None or t[1] == acc for t in (tg, tb, tbias))
        d1 = conv1.desc(*x4.shape[:3])
        m1 = conv1.mode(d1)
        tk = grad_target(conv1.kernel) if nk else (None, 0, None)
        if (STEM_FUSED and z0 is None and m1 in (1, 2) and nk and nbias and ng and nbe and
                tk[1] == acc):
            fws = _lib.lib().of_stem_bwd_fused_workspace(C.byref(d1), m1)
            if fws > 0:
                # the whole stem backward in the weight-gradient kernel: dz never stored
                wsf = torch.empty(fws // 4 + 1, device=y0.device)
                _tag(conv1, 2)
                call("of_stem_bwd_fused", C.byref(d1), m1, _ptr(x4), x4.shape[-1],
                     _ptr(dy.contiguous()), _ptr(gouts[0]), _ptr(y0), _ptr(gamma), _ptr(beta),
                     _ptr(var), BN_EPS, _ptr(tk[0]), _ptr(tbias[0]), _ptr(tg[0]), _ptr(tb[0]),
                     acc, _ptr(wsf), fws, _stream())
                _grad_ready(conv1.kernel, conv1.bias, gamma, beta)
                stem = [tk[2], tbias[2], tg[2], tb[2]]
                return (None, *stem, *grads, None)
        dz0 = torch.empty_like(y0)
        ws = torch.empty(_lib.lib().of_maxpool_bn_act_bwd_workspace(n, h, w, c) // 4 + 1,
                         device=y0.device)
        if z0 is not None:              # zhat from the stored z (BNZGuard)
            call("of_maxpool_bn_act_bwd", n, h, w, c, _ptr(dy.contiguous()), _ptr(gouts[0]),
                 _ptr(y0), _ptr(z0), _ptr(gamma), _ptr(mean), _ptr(var), BN_EPS, _ptr(dz0),
                 _ptr(tg[0]), _ptr(tb[0]), _ptr(tbias[0]), acc, _ptr(ws), _stream())
        else:
            call("of_maxpool_bn_relu_bwd", n, h, w, c, _ptr(dy.contiguous()), _ptr(gouts[0]),
                 _ptr(y0), _ptr(gamma), _ptr(beta), _ptr(var), BN_EPS, _ptr(dz0), _ptr(tg[0]),
                 _ptr(tb[0]), _ptr(tbias[0]), acc, _ptr(ws), _stream())
        _, gk, _, _, _, _ = _conv_backward(conv1, x4, y0, z0, None, False,
                                           (False, nk, nbias, ng, nbe, False), dz_given=dz0)
        stem = [gk, tbias[2], tg[2], tb[2]]
        return (None, *stem, *grads, None)


# ------------------------------------------------- BatchNormalization, training mode ----
# bn_mode="training" (SURVEY.md §8 P5): keras BatchNormalization(training=True) as the legacy
# loop calls it (old/train.py:59); the reference's own train.py:51 runs inference mode, the
# default above.  Each BN layer normalises with the statistics of the batch it is called on --
# per Siamese half (``groups`` = 2 on the (2B) encoder batch: model.py:131-132 calls the
# encoder once per image) -- and updates its moving statistics in place (momentum 0.99, Keras'
# default).  The conv writes z (bias included, no BN epilogue), of_bn_train_stats /
# of_bn_train_apply normalise, and the backward is FusedBatchNormGradV3's (of_bn_train_bwd)
# followed by the plain conv gradients of dz: nothing of the inference path's BN fold applies.
# Not the benchmarked configuration: one autograd node per conv, gradients summed by autograd.
BN_MOMENTUM = 0.99


class _ConvBNTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, bias, gamma, beta, residual, layer: ConvLayer, groups: int):
        _check_dev(x, kernel, bias, residual)
        x = x.contiguous()
        n, h, w, cx = x.shape
        assert cx == layer.cin_p and layer.bn is not None and layer.bn_train
        d = layer.desc(n, h, w)
        wf, _ = layer.packed(d)
        z = torch.empty((n, d.ho, d.wo, layer.cout), device=x.device)
        entry, wsz = layer.fwd_entry(d)
        wsk, wsp, wsb = _workspace(wsz, x.device)
        s = _stream()
        _tag(layer, 0)
        call(entry, C.byref(d), _ptr(x), cx, _ptr(wf), _ptr(layer.bias), None, None, None, None,
             BN_EPS, None, layer.cout, ACT_NONE, 0.0, None, layer.cout, _ptr(z), layer.cout, wsp,
             wsb, s)
        npix, c = n * d.ho * d.wo, layer.cout
        assert n % groups == 0
        g_, be, mm, mv = layer.bn
        mean = torch.empty((groups, c), device=x.device)
        invstd = torch.empty((groups, c), device=x.device)
        ws = torch.empty(_lib.lib().of_bn_train_workspace(npix, c, groups) // 4 + 1,
                         device=x.device)
        call("of_bn_train_stats", npix, c, groups, _ptr(z), BN_EPS, BN_MOMENTUM, _ptr(mean),
             _ptr(invstd), _ptr(mm), _ptr(mv), _ptr(ws), s)
        if residual is not None:
            residual = residual.contiguous()
            assert residual.shape == z.shape
        y = torch.empty_like(z)
        call("of_bn_train_apply", npix, c, groups, _ptr(z), _ptr(mean), _ptr(invstd), _ptr(g_),
             _ptr(be), _ptr(residual), layer.act, _ptr(y), s)
        ctx.layer, ctx.groups = layer, groups
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, z, y, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, z, y, mean, invstd = ctx.saved_tensors
        layer, groups = ctx.layer, ctx.groups
        need_x, need_k, need_b, need_g, need_be, need_res = ctx.needs_input_grad[:6]
        dy = dy.contiguous()
        n, h, w, cx = x.shape
        d = layer.desc(n, h, w)
        _, wd = layer.packed(d)
        npix, c = n * d.ho * d.wo, layer.cout
        s = _stream()
        g_ = layer.bn[0]
        tg = grad_target(g_) if need_g else (None, 0, None)
        tb = grad_target(layer.bn[1]) if need_be else (None, 0, None)
        acc = tg[1] if need_g else tb[1]
        assert tb[0] is None or tb[1] == acc
        dz = torch.empty_like(z)
        t = torch.empty_like(z) if (ctx.has_res and need_res) else None
        ws = torch.empty(_lib.lib().of_bn_train_workspace(npix, c, groups) // 4 + 1,
                         device=z.device)
        call("of_bn_train_bwd", npix, c, groups, layer.act, _ptr(dy), _ptr(y), _ptr(z),
             _ptr(mean), _ptr(invstd), _ptr(g_), _ptr(dz), _ptr(t), _ptr(tg[0]), _ptr(tb[0]),
             acc, _ptr(ws), s)
        ret_k = ret_b = dx = None
        if need_k or need_b:
            tk = grad_target(layer.kernel)
            tbias = grad_target(layer.bias)
            assert tk[1] == tbias[1]
            went, wsb = layer.wgrad_entry(d)
            wsw = torch.empty(wsb // 4 + 1, device=z.device)
            _tag(layer, 2)
            call(went, C.byref(d), _ptr(x), cx, _ptr(dz), c, _ptr(tk[0]), _ptr(tbias[0]), tk[1],
                 _ptr(wsw), wsb, s)
            ret_k, ret_b = tk[2], tbias[2]
            _grad_ready(layer.kernel, layer.bias, g_, layer.bn[1])
        if need_x:
            dx = torch.empty_like(x)
            entry, wsz = layer.dgrad_entry(d)
            wsk, wsp, wsb = _workspace(wsz, z.device)
            _tag(layer, 1)
            call(entry, C.byref(d), _ptr(dz), c, _ptr(wd), None, 0, ACT_NONE, 0.0, _ptr(dx), cx,
                 wsp, wsb, s)
        return dx, ret_k, ret_b, tg[2], tb[2], t, None, None


def conv_bn_train(layer: ConvLayer, x, residual=None, groups: int = 1):
    """Conv2D + BiasAdd + BatchNormalization(training=True) [+ residual] [+ activation]."""
    g_, be = layer.bn[0], layer.bn[1]
    return _ConvBNTrainFn.apply(x, layer.kernel, layer.bias, g_, be, residual, layer, groups)


def encoder_forward_train(x4, conv1: ConvLayer, blocks, groups: int = 2):
    """reset18_encoder (model.py:10-26) with BN in training mode: [out0, out1, ...]."""
    y = conv_bn_train(conv1, x4, groups=groups)
    outs = [y]
    x = maxpool2(y)
    for i, (a, b, p) in enumerate(blocks):
        ya = conv_bn_train(a, x, groups=groups)
        sc = conv_bn_train(p, x, groups=groups) if p is not None else x
        x = conv_bn_train(b, ya, residual=sc, groups=groups)
        if i % 2 == 1:
            outs.append(x)
    return outs


# The stem's backward (max-pool + out0 gradient + BN + ReLU, then the 7x7 weight gradient) in
# the weight-gradient kernel itself (of_stem_bwd_fused): dz0, the encoder's largest tensor, is
# never written and read back.  Off by default: measured on the bench step (profiles/r5_*) the
# fused weight gradient took 340 us + 65 us of stem_bn_final against 150 + 132 us for
# of_maxpool_bn_relu_bwd + the plain wgrad (it re-forms dz per K slice).  OFLOW_STEM_FUSED=1.
STEM_FUSED = os.environ.get("OFLOW_STEM_FUSED", "0") == "1"


# The stem forward writes the max-pooled tensor too (of_conv2d_fwd_pool: MaxPool2D,
# model.py:17, in the stem kernel's epilogue), so the pool does not re-read the encoder's
# largest activation.  OFLOW_STEM_POOL=0 keeps the separate of_maxpool2_fwd pass.
STEM_POOL = os.environ.get("OFLOW_STEM_POOL", "1") == "1"


def _stem_forward_pool(conv1: ConvLayer, x4):
    """conv1 + BN + ReLU -> (y0, z0, max-pool of y0)."""
    n, h, w, cx = x4.shape
    d = conv1.desc(n, h, w)
    m = conv1.mode(d)
    if STEM_POOL and m in (1, 2) and not conv1.store_z and d.ho % 2 == 0 and d.wo % 2 == 0:
        wf, _ = conv1.packed(d)
        y0 = torch.empty((n, d.ho, d.wo, conv1.cout), device=x4.device)
        xp = torch.empty((n, d.ho // 2, d.wo // 2, conv1.cout), device=x4.device)
        entry, wsz = conv1.fwd_entry(d)
        wsk, wsp, wsb = _workspace(wsz, x4.device)
        bn = conv1.bn
        _tag(conv1, 0)
        st = _lib.lib().of_conv2d_fwd_pool(
            C.byref(d), m, _ptr(x4), cx, _ptr(wf), _ptr(conv1.bias), _ptr(bn[0]), _ptr(bn[1]),
            _ptr(bn[2]), _ptr(bn[3]), BN_EPS, conv1.act, conv1.alpha, None, conv1.cout, _ptr(y0),
            conv1.cout, _ptr(xp), wsp, wsb, _stream())
        if st == _lib.OF_OK:
            return y0, None, xp
        if st != _lib.OF_EUNSUPPORTED:
            _lib.check(st, "of_conv2d_fwd_pool")
        if TIMING_TAGS and TIMING_TAGS[-1] == (conv1.name, 0):
            TIMING_TAGS.pop()                # nothing was launched: the tag is re-added below
    y0, z0 = _conv_forward(conv1, x4)
    n, h, w, c = y0.shape
    xp = torch.empty((n, h // 2, w // 2, c), device=y0.device)
    call("of_maxpool2_fwd", _ptr(y0), n, h, w, c, _ptr(xp), _stream())
    return y0, z0, xp


def encoder_forward(x4, conv1: ConvLayer, blocks):
    """All encoder outputs [out0, out1, ...] of x4 (N, H, W, 4) through _EncoderFn."""
    params = [conv1.kernel, conv1.bias, conv1.bn[0], conv1.bn[1]]
    for a, b, p in blocks:
        for L in (a, b) + ((p,) if p is not None else ()):
            params += [L.kernel, L.bias, L.bn[0], L.bn[1]]
    return list(_EncoderFn.apply(x4, *params, (conv1, blocks)))


def res_block(x, a: ConvLayer, b: ConvLayer, p: Optional[ConvLayer] = None):
    params = []
    for L in (a, b) + ((p,) if p is not None else ()):
        params += [L.kernel, L.bias, L.bn[0], L.bn[1]]
    return _ResBlockFn.apply(x, *params, (a, b, p))


# bf16 activation images for the bf16 flow heads (configs 3-5; conv_b16i.hip).  In bf16 mode
# every consumer of a head conv's output rounds it to bf16 anyway (the next conv's forward and
# weight gradient) or needs only its sign (the LeakyReLU derivative), so the outputs of c0..c3
# are stored as bf16 NHWC images only, the input gradients between them likewise, and the
# convs run on the DMA-fed large-tile kernels (of_conv2d_b16i, of_conv2d_wgrad_b16i); the bias
# gradients come from the input-gradient kernels' column sums of the fp32 values (exact sums,
# as the oracle's).  The rounding points are those of the fp32-image path, so the results
# agree with it up to fp32 summation order.  Used for levels whose forward grid has at least
# B16I_MIN_TILES 16 x 32 tiles (the kernels take one K slice: smaller grids keep the halo
# kernels with K splits); OFLOW_B16I=0 turns it off, OFLOW_B16I_MIN_TILES overrides the size.
# 128 (round 4, with the fused cost-volume backward): the H/8 head at B = 32 (192 tiles) too,
# bf16 B=32 1703.9 (256) -> 1716.4 (128) / 1712.0 (64) pairs/s, profiles/r4_late/step_ab.txt.
B16I = os.environ.get("OFLOW_B16I", "1") == "1"
B16I_MIN_TILES = int(os.environ.get("OFLOW_B16I_MIN_TILES", "128"))
# The forwards of the bf16-image heads write their outputs' act' signs (of_b16i_io mask_out)
# and the input gradients read those (mask_in) on conv_halo_b16's direct epilogue;
# OFLOW_B16I_MASK=0 keeps the act16 form (the general epilogue).
B16I_MASK = os.environ.get("OFLOW_B16I_MASK", "1") == "1"
# The bf16-image heads' input, concat([f1, cost volume, flow]), written as its bf16 image by the
# cost-volume kernel (of_corr_concat_fwd16) instead of an fp32 row plus a conversion pass;
# OFLOW_CONCAT_IMG16=0 keeps the fp32 row.
CONCAT_IMG16 = os.environ.get("OFLOW_CONCAT_IMG16", "1") == "1"


def _img16_ok(layers, x) -> bool:
    if not B16I or len(layers) < 3:
        return False
    n, h, w, _ = x.shape
    if (n * ((h + 15) // 16) * ((w + 31) // 32)) < B16I_MIN_TILES:
        return False
    for L in layers[:-1]:
        if not (L.precision == "bf16" and L.kh == 3 and L.kw == 3 and L.stride == 1 and
                L.bn is None and L.cout % 32 == 0 and L.act == ACT_LEAKY):
            return False
    last = layers[-1]
    return last.kh == 3 and last.stride == 1 and last.cout <= 4 and last.cin_p == layers[-2].cout


def _img(shape, device):
    return torch.empty(shape, device=device, dtype=torch.bfloat16)


def _to_img16(t, ld):
    """fp32 NHWC -> bf16 image with ld channels (zero-padded)."""
    n, h, w, c = t.shape
    out = _img((n, h, w, ld), t.device)
    call("of_to_bf16_image", _ptr(t), n * h * w, c, c, _ptr(out), ld, _stream())
    return out


def _b16i_io(**kw):
    r = _lib.B16iIO()
    for k, v in kw.items():
        setattr(r, k, v.data_ptr() if isinstance(v, torch.Tensor) else v)
    return r


def _stack_fwd_img16(layers, x):
    """Forward of a bf16 flow head on images: returns (saved tensors, output)."""
    nb, h, w, cx = x.shape
    s = _stream()
    x16 = getattr(x, "_of_img16", None)   # written by corr_concat directly
    if x16 is None:
        x16 = _to_img16(x.contiguous(), (cx + 31) // 32 * 32)
    imgs, masks = [x16], []
    cur = x16
    for i, layer in enumerate(layers[:-2]):
        d = layer.desc(nb, h, w)
        wf, _ = layer.packed(d)
        y16 = _img((nb, h, w, layer.cout), x.device)
        # the output's act' signs, in the layout the next layer's input gradient reads them
        mask = (torch.empty(_lib.lib().of_conv2d_b16i_mask_bytes(C.byref(d)) // 4,
                            dtype=torch.int32, device=x.device) if B16I_MASK else None)
        _tag(layer, 0)
        io = _b16i_io(a16=cur, lda16=cur.shape[-1], y16=y16, ldy16=layer.cout, mask_out=mask)
        call("of_conv2d_b16i", 0, C.byref(d), C.byref(io), _ptr(wf), _ptr(layer.bias), None, None,
             None, None, BN_EPS, layer.act, layer.alpha, s)
        imgs.append(y16)
        masks.append(mask)
        cur = y16
    l4 = layers[-2]                      # fp32 output: the narrow flow conv reads it
    d = l4.desc(nb, h, w)
    wf, _ = l4.packed(d)
    y4 = torch.empty((nb, h, w, l4.cout), device=x.device)
    _tag(l4, 0)
    io = _b16i_io(a16=cur, lda16=cur.shape[-1], y=y4, ldy=l4.cout)
    call("of_conv2d_b16i", 0, C.byref(d), C.byref(io), _ptr(wf), _ptr(l4.bias), None, None, None,
         None, BN_EPS, l4.act, l4.alpha, s)
    l5 = layers[-1]
    d = l5.desc(nb, h, w)
    wf, _ = l5.packed(d)
    y5 = torch.empty((nb, h, w, l5.cout), device=x.device)
    _tag(l5, 0)
    entry, wsz = l5.fwd_entry(d)
    wsk, wsp, wsb = _workspace(wsz, x.device)
    call(entry, C.byref(d), _ptr(y4), l4.cout, _ptr(wf), _ptr(l5.bias), None, None, None, None,
         BN_EPS, None, 0, l5.act, l5.alpha, None, 0, _ptr(y5), l5.cout, wsp, wsb, s)
    return imgs + [y4, y5] + masks, y5


def _wgrad_img16(layer, d, x16, dy16, tk, part=None, dy32=None):
    """Weight gradient of one head conv from images + its bias gradient (from the column
    sums the input-gradient kernel left in ``part``, or from the fp32 dy32)."""
    tb = grad_target(layer.bias)
    if tk[1] != tb[1]:
        raise RuntimeError("kernel and bias gradients must both use the arena or not")
    side = SIDE_STREAM_WGRAD and tk[1] == 1 and d.n * d.ho * d.wo <= _side_max_pix(layer)
    with torch.cuda.stream(side_stream(x16, dy16, part, dy32)) if side else \
            contextlib.nullcontext():
        ss = _stream()
        wsb = _lib.lib().of_conv2d_wgrad_b16i_workspace(C.byref(d))
        ws = torch.empty(wsb // 4 + 1, device=x16.device)
        _tag(layer, 2)
        call("of_conv2d_wgrad_b16i", C.byref(d), _ptr(x16), x16.shape[-1], _ptr(dy16),
             dy16.shape[-1], _ptr(tk[0]), tk[1], None, None, 0.0, _ptr(ws), wsb, ss)
        if part is not None:
            call("of_col_part_reduce", _ptr(part), part.shape[0], layer.cout, _ptr(tb[0]), tb[1],
                 ss)
        else:
            npix = dy32.numel() // dy32.shape[-1]
            cws = torch.empty(_lib.lib().of_colsum_workspace(npix, layer.cout) // 4 + 1,
                              device=dy32.device)
            call("of_colsum", _ptr(dy32), npix, layer.cout, dy32.shape[-1], _ptr(tb[0]), tb[1],
                 _ptr(cws), ss)
    return tb


def _stack_bwd_img16(layers, saved, g, need_x):
    """Backward of _stack_fwd_img16 (g: the padded flow gradient of the last conv)."""
    nimg = len(layers) - 1                 # x16 and the outputs of the bf16-image layers
    imgs, (y4, y5), masks = saved[:nimg], saved[nimg:nimg + 2], saved[nimg + 2:]
    nb, h, w, _ = y4.shape
    s = _stream()
    rets = {}
    l5, l4 = layers[-1], layers[-2]
    # c5 (narrow, fp32): weight gradient and input gradient (with c4's LeakyReLU derivative)
    d5 = l5.desc(nb, h, w)
    _, wd5 = l5.packed(d5)
    tk5, tb5 = grad_target(l5.kernel), grad_target(l5.bias)
    wgrad_stack(l5, y4, g, d5, tk5, tb5)
    _grad_ready(l5.kernel, l5.bias)
    gy4 = torch.empty_like(y4)
    _tag(l5, 1)
    entry, wsz = l5.dgrad_entry(d5)
    wsk, wsp, wsb = _workspace(wsz, y4.device)
    call(entry, C.byref(d5), _ptr(g), g.shape[-1], _ptr(wd5), _ptr(y4), l4.cout, l4.act, l4.alpha,
         _ptr(gy4), l4.cout, wsp, wsb, s)
    rets[l5.name] = (tk5[2], tb5[2])
    dy16 = _to_img16(gy4, l4.cout)
    dy32 = gy4
    part = None
    dx = None
    for i in range(len(layers) - 2, -1, -1):
        layer = layers[i]
        x16 = imgs[i]
        d = layer.desc(nb, h, w)
        _, wd = layer.packed(d)
        tk = grad_target(layer.kernel)
        tb = _wgrad_img16(layer, d, x16, dy16, tk, part=part, dy32=dy32 if part is None else None)
        _grad_ready(layer.kernel, layer.bias)
        rets[layer.name] = (tk[2], tb[2])
        if i > 0:
            prev = layers[i - 1]
            tiles = _lib.lib().of_conv2d_b16i_tiles(1, C.byref(d))
            part = torch.empty((tiles, layer.cin_p), device=y4.device)
            gx16 = _img((nb, h, w, layer.cin_p), y4.device)
            _tag(layer, 1)
            # act' of the producer (layer i - 1): the signs its forward wrote, or its image
            mk = masks[i - 1] if masks[i - 1] is not None else None
            io = _b16i_io(a16=dy16, lda16=dy16.shape[-1], y16=gx16, ldy16=layer.cin_p,
                          act16=None if mk is not None else x16, ld_act16=x16.shape[-1],
                          col_part=part, mask_in=mk)
            call("of_conv2d_b16i", 1, C.byref(d), C.byref(io), _ptr(wd), None, None, None, None,
                 None, 0.0, prev.act, prev.alpha, s)
            dy16, dy32 = gx16, None
        elif need_x:
            dx = torch.empty((nb, h, w, layer.cin_p), device=y4.device)
            _tag(layer, 1)
            io = _b16i_io(a16=dy16, lda16=dy16.shape[-1], y=dx, ldy=layer.cin_p)
            call("of_conv2d_b16i", 1, C.byref(d), C.byref(io), _ptr(wd), None, None, None, None,
                 None, 0.0, ACT_NONE, 0.0, s)
    out = []
    for layer in layers:
        out += list(rets[layer.name])
    return dx, out


class _ConvStackFn(torch.autograd.Function):
    """A chain of plain convs (bias + activation, no BN / residual): the six-conv flow head
    of ``flow_module`` (model.py:104-114).  The backward is fused across layers: each input
    gradient kernel multiplies by the producer layer's LeakyReLU derivative in its epilogue
    (act_src = that layer's saved output), so no separate activation-backward pass runs.
    bf16 heads on large grids keep their activations as bf16 images (_img16_ok)."""

    @staticmethod
    def forward(ctx, x, *args):
        layers, ctx.fg = args[-1], args[-2]
        args = args[:-1]
        n = len(layers)
        _check_dev(x)
        ctx.img16 = _img16_ok(layers, x)
        if ctx.img16:
            saved, out = _stack_fwd_img16(layers, x)
            ctx.layers = layers
            ctx.save_for_backward(*saved)
            return out
        if getattr(x, "_of_img16", None) is not None:
            # corr_concat wrote only the bf16 image (its fp32 output is a placeholder)
            raise RuntimeError("conv stack: the input carries only a bf16 concat image, but "
                               "this stack does not run on images")
        x = x.contiguous()
        s = _stream()
        acts = [x]
        for i, layer in enumerate(layers):
            assert layer.bn is None
            nb, h, w, cx = acts[-1].shape
            assert cx == layer.cin_p, "conv %s: %d channels, expected %d" % (layer.name, cx,
                                                                             layer.cin_p)
            d = layer.desc(nb, h, w)
            wf, _ = layer.packed(d)
            y = torch.empty((nb, d.ho, d.wo, layer.cout), device=x.device)
            _tag(layer, 0)
            entry, wsz = layer.fwd_entry(d)
            wsk, wsp, wsb = _workspace(wsz, x.device)
            call(entry, C.byref(d), _ptr(acts[-1]), cx, _ptr(wf), _ptr(layer.bias),
                 None, None, None, None, BN_EPS, None, 0, layer.act, layer.alpha, None, 0,
                 _ptr(y), layer.cout, wsp, wsb, s)
            if i + 1 < n:
                assert layers[i + 1].cin_p == layer.cout, "stacked convs need cout % 4 == 0"
            acts.append(y)
        ctx.layers = layers
        ctx.save_for_backward(*acts)
        return acts[-1]

    @staticmethod
    def backward(ctx, dy):
        layers = ctx.layers
        acts = ctx.saved_tensors
        s = _stream()
        n = len(layers)
        needs = ctx.needs_input_grad
        fg = ctx.fg
        if (fg is not None and fg.filled and dy.data_ptr() == fg.buffer().data_ptr() and
                dy.stride()[-2] == 4):
            g = fg.buffer()                 # loss (+ upscale) gradient, already padded
            fg.filled = fg.added = False
            ctx.fg_release = fg             # back to the pool once its readers are enqueued
        else:
            if fg is not None and fg.added:
                # autograd summed the loss gradient with a further consumer's before the
                # upscale backward added its part into the buffer: that part is not in dy
                raise RuntimeError("flow gradient routing: this flow has consumers besides the "
                                   "photometric loss and upscale_flow; run with "
                                   "OFLOW_FLOW_GRAD_ROUTING=0")
            if fg is not None:
                fg.filled = False
            g = _pad_channels(dy.contiguous(), _c4(layers[-1].cout))
        if ctx.img16:
            assert layers[-1].act == ACT_NONE
            dx, rets = _stack_bwd_img16(layers, acts, g, needs[0])
            if getattr(ctx, "fg_release", None) is not None:
                ctx.fg_release.release()
            return (dx, *rets, None, None)
        if layers[-1].act != ACT_NONE:
            gz = torch.empty_like(g)
            y = _pad_channels(acts[-1], g.shape[-1])
            call("of_act_bwd", _ptr(g), _ptr(y), layers[-1].act, layers[-1].alpha, _ptr(gz),
                 g.numel(), s)
            g = gz
        dx = None
        for i in range(n - 1, -1, -1):
            layer = layers[i]
            x = acts[i]
            nb, h, w, cx = x.shape
            d = layer.desc(nb, h, w)
            _, wd = layer.packed(d)
            tk = grad_target(layer.kernel)
            tb = grad_target(layer.bias)
            if tk[1] != tb[1]:
                raise RuntimeError("kernel and bias gradients must both use the arena or not")
            # weight gradient, input gradient (order: DGRAD_FIRST) from the same g
            gx = None
            if not DGRAD_FIRST:
                wgrad_stack(layer, x, g, d, tk, tb)
                _grad_ready(layer.kernel, layer.bias)     # the all-reduce forks before dgrad
            if i > 0:
                prev = layers[i - 1]
                gx = torch.empty((nb, h, w, cx), device=x.device)
                _tag(layer, 1)
                entry, wsz = layer.dgrad_entry(d)
                wsk, wsp, wsb = _workspace(wsz, x.device)
                call(entry, C.byref(d), _ptr(g), g.shape[-1], _ptr(wd), _ptr(x), cx,
                     prev.act, prev.alpha, _ptr(gx), cx, wsp, wsb, s)
            elif needs[0]:
                dx = torch.empty((nb, h, w, cx), device=x.device)
                _tag(layer, 1)
                entry, wsz = layer.dgrad_entry(d)
                wsk, wsp, wsb = _workspace(wsz, x.device)
                call(entry, C.byref(d), _ptr(g), g.shape[-1], _ptr(wd), None, 0,
                     ACT_NONE, 0.0, _ptr(dx), cx, wsp, wsb, s)
            if DGRAD_FIRST:
                wgrad_stack(layer, x, g, d, tk, tb)
                _grad_ready(layer.kernel, layer.bias)
            layer._ret = (tk[2], tb[2])
            if gx is not None:
                g = gx
        rets = []
        for layer in layers:
            rets += list(layer._ret)
            layer._ret = None
        if getattr(ctx, "fg_release", None) is not None:
            ctx.fg_release.release()
        return (dx, *rets, None, None)


def wgrad_stack(layer, x, g, d, tk, tb):
    """Weight + bias gradient of one conv of a _ConvStackFn (side stream for small layers)."""
    cx = x.shape[-1]
    went, wsb = layer.wgrad_entry(d)
    side = SIDE_STREAM_WGRAD and tk[1] == 1 and d.n * d.ho * d.wo <= _side_max_pix(layer)
    with torch.cuda.stream(side_stream(x, g)) if side else contextlib.nullcontext():
        ws = torch.empty(wsb // 4 + 1, device=x.device)
        _tag(layer, 2)
        call(went, C.byref(d), _ptr(x), cx, _ptr(g), g.shape[-1], _ptr(tk[0]),
             _ptr(tb[0]), tk[1], _ptr(ws), wsb, _stream())


FLOW_GRAD_ROUTING = os.environ.get("OFLOW_FLOW_GRAD_ROUTING", "1") == "1"


def conv_stack(x, layers):
    flat = []
    for layer in layers:
        flat += [layer.kernel, layer.bias]
    fg = None
    if FLOW_GRAD_ROUTING and layers[-1].cout == 2 and x.is_cuda:     # a flow head (model.py:114)
        n, h, w, _ = x.shape
        fg = FlowGrad((n, h, w, 2), x.device)
    out = _ConvStackFn.apply(x, *flat, fg, list(layers))
    if fg is not None:
        out._of_flowgrad = fg
    return out


# ========================================================================= max pool ====
class _MaxPool2(torch.autograd.Function):
    """layers.MaxPool2D() (model.py:17): 2x2 / stride 2 / valid."""

    @staticmethod
    def forward(ctx, x):
        _check_dev(x)
        x = x.contiguous()
        n, h, w, c = x.shape
        y = torch.empty((n, h // 2, w // 2, c), device=x.device)
        call("of_maxpool2_fwd", _ptr(x), n, h, w, c, _ptr(y), _stream())
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        n, h, w, c = x.shape
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        call("of_maxpool2_bwd", _ptr(x), _ptr(dy), n, h, w, c, _ptr(dx), _stream())
        return dx


def maxpool2(x):
    return _MaxPool2.apply(x)


# ===================================================================== cost volume =====
class _CostVolume(torch.autograd.Function):
    """create_cost_volume(f1, f2, max_disp) (model.py:29-42)."""

    @staticmethod
    def forward(ctx, f1, f2, max_disp):
        _check_dev(f1, f2)
        f1, f2 = f1.contiguous(), f2.contiguous()
        n, h, w, c = f1.shape
        nk = (2 * max_disp + 1) ** 2
        out = torch.empty((n, h, w, nk), device=f1.device)
        ws, wp, wb = _workspace(_lib.lib().of_corr_fwd_workspace(n, h, w, c, max_disp), f1.device)
        call("of_corr_fwd", _ptr(f1), c, _ptr(f2), c, n, h, w, c, max_disp, _ptr(out), nk, wp,
             wb, _stream())
        ctx.save_for_backward(f1, f2)
        ctx.max_disp = max_disp
        return out

    @staticmethod
    def backward(ctx, dcv):
        f1, f2 = ctx.saved_tensors
        n, h, w, c = f1.shape
        dcv = dcv.contiguous()
        df1 = torch.empty_like(f1) if ctx.needs_input_grad[0] else None
        df2 = torch.empty_like(f2) if ctx.needs_input_grad[1] else None
        call("of_corr_bwd", _ptr(dcv), dcv.shape[-1], _ptr(f1), c, _ptr(f2), c, n, h, w, c,
             ctx.max_disp, _ptr(df1), c, 0, _ptr(df2), c, 0, _stream())
        return df1, df2, None


def cost_volume(f1, f2, max_disp=3):
    return _CostVolume.apply(f1, f2, max_disp)


class _CorrConcat(torch.autograd.Function):
    """The flow-module input ``concat([features1, cost_volume, flow_up])`` (model.py:97-102)
    built in one zero-padded NHWC buffer of ``cp`` channels by one kernel (f1 copy, cost
    volume, flow and padding per pixel row); the backward reads the f1 slice of the gradient
    as the initial value of df1 (no copy or concat passes)."""

    @staticmethod
    def forward(ctx, f1, f2w, flow_up, max_disp, cp, fa, df1_side=False, img=None):
        _check_dev(f1, f2w, flow_up)
        ctx.fa = fa
        ctx.df1_side = df1_side
        f1, f2w = f1.contiguous(), f2w.contiguous()
        n, h, w, c = f1.shape
        nk = (2 * max_disp + 1) ** 2
        used = c + nk + (2 if flow_up is not None else 0)
        assert used <= cp
        if img is not None:
            # the fp32 row is never written on this path: a zero-stride placeholder of the
            # row's shape is the autograd output (no (n, h, w, cp) allocation per level)
            x = torch.empty((1, 1, 1, 1), device=f1.device).expand(n, h, w, cp)
        else:
            x = torch.empty((n, h, w, cp), device=f1.device)
        ctx.dst = (grad_dst(f1), grad_dst(f2w))
        fu = flow_up.contiguous() if flow_up is not None else None
        if img is not None:
            # the consumer (a bf16-image flow head) reads only the row's bf16 image: written
            # directly, x stays unwritten (its shape and gradient are the autograd interface)
            x16 = _img((n, h, w, img["ld"]), f1.device)
            call("of_corr_concat_fwd16", _ptr(f1), _ptr(f2w), _ptr(fu), n, h, w, c, max_disp,
                 _ptr(x16), img["ld"], _stream())
            img["x16"] = x16
        else:
            ws, wp, wb = _workspace(_lib.lib().of_corr_fwd_workspace(n, h, w, c, max_disp),
                                    f1.device)
            call("of_corr_concat_fwd", _ptr(f1), _ptr(f2w), _ptr(fu), n, h, w, c, max_disp,
                 _ptr(x), cp, wp, wb, _stream())
        ctx.save_for_backward(f1, f2w)
        ctx.meta = (max_disp, cp, nk, flow_up is not None)
        return x

    @staticmethod
    def backward(ctx, dx):
        f1, f2w = ctx.saved_tensors
        max_disp, cp, nk, has_flow = ctx.meta
        n, h, w, c = f1.shape
        dx = dx.contiguous()
        df1 = new_grad(ctx.dst[0], f1)
        df2 = new_grad(ctx.dst[1], f2w) if ctx.needs_input_grad[1] else None
        dflow = None
        defer = (has_flow and ctx.needs_input_grad[2] and ctx.fa is not None and
                 ctx.fa.warp_flow_grad)
        if defer:                      # the warp backward adds this slice (FlowAdd)
            ctx.fa.addend = (dx, c + nk, cp)
        elif has_flow and ctx.needs_input_grad[2]:
            dflow = torch.empty((n, h, w, 2), device=dx.device)
        if ctx.df1_side and dx.is_cuda and _in_slab(ctx.dst[0], df1):
            # df1 lands in the encoder output's gradient slab: its only reader is the encoder
            # backward (corr_side_wait there and in _Halves' copy path); a df1 that autograd
            # would sum with another consumer's gradient stays on the current stream
            s = _stream()
            if df2 is not None:
                call("of_corr_bwd", C.c_void_p(dx.data_ptr() + 4 * c), cp, _ptr(f1), c,
                     _ptr(f2w), c, n, h, w, c, max_disp, None, c, 0, _ptr(df2), c, 0, s)
            if dflow is not None:
                call("of_copy_strided", C.c_void_p(dx.data_ptr() + 4 * (c + nk)), cp,
                     _ptr(dflow), 2, n * h * w, 2, s)
            with torch.cuda.stream(corr_side_stream(dx, f1, f2w, df1)):
                call("of_corr_concat_bwd", _ptr(dx), cp, _ptr(f1), _ptr(f2w), n, h, w, c,
                     max_disp, _ptr(df1), None, None, _stream())
            return df1, df2, dflow, None, None, None, None, None
        call("of_corr_concat_bwd", _ptr(dx), cp, _ptr(f1), _ptr(f2w), n, h, w, c, max_disp,
             _ptr(df1), _ptr(df2), _ptr(dflow), _stream())
        return df1, df2, dflow, None, None, None, None, None


def corr_concat(f1, f2w, flow_up, max_disp, cp, precision="fp32", layers=None):
    """``precision``: that of the flow module's convs; it picks whether df1 runs on a stream
    of its own (corr_df1_side).  ``layers``: the head convs that will read the result; when
    they run on bf16 images (_img16_ok) the concat is written as that image directly
    (of_corr_concat_fwd16, attached to the result as ``_of_img16``) and the fp32 row is not
    written."""
    fa = getattr(flow_up, "_of_flowadd", None) if flow_up is not None else None
    img = None
    if (layers is not None and CONCAT_IMG16 and f1.is_cuda and
            _img16_ok(layers, f1) and layers[0].cin_p == cp and
            _lib.lib().of_corr_concat_fwd16_ok(*f1.shape) == 1):
        img = {"ld": (cp + 31) // 32 * 32}
    x = _CorrConcat.apply(f1, f2w, flow_up, max_disp, cp, fa, corr_df1_side(precision), img)
    if img is not None:
        x._of_img16 = img["x16"]
    return x


# ============================================================================ warp =====
class _Warp(torch.autograd.Function):
    """warp_features (model.py:55-73) / bilinear_interpolation (transformations.py:85-129)."""

    @staticmethod
    def forward(ctx, inp, flow, absolute, fa=None):
        _check_dev(inp, flow)
        ctx.fa = fa
        if fa is not None and flow.requires_grad:
            fa.warp_flow_grad = True
        inp, flow = inp.contiguous(), flow.contiguous()
        n, h, w, c = inp.shape
        assert flow.shape == (n, h, w, 2), "flow must be (B, h, w, 2) like features"
        out = torch.empty_like(inp)
        ctx.dst = grad_dst(inp)
        call("of_bilinear_fwd" if absolute else "of_warp_fwd", _ptr(inp), n, h, w, c,
             _ptr(flow), _ptr(out), _stream())
        ctx.save_for_backward(inp, flow)
        ctx.absolute = absolute
        return out

    @staticmethod
    def backward(ctx, dout):
        inp, flow = ctx.saved_tensors
        n, h, w, c = inp.shape
        dout = dout.contiguous()
        s = _stream()
        dinp = None
        if ctx.needs_input_grad[0]:
            dinp = new_grad(ctx.dst, inp)
        dflow = torch.empty_like(flow)
        fa = ctx.fa
        if DETERMINISTIC:       # fixed-order gather / exact fixed point: dinp written, no fill
            add, ld = None, 0
            if fa is not None and fa.addend is not None and ctx.needs_input_grad[1]:
                dcat, off, ld = fa.addend
                add = C.c_void_p(dcat.data_ptr() + 4 * off)
                fa.addend = None
            wsk, wsp, wsb = _workspace(
                _lib.lib().of_warp_bwd_det_workspace(n, h, w, c) if dinp is not None else 0,
                dout.device)
            call("of_warp_bwd_det", _ptr(dout), _ptr(inp), n, h, w, c, _ptr(flow),
                 int(ctx.absolute), _ptr(dinp), _ptr(dflow), add, ld, wsp, wsb, s)
            return dinp, (dflow if ctx.needs_input_grad[1] else None), None, None
        if dinp is not None:
            call("of_fill", _ptr(dinp), 0.0, dinp.numel(), s)
        if fa is not None and fa.addend is not None and ctx.needs_input_grad[1]:
            dcat, off, ld = fa.addend            # the concat's flow slice (FlowAdd)
            call("of_warp_bwd_add", _ptr(dout), _ptr(inp), n, h, w, c, _ptr(flow), _ptr(dinp),
                 _ptr(dflow), C.c_void_p(dcat.data_ptr() + 4 * off), ld, s)
            fa.addend = None
        else:
            call("of_bilinear_bwd" if ctx.absolute else "of_warp_bwd", _ptr(dout), _ptr(inp), n,
                 h, w, c, _ptr(flow), _ptr(dinp), _ptr(dflow), s)
        return dinp, (dflow if ctx.needs_input_grad[1] else None), None, None


def warp(inp, flow):
    return _Warp.apply(inp, flow, False, getattr(flow, "_of_flowadd", None))


def bilinear(inp, points):
    return _Warp.apply(inp, points, True)


# ====================================================================== upscale x2 =====
class _Upscale2x(torch.autograd.Function):
    """upscale_flow (model.py:76-77): resize x2 (half-pixel bilinear) times 2.0."""

    @staticmethod
    def forward(ctx, x, scale, fg=None):
        _check_dev(x)
        ctx.fg = fg
        x = x.contiguous()
        n, h, w, c = x.shape
        out = torch.empty((n, 2 * h, 2 * w, c), device=x.device)
        call("of_upscale2x_fwd", _ptr(x), n, h, w, c, scale, _ptr(out), c, _stream())
        ctx.shape = (n, h, w, c)
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, dout):
        n, h, w, c = ctx.shape
        dout = dout.contiguous()
        fg = ctx.fg
        if fg is not None and fg.filled and c == 2:
            # add into the loss gradient of the same flow (FlowGrad); autograd gets None
            call("of_upscale2x_bwd_ld", _ptr(dout), c, n, h, w, c, ctx.scale, _ptr(fg.buffer()),
                 4, 1, _stream())
            fg.added = True
            return None, None, None
        dx = torch.empty((n, h, w, c), device=dout.device)
        call("of_upscale2x_bwd", _ptr(dout), c, n, h, w, c, ctx.scale, _ptr(dx), 0, _stream())
        return dx, None, None


def upscale2x(x, scale=2.0):
    out = _Upscale2x.apply(x, scale, getattr(x, "_of_flowgrad", None))
    if FLOW_GRAD_ROUTING and out.requires_grad:
        out._of_flowadd = FlowAdd()
    return out


# ================================================================= Siamese batching ====
def split_pair(batch_imgs):
    """(B,H,W,6) -> (2B,H,W,4): image1s then image2s, 4th channel zero (model.py:122-123);
    the images are constants of the graph (no gradient)."""
    _check_dev(batch_imgs)
    b = batch_imgs.contiguous()
    n, h, w, c = b.shape
    assert c == 6
    out = torch.empty((2 * n, h, w, 4), device=b.device)
    call("of_split_pair", _ptr(b), n, h, w, _ptr(out), _stream())
    return out


class GradSlab:
    """The (2B, ...) gradient buffer of a Siamese activation, allocated on first use.  The
    backward of a consumer of one half writes that half's gradient straight into it
    (``grad_dst``), so _Halves.backward returns the slab without copying.  A half is handed
    out once; a second consumer of the same half gets a fresh tensor (autograd then sums as
    usual and _Halves falls back to copying)."""

    def __init__(self, shape, device):
        self.shape, self.device = tuple(shape), device
        self.full = None
        self.given = [False, False]

    def half(self, k):
        n = self.shape[0] // 2
        if self.given[k]:
            return torch.empty((n,) + self.shape[1:], device=self.device)
        if self.full is None:
            self.full = torch.empty(self.shape, device=self.device)
        self.given[k] = True
        return self.full.narrow(0, k * n, n)


def grad_dst(t):
    """Forward-time capture: where the gradient of input ``t`` should be written."""
    return getattr(t, "_of_grad_slab", None)


def _in_slab(dst, g) -> bool:
    """True when ``g`` is the GradSlab half that grad_dst() captured (not a fresh tensor
    handed to a second consumer of the same half)."""
    if dst is None or dst[0].full is None:
        return False
    slab, k = dst
    return g.data_ptr() == slab.full.data_ptr() + k * (slab.full.numel() // 2) * 4


def new_grad(dst, like):
    """Backward-time buffer for an input gradient captured by grad_dst()."""
    if dst is not None:
        return dst[0].half(dst[1])
    return torch.empty_like(like)


class FlowGrad:
    """Gradient routing for a flow head's output flow (B, h, w, 2) (model.py:114), whose
    consumers are the photometric loss (loss.py:20-30) and, for the coarser levels,
    upscale_flow (model.py:76-77).  The loss backward writes d(flow) into a channel-padded
    (B, h, w, 4) buffer (channels 2-3 stay zero) and returns a view of it; the upscale
    backward, which autograd runs afterwards, adds its input gradient into the same buffer
    and returns None; the flow head's backward then reads the buffer as its padded dy.  This
    replaces autograd's add pass and the channel-padding fill + copy per level.  Each FlowGrad
    (one per forward of a flow head) owns its buffer from first use until the head's backward
    has consumed it (or the FlowGrad is dropped): two forwards before one backward (micro-batch
    accumulation, two same-shape models) get distinct buffers.  Released buffers are pooled per
    (device, shape) for the next steps; stream order protects their reuse."""
    _pool = {}

    def __init__(self, shape, device):
        self.shape, self.device = tuple(shape), device
        self.filled = False             # the loss backward wrote the buffer this backward
        self.added = False              # the upscale backward added into it
        self._buf = None

    def _key(self):
        return (str(self.device), self.shape)

    def buffer(self):
        if self._buf is None:
            free = FlowGrad._pool.setdefault(self._key(), [])
            self._buf = free.pop() if free else torch.zeros(self.shape[:3] + (4,),
                                                            device=self.device)
        return self._buf

    def release(self):
        """Return the buffer to the pool (its consumers are enqueued; channels 2-3 stay 0).
        Inside a backward that forked side streams the head's weight gradient may still read
        the buffer there, and the next pop would write it on the current stream with nothing
        ordering the two (two forwards, one backward: loss 1's FlowGrad pops the buffer that
        forward 2's backward released).  The buffer is then pooled at the end-of-backward
        join (_side_join), after the current stream waits for the side streams."""
        if self._buf is not None:
            if _side_armed:
                _DEFERRED_RELEASE.append((self._key(), self._buf))
            else:
                FlowGrad._pool.setdefault(self._key(), []).append(self._buf)
            self._buf = None

    def __del__(self):
        try:
            self.release()
        except Exception:       # interpreter shutdown
            pass


class FlowAdd:
    """Gradient routing for an upscaled flow (flow_up, model.py:91-102) that feeds both
    warp_features and the concat: the concat backward (autograd runs it first) leaves its
    flow-slice gradient here instead of returning it, and the warp backward adds it in its
    d(flow) store (of_warp_bwd_add) -- the same fp32 sum without autograd's add pass."""

    def __init__(self):
        self.warp_flow_grad = False     # a warp of this flow computes d(flow)
        self.addend = None              # (concat gradient tensor, channel offset, row stride)


class _Halves(torch.autograd.Function):
    """Split a (2B, ...) Siamese activation into its two (B, ...) halves; the backward returns
    the GradSlab both halves' gradients were written into (no copies when the consumers used
    it), else writes them into one buffer."""

    @staticmethod
    def forward(ctx, x, slab):
        n = x.shape[0] // 2
        ctx.shape = x.shape
        ctx.slab = slab
        return x.narrow(0, 0, n), x.narrow(0, n, n)

    @staticmethod
    def backward(ctx, g1, g2):
        shape = ctx.shape
        slab = ctx.slab
        n = shape[0] // 2
        if slab.full is not None and g1 is not None and g2 is not None:
            base = slab.full.data_ptr()
            half_bytes = slab.full.numel() // 2 * slab.full.element_size()
            if (g1.data_ptr() == base and g2.data_ptr() == base + half_bytes and
                    g1.is_contiguous() and g2.is_contiguous()):
                return slab.full, None
        dev = (g1 if g1 is not None else g2).device
        corr_side_wait(dev)                  # a df1 may still be in flight on its stream
        out = torch.empty(shape, device=dev)
        half = out.numel() // 2
        s = _stream()
        for k, g in enumerate((g1, g2)):
            dst = C.c_void_p(out.data_ptr() + 4 * k * half)
            if g is None:
                call("of_fill", dst, 0.0, half, s)
            else:
                g = g.contiguous()
                call("of_copy_strided", _ptr(g), 1, dst, 1, half, 1, s)
        return out, None


def halves(x):
    slab = GradSlab(x.shape, x.device)
    f1, f2 = _Halves.apply(x, slab)
    f1._of_grad_slab = (slab, 0)
    f2._of_grad_slab = (slab, 1)
    return f1, f2


# ================================================================ photometric loss =====
class _PhotoLoss(torch.autograd.Function):
    """LossLayer.__call__ (loss.py:5-32): mean over scales of mean |img1_s - warp(img2_s)|.
    The image pyramid (tf.image.resize) is built by one kernel per level; the warp, the
    difference, |.| and the reduction are fused per scale; the backward writes d(flow) per
    scale directly (the images are constants)."""

    @staticmethod
    def forward(ctx, batch_imgs, fgs, *flows):
        _check_dev(batch_imgs, *flows)
        ctx.fgs = fgs
        b = batch_imgs.contiguous()
        n, H, W, c = b.shape
        assert c == 6
        ns = len(flows)
        s = _stream()
        pyr = []
        for k in range(ns):
            h = int(H / (2.0 ** (k + 1)))
            w = int(W / (2.0 ** (k + 1)))
            assert flows[k].shape[1] == h and flows[k].shape[2] == w, \
                "flow %d has shape %s, expected (B,%d,%d,2)" % (k, tuple(flows[k].shape), h, w)
            pyr.append(torch.empty((n, h, w, 6), device=b.device))
        # every level is a resize of the full-resolution batch (loss.py:17-18)
        outs = (C.c_void_p * ns)(*[p.data_ptr() for p in pyr])
        call("of_pyramid6", _ptr(b), n, H, W, ns, outs, s)
        # every scale's partial sums in one launch (of_photo_l1_fwd_multi), one partial array
        fl = [f.contiguous() for f in flows]
        hs = [p.shape[1] for p in pyr]
        ws_ = [p.shape[2] for p in pyr]
        nparts = [_lib.lib().of_photo_l1_partials(n, h, w) for h, w in zip(hs, ws_)]
        coefs = [1.0 / (ns * n * h * w * 3) for h, w in zip(hs, ws_)]
        parts = torch.empty(sum(nparts), device=b.device)
        call("of_photo_l1_fwd_multi", (C.c_void_p * ns)(*[p.data_ptr() for p in pyr]),
             (C.c_void_p * ns)(*[f.data_ptr() for f in fl]), n, (C.c_int * ns)(*hs),
             (C.c_int * ns)(*ws_), ns, _ptr(parts), s)
        offs = [0]
        for k in range(ns):
            offs.append(offs[-1] + nparts[k])
        loss = torch.empty((), device=b.device)
        call("of_sum_partials",
             (C.c_void_p * ns)(*[parts.data_ptr() + 4 * offs[k] for k in range(ns)]),
             (C.c_int * ns)(*nparts), (C.c_float * ns)(*coefs), ns, _ptr(loss), s)
        ctx.save_for_backward(*pyr, *fl)
        ctx.ns = ns
        ctx.coefs = coefs
        return loss

    @staticmethod
    def backward(ctx, dloss):
        ns = ctx.ns
        saved = ctx.saved_tensors
        pyr, flows = saved[:ns], saved[ns:]
        dloss = dloss.contiguous()
        s = _stream()
        grads, lv = [], []          # lv: (level, output, row stride) of one multi launch
        for k in range(ns):
            if not ctx.needs_input_grad[2 + k]:
                grads.append(None)
                continue
            fg = ctx.fgs[k]
            if fg is not None:         # into the flow head's padded gradient (FlowGrad)
                buf = fg.buffer()
                fg.filled = True
                grads.append(buf[..., :2])
                lv.append((k, buf, 4))
                continue
            df = torch.empty_like(flows[k])
            grads.append(df)
            lv.append((k, df, 2))
        if lv:
            m = len(lv)
            n = pyr[0].shape[0]
            call("of_photo_l1_bwd_multi", (C.c_void_p * m)(*[pyr[k].data_ptr() for k, _, _ in lv]),
                 (C.c_void_p * m)(*[flows[k].data_ptr() for k, _, _ in lv]), n,
                 (C.c_int * m)(*[pyr[k].shape[1] for k, _, _ in lv]),
                 (C.c_int * m)(*[pyr[k].shape[2] for k, _, _ in lv]), m,
                 (C.c_float * m)(*[ctx.coefs[k] for k, _, _ in lv]), _ptr(dloss),
                 (C.c_void_p * m)(*[o.data_ptr() for _, o, _ in lv]),
                 (C.c_int * m)(*[ld for _, _, ld in lv]), s)
        return (None, None, *grads)


def photometric_loss(batch_imgs, flows):
    fgs = [getattr(f, "_of_flowgrad", None) for f in flows]
    if any(fg is not None and fg.shape != tuple(f.shape) for fg, f in zip(fgs, flows)):
        fgs = [None] * len(flows)
    return _PhotoLoss.apply(batch_imgs, fgs, *flows)
