"""optical_flow_amd -- MI355X-native (gfx950) training hot path of xianlopez/optical_flow.

Reference-compatible surface (see model.py / loss.py / train.py / transformations.py):
build_flow_net, reset18_encoder, flow_module, create_cost_volume, warp_features,
upscale_flow, LossLayer, bilinear_interpolation, KerasAdam, Trainer.

Every op on the path is a hand-written HIP kernel in liboflow.so (csrc/), reached through the
C ABI declared in include/oflow.h.  There is no CPU fallback: importing the model works
anywhere, running it requires the .so and a GPU.
"""
from .params import flow_net_spec, init_params  # noqa: F401

__all__ = ["build_flow_net", "reset18_encoder", "flow_module", "create_cost_volume",
           "warp_features", "upscale_flow", "LossLayer", "bilinear_interpolation",
           "KerasAdam", "Trainer"]


def __getattr__(name):
    if name in ("build_flow_net", "reset18_encoder", "flow_module", "create_cost_volume",
                "warp_features", "upscale_flow", "FlowNet"):
        from . import model
        return getattr(model, name)
    if name == "LossLayer":
        from .loss import LossLayer
        return LossLayer
    if name == "bilinear_interpolation":
        from .transformations import bilinear_interpolation
        return bilinear_interpolation
    if name in ("KerasAdam", "Trainer"):
        from . import train
        return getattr(train, name)
    raise AttributeError(name)
