"""MI355X-native forward path of westlake-moonlight/vision_transformer_detector.

Drop-in for the reference's `model(images, training=False)` / `model.predict` path
(`vision_transformer_detector.py:498-647`): the same `create_vision_transformer_detector`
kwargs, NHWC fp32 images in, (B, 17, 6) logits out, `transform_predictions` decode.
All arithmetic runs in hand-written gfx950 HIP kernels in `libvtd.so` (C-ABI:
`include/vtd.h`); importing this package fails if that library is missing.
"""
import os as _os


def enable_device_kernel_arguments() -> bool:
    """Opt-in: kernel arguments in device memory (the HIP runtime's HIP_FORCE_DEV_KERNARG=1;
    +1.8 % on the C2 forward, profiles/r04_dev_kernarg_ab.log).  It changes how EVERY HIP
    kernel of the process receives its arguments and is read once, when the HIP runtime
    initialises, so call this before anything touches the GPU (bench.py and
    __graft_entry__.smoke do); an explicit HIP_FORCE_DEV_KERNARG setting wins.  Returns
    whether the setting takes effect in this process: False (with a warning) when the HIP
    runtime is already initialised here (e.g. after an earlier torch.cuda call), or when the
    environment already says otherwise.  VTD_DEV_KERNARG=1 in the environment does the same
    at import time."""
    import sys
    import warnings
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        warnings.warn("enable_device_kernel_arguments(): the HIP runtime is already initialised "
                      "in this process; HIP_FORCE_DEV_KERNARG has no effect now", RuntimeWarning)
        return False
    _os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
    return _os.environ["HIP_FORCE_DEV_KERNARG"] == "1"


if _os.environ.get("VTD_DEV_KERNARG", "0") == "1":
    enable_device_kernel_arguments()

from .detector import (Constants, Model, create_vision_transformer_detector,  # noqa: F401
                       decode_detections, detection_list, keras_default_init,
                       keras_weight_names, transform_predictions)
from .metrics import MeanAveragePrecision, iou_calculator  # noqa: F401
from . import presets  # noqa: F401
from .preprocess import get_image_tensors  # noqa: F401

__all__ = ["Constants", "Model", "create_vision_transformer_detector",
           "transform_predictions", "decode_detections", "detection_list", "presets",
           "MeanAveragePrecision", "iou_calculator", "get_image_tensors",
           "enable_device_kernel_arguments"]
