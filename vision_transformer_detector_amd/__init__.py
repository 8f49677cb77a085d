"""MI355X-native forward path of westlake-moonlight/vision_transformer_detector.

Drop-in for the reference's `model(images, training=False)` / `model.predict` path
(`vision_transformer_detector.py:498-647`): the same `create_vision_transformer_detector`
kwargs, NHWC fp32 images in, (B, 17, 6) logits out, `transform_predictions` decode.
All arithmetic runs in hand-written gfx950 HIP kernels in `libvtd.so` (C-ABI:
`include/vtd.h`); importing this package fails if that library is missing.
"""
import os as _os

# Kernel arguments in device memory (HIP runtime option; +1.8 % on the C2 forward,
# profiles/r04_dev_kernarg_ab.log).  Takes effect only if the HIP runtime has not been
# initialised yet in this process; an explicit setting by the caller wins.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

from .detector import (Constants, Model, create_vision_transformer_detector,  # noqa: F401
                       decode_detections, detection_list, keras_default_init,
                       keras_weight_names, transform_predictions)
from .metrics import MeanAveragePrecision, iou_calculator  # noqa: F401
from . import presets  # noqa: F401
from .preprocess import get_image_tensors  # noqa: F401

__all__ = ["Constants", "Model", "create_vision_transformer_detector",
           "transform_predictions", "decode_detections", "detection_list", "presets",
           "MeanAveragePrecision", "iou_calculator", "get_image_tensors"]
