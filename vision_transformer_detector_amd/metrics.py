"""Detection metric on the device, mirroring the reference's API.

`MeanAveragePrecision` (vision_transformer_detector.py:1268-2060) and `iou_calculator`
(vision_transformer_detector.py:761-875) with the same names, arguments, state attributes
and results; the work runs in libvtd.so (vtd_map_update / vtd_map_result / vtd_iou,
include/vtd.h), one launch per batch update instead of the reference's Python loop over
images x 80 classes.  The state lives in device memory as torch tensors with the
reference Variables' shapes.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L
from .detector import transform_predictions


def _device_f32(x, device):
    t = x if torch.is_tensor(x) else torch.as_tensor(np.asarray(x, dtype=np.float32))
    return t.to(device=device, dtype=torch.float32).contiguous()


def iou_calculator(label_bbox, prediction_bbox):
    """vtd.py:761-875: IoU of the boxes at matching positions.  Both inputs have the
    same shape (..., k) with k >= 4; the last 4 channels are (x, y, height, width).
    Returns a (...) float32 tensor on the device."""
    dev = prediction_bbox.device if torch.is_tensor(prediction_bbox) and \
        prediction_bbox.is_cuda else torch.device("cuda")
    lb, pb = _device_f32(label_bbox, dev), _device_f32(prediction_bbox, dev)
    if lb.shape != pb.shape or lb.dim() == 0 or lb.shape[-1] < 4:
        raise ValueError(f"iou_calculator: shapes {tuple(lb.shape)} / {tuple(pb.shape)} must "
                         "match and end in >= 4 box channels")
    out = torch.empty(lb.shape[:-1], device=dev, dtype=torch.float32)
    n = out.numel()
    with torch.cuda.device(dev):
        L.check(L.lib.vtd_iou(lb.data_ptr(), pb.data_ptr(), n, lb.shape[-1], out.data_ptr(),
                              L.stream_ptr()), "vtd_iou")
    return out


class MeanAveragePrecision:
    """COCO-style AP of the reference (vtd.py:1268-2060): the mean over 10 IoU thresholds
    of the per-class AP averaged over the classes seen so far, computed from the latest
    LATEST_RELATED_IMAGES (3) related images per class, BBOXES_PER_IMAGE (14) entries
    each."""

    CLASSES, LATEST_RELATED_IMAGES, BBOXES_PER_IMAGE = L.MAP_CLASSES, L.MAP_LATEST, L.MAP_PER_IMAGE

    def __init__(self, name: str = "AP", device=None):
        self.name = name
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        if self.device.type != "cuda":
            raise ValueError("MeanAveragePrecision runs on the HIP device")
        C, Lt, P = self.CLASSES, self.LATEST_RELATED_IMAGES, self.BBOXES_PER_IMAGE
        self.latest_positive_bboxes = torch.zeros((C, Lt, P, 2), device=self.device)
        self.labels_quantity_per_image = torch.zeros((C, Lt), device=self.device)
        self.showed_up_classes = torch.zeros((C,), dtype=torch.bool, device=self.device)
        self._out = torch.zeros(11, device=self.device)
        self.reset_state()

    def _state_ptrs(self):
        return (self.latest_positive_bboxes.data_ptr(), self.labels_quantity_per_image.data_ptr(),
                self.showed_up_classes.data_ptr())

    def update_state(self, y_true, y_pred, sample_weight=None, use_transform_predictions=True):
        """vtd.py:1310-1862.  y_true: (B, boxes, 6) labels (class -8 marks empty rows);
        y_pred: (B, boxes, 6) model logits, or decoded predictions when
        use_transform_predictions=False.  `sample_weight` is accepted and ignored, as in
        the reference."""
        del sample_weight
        yt = _device_f32(y_true, self.device)
        yp = _device_f32(y_pred, self.device)
        if yt.dim() != 3 or yt.shape[-1] != 6 or yt.shape != yp.shape:
            raise ValueError(f"update_state: y_true {tuple(yt.shape)} and y_pred "
                             f"{tuple(yp.shape)} must both be (batch, boxes, 6)")
        if yt.shape[1] > L.MAP_MAX_BOXES:
            raise ValueError(f"update_state: at most {L.MAP_MAX_BOXES} boxes per image")
        if use_transform_predictions:
            yp = transform_predictions(yp)
        with torch.cuda.device(self.device):
            L.check(L.lib.vtd_map_update(*self._state_ptrs(), yt.data_ptr(), yp.data_ptr(),
                                         yt.shape[0], yt.shape[1], L.stream_ptr()),
                    "vtd_map_update")

    def _compute(self):
        with torch.cuda.device(self.device):
            L.check(L.lib.vtd_map_result(*self._state_ptrs(), self._out.data_ptr(),
                                         L.stream_ptr()), "vtd_map_result")
        return self._out

    def result(self):
        """vtd.py:1865-2049: the mAP as a 0-d float32 device tensor."""
        return self._compute()[10].clone()

    def average_precision_per_iou(self):
        """The 10 per-threshold APs result() averages (IoU 0.5, 0.55, ..., 0.95)."""
        return self._compute()[:10].clone()

    def reset_state(self):
        """vtd.py:2052-2060."""
        with torch.cuda.device(self.device):
            L.check(L.lib.vtd_map_reset(*self._state_ptrs(), L.stream_ptr()), "vtd_map_reset")
