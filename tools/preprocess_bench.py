"""vtd_resize_with_pad throughput: a batch of decoded 640x480 COCO-shaped uint8 images
(resident in HBM) -> the model's NHWC fp32 input at 608x608 and 224x224. Prints one JSON
line per target with images/s and achieved GB/s of algorithmic bytes (pixels read once,
output written once) against the 8 TB/s HBM peak.

  python tools/preprocess_bench.py [--batch 256] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_transformer_detector_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, h, w = a.batch, 480, 640
    g = torch.Generator(device=dev).manual_seed(0)
    pixels = torch.randint(0, 256, (B * h * w * 3,), generator=g, device=dev, dtype=torch.uint8)
    offs = torch.arange(B, device=dev, dtype=torch.int64) * (h * w * 3)
    sizes = torch.tensor([[h, w]] * B, device=dev, dtype=torch.int32)
    for th, tw in ((608, 608), (224, 224)):
        out = torch.empty(B, th, tw, 3, device=dev)
        st = L.stream_ptr()
        call = lambda: L.check(L.lib.vtd_resize_with_pad(  # noqa: E731
            L.ptr(pixels), L.ptr(offs), L.ptr(sizes), B, th, tw, L.ptr(out), st))
        for _ in range(3):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        nbytes = B * (h * w * 3 + th * tw * 12)
        print(json.dumps({"op": "resize_with_pad",
                          "batch": B, "source": [h, w],
                          "target": [th, tw], "us": round(us, 1),
                          "images_per_s": round(B / us * 1e6),
                          "gbps": round(nbytes / us / 1e3, 1), "peak_gbps": 8000,
                          "frac": round(nbytes / us / 1e3 / 8000, 3)}))


if __name__ == "__main__":
    main()
