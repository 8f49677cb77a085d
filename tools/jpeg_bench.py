"""Device JPEG decode throughput (vtd_jpeg_decode) on COCO-shaped JPEGs (640x480, 4:2:0,
quality 85, Pillow-encoded synthetic photo-like content), next to Pillow/libjpeg-turbo on the
host for the same files.  Reports per-kernel times (hipEvents on the decode stream) and the
end-to-end call time (host parsing + staging copy + kernels).
  python tools/jpeg_bench.py [--n 256] [--reps 5]"""
import argparse
import io
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_transformer_detector_amd.preprocess import decode_jpegs  # noqa: E402


def image(h, w, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    base = np.stack([127 + 100 * np.sin(x / (5 + 7 * c) + y / (9 + 3 * c) + c) for c in range(3)], -1)
    img = np.clip(base + rng.normal(0, 18, (h, w, 3)), 0, 255).astype(np.uint8)
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="JPEG", quality=85, subsampling=2)
    return b.getvalue()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    files = [image(480, 640, i % 16) for i in range(a.n)]
    dev = torch.device("cuda:0")
    for _ in range(3):     # both pinned staging slots sized for the full batch
        decode_jpegs(files, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_s = 0.0
    for _ in range(a.reps):
        h0 = time.perf_counter()
        decode_jpegs(files, device=dev)
        host_s += time.perf_counter() - h0
    torch.cuda.synchronize()
    gpu_s = (time.perf_counter() - t0) / a.reps
    host_s /= a.reps
    threads = min(16, os.cpu_count() or 1)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda f: np.asarray(Image.open(io.BytesIO(f)).convert("RGB")), files[:32]))
        t0 = time.perf_counter()
        list(ex.map(lambda f: np.asarray(Image.open(io.BytesIO(f)).convert("RGB")), files))
        cpu_s = time.perf_counter() - t0
    print(json.dumps({"images": a.n, "shape": [480, 640], "avg_jpeg_bytes": int(np.mean([len(f) for f in files])),
                      "device_decode_ms": round(gpu_s * 1e3, 2),
                      "device_img_per_s": round(a.n / gpu_s, 1),
                      "host_enqueue_ms": round(host_s * 1e3, 2),
                      "pillow_threads": threads, "pillow_ms": round(cpu_s * 1e3, 2),
                      "pillow_img_per_s": round(a.n / cpu_s, 1)}), flush=True)


if __name__ == "__main__":
    main()
