"""TEST INFRASTRUCTURE ONLY — float32 NumPy restatement of the reference's image transform.

`_get_image_tensor_coco` (`/root/reference/vision_transformer_utilities.py:418-449`) after
`tf.image.decode_image`:

    image = tf.image.resize_with_pad(image, MODEL_IMAGE_HEIGHT, MODEL_IMAGE_WIDTH)  # :438-440
    image = tf.clip_by_value(image, 0, 255)                                        # :443-444
    image /= 127.5; image -= 1                                                     # :446-447

The arithmetic lives upstream in TensorFlow 2.9.1 (not importable here), restated from its
published algorithm:
  * `image_ops_impl._resize_image_with_pad_common`: float32 geometry
    ratio = max(w / tw, h / th); resized = floor(side / ratio);
    pad_before = max(0, floor((target - side / ratio) / 2)); then `pad_to_bounding_box`
    (zeros) after the resize;
  * `resize_images_v2(method=BILINEAR, antialias=False)` -> `ResizeBilinear(
    half_pixel_centers=True)`, CPU kernel `resize_bilinear_op.cc`:
    scale = in / (float)out; in = (i + 0.5) * scale - 0.5; lower = max(floor(in), 0);
    upper = min(ceil(in), in_size - 1); lerp = in - floor(in);
    compute_lerp: top = tl + (tr - tl) * xl; bottom = bl + (br - bl) * xl;
    out = top + (bottom - top) * yl — every step a float32 operation (no FMA).

PARITY STATUS: parity unpinned against executed TF output (the reference holds no
preprocessed-image fixtures). Pinned instead by hand-derived known answers in
`tests/test_preprocess_kat.py` (geometry of COCO 640x480 -> 608, half-pixel 2x upsample
weights, identity at equal size, pad value -1).
"""
from __future__ import annotations

import numpy as np

F = np.float32


def geometry(h: int, w: int, th: int, tw: int):
    """(resized_h, resized_w, pad_top, pad_left) as TF computes them in float32."""
    fh, fw, fth, ftw = F(h), F(w), F(th), F(tw)
    ratio = max(fw / ftw, fh / fth)
    rhf, rwf = fh / ratio, fw / ratio
    rh, rw = int(np.floor(rhf)), int(np.floor(rwf))
    ph = max(0, int(np.floor((fth - rhf) / F(2))))
    pw = max(0, int(np.floor((ftw - rwf) / F(2))))
    return rh, rw, ph, pw


def _weights(out_size: int, in_size: int):
    scale = F(in_size) / F(out_size)
    i = np.arange(out_size).astype(F)
    x = (i + F(0.5)) * scale - F(0.5)
    xf = np.floor(x)
    lo = np.maximum(xf.astype(np.int64), 0)
    hi = np.minimum(np.ceil(x).astype(np.int64), in_size - 1)
    return lo, hi, (x - xf).astype(F)


def resize_bilinear(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """ResizeBilinear(half_pixel_centers=True) of an HWC image -> float32."""
    src = img.astype(F)
    h, w = src.shape[:2]
    y0, y1, yl = _weights(out_h, h)
    x0, x1, xl = _weights(out_w, w)
    xl = xl[None, :, None]
    yl = yl[:, None, None]
    tl, tr = src[y0][:, x0], src[y0][:, x1]
    bl, br = src[y1][:, x0], src[y1][:, x1]
    top = tl + (tr - tl) * xl
    bottom = bl + (br - bl) * xl
    return (top + (bottom - top) * yl).astype(F)


def resize_with_pad(img: np.ndarray, th: int, tw: int) -> np.ndarray:
    """tf.image.resize_with_pad (bilinear) of one HWC image -> float32 (th, tw, C)."""
    h, w = img.shape[:2]
    rh, rw, ph, pw = geometry(h, w, th, tw)
    if rh <= 0 or rw <= 0:
        raise ValueError(f"resize_with_pad: {h}x{w} resizes to {rh}x{rw} (TF raises)")
    out = np.zeros((th, tw, img.shape[2]), F)
    out[ph:ph + rh, pw:pw + rw] = resize_bilinear(img, rh, rw)
    return out


def get_image_tensor(img: np.ndarray, th: int = 608, tw: int = 608) -> np.ndarray:
    """vision_transformer_utilities.py:438-447 on a decoded uint8 HWC image."""
    x = resize_with_pad(img, th, tw)
    x = np.clip(x, F(0), F(255))
    x = x / F(127.5)
    return (x - F(1)).astype(F)
