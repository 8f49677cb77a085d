"""Input pipeline image transform on the device.

Mirrors `_get_image_tensor_coco` (`vision_transformer_utilities.py:418-449`) for a batch:
`tf.image.decode_image(file, channels=3)` for JPEG files (`decode_jpegs`: libjpeg-turbo's
baseline decode path on the device, vtd_jpeg_decode), then `tf.image.resize_with_pad` to the
model size (bilinear, half-pixel centers), `clip_by_value(0, 255)`, `/ 127.5 - 1`, written as
one NHWC fp32 batch that `Model.__call__` takes directly (one `vtd_resize_with_pad` launch).
File reading stays with the caller (`get_image_tensors_from_files` reads the bytes).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L

MODEL_IMAGE_HEIGHT, MODEL_IMAGE_WIDTH = 608, 608   # vtd.py:22 Constants.MODEL_IMAGE_SIZE


def _resized_side_positive(h: int, w: int, th: int, tw: int) -> bool:
    # TF's float32 geometry (image_ops_impl._resize_image_with_pad_common): a side that
    # floors to 0 makes ResizeBilinear raise; reject it here the same way.
    f = np.float32
    ratio = max(f(w) / f(tw), f(h) / f(th))
    return np.floor(f(h) / ratio) >= 1 and np.floor(f(w) / ratio) >= 1


def get_image_tensors(images, target_height: int = MODEL_IMAGE_HEIGHT,
                      target_width: int = MODEL_IMAGE_WIDTH, device="cuda", stream=None):
    """Decoded uint8 HWC images (numpy arrays or torch tensors, any sizes, 3 channels) ->
    (images (B, target_height, target_width, 3) fp32 in [-1, 1] on `device`,
     original sizes [(height, width), ...]) — the batched form of the reference's
    `image_tensor, image_original_size = _get_image_tensor_coco(path)`."""
    if len(images) == 0:
        raise ValueError("get_image_tensors: empty image list")
    if target_height <= 0 or target_width <= 0:
        raise ValueError("get_image_tensors: target size must be positive")
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError(f"get_image_tensors runs on a HIP device, got {dev}")
    sizes, flats = [], []
    for img in images:
        t = torch.as_tensor(img)
        if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] != 3:
            raise ValueError(f"expected a uint8 (H, W, 3) image, got {tuple(t.shape)} {t.dtype}")
        h, w = int(t.shape[0]), int(t.shape[1])
        if h <= 0 or w <= 0 or not _resized_side_positive(h, w, target_height, target_width):
            raise ValueError(f"image {h}x{w} cannot be resized with pad to "
                             f"{target_height}x{target_width} (a resized side would be 0)")
        sizes.append((h, w))
        flats.append(t.reshape(-1))
    lengths = [int(f.numel()) for f in flats]
    offsets = np.zeros(len(flats), np.int64)
    offsets[1:] = np.cumsum(lengths[:-1])
    packed = torch.cat([f.cpu() for f in flats]).pin_memory()
    pixels = packed.to(dev, non_blocking=True)
    offs = torch.from_numpy(offsets).to(dev)
    szs = torch.tensor(sizes, dtype=torch.int32).to(dev)
    out = torch.empty(len(flats), target_height, target_width, 3, dtype=torch.float32, device=dev)
    _on_stream(stream, dev, pixels, offs, szs, out)
    with torch.cuda.device(dev):
        L.check(L.lib.vtd_resize_with_pad(L.ptr(pixels), L.ptr(offs), L.ptr(szs), len(flats),
                                          target_height, target_width, L.ptr(out),
                                          L.stream_ptr(stream)), "resize_with_pad")
    return out, sizes


def decode_jpegs(files, device="cuda", stream=None):
    """JPEG file bytes (a list of `bytes`) -> (packed RGB uint8 pixels on `device`, per-image
    byte offsets (int64, host), [(height, width), ...]): `tf.image.decode_image(f, channels=3)`
    (vision_transformer_utilities.py:431) for baseline / extended sequential and progressive
    Huffman JPEGs (1, 3 or 4 -- CMYK / YCCK -- components), decoded on the device by
    vtd_jpeg_decode.  Unsupported JPEG flavours
    (arithmetic-coded, lossless, 12-bit, 4:4:0) raise ValueError naming the
    reason; nothing falls back to a host decoder."""
    import ctypes
    if len(files) == 0:
        raise ValueError("decode_jpegs: empty file list")
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError(f"decode_jpegs runs on a HIP device, got {dev}")
    files = [bytes(f) for f in files]      # c_char_p points into each bytes object: no copy
    n = len(files)
    ptrs = (ctypes.c_char_p * n)(*files)
    lens = (ctypes.c_size_t * n)(*[len(f) for f in files])
    dims = np.zeros((n, 2), np.int32)
    ws_bytes = ctypes.c_size_t()
    rc = L.lib.vtd_jpeg_workspace_bytes(ptrs, lens, n, dims.ctypes.data, ctypes.byref(ws_bytes))
    if rc != 0:
        raise ValueError(L.lib.vtd_last_error().decode())
    sizes = [(int(h), int(w)) for h, w in dims]
    offsets = np.zeros(n, np.int64)
    offsets[1:] = np.cumsum(dims[:, 0].astype(np.int64) * dims[:, 1] * 3)[:-1]
    total = int(offsets[-1]) + sizes[-1][0] * sizes[-1][1] * 3
    pixels = torch.empty(total, dtype=torch.uint8, device=dev)
    ws = torch.empty(int(ws_bytes.value), dtype=torch.uint8, device=dev)
    offs = (ctypes.c_int64 * n)(*offsets.tolist())
    _on_stream(stream, dev, pixels, ws)
    with torch.cuda.device(dev):
        L.check(L.lib.vtd_jpeg_decode(ptrs, lens, n, L.ptr(pixels), offs, L.ptr(ws),
                                      ws_bytes.value, L.stream_ptr(stream)), "jpeg_decode")
    return pixels, offsets, sizes


def _decode_with(kind, files, pixels, offsets, dev, stream):
    """Run the `kind` ("jpeg" / "png") device decoder on `files` into `pixels` at `offsets`."""
    import ctypes
    n = len(files)
    ptrs = (ctypes.c_char_p * n)(*files)
    lens = (ctypes.c_size_t * n)(*[len(f) for f in files])
    dims = np.zeros((n, 2), np.int32)
    ws_bytes = ctypes.c_size_t()
    rc = getattr(L.lib, f"vtd_{kind}_workspace_bytes")(ptrs, lens, n, dims.ctypes.data,
                                                      ctypes.byref(ws_bytes))
    if rc != 0:
        raise ValueError(L.lib.vtd_last_error().decode())
    ws = torch.empty(max(1, int(ws_bytes.value)), dtype=torch.uint8, device=dev)
    offs = (ctypes.c_int64 * n)(*[int(o) for o in offsets])
    _on_stream(stream, dev, pixels, ws)
    with torch.cuda.device(dev):
        L.check(getattr(L.lib, f"vtd_{kind}_decode")(ptrs, lens, n, L.ptr(pixels), offs, L.ptr(ws),
                                                    ws_bytes.value, L.stream_ptr(stream)),
                f"{kind}_decode")


def _kind(f: bytes) -> str:
    if f[:3] == b"\xff\xd8\xff":
        return "jpeg"
    if f[:8] == b"\x89PNG\r\n\x1a\n":
        return "png"
    if f[:2] == b"BM":
        return "bmp"
    raise ValueError("decode_images: not a JPEG, PNG or BMP file (GIF is not supported)")


def decode_images(files, device="cuda", stream=None):
    """`tf.image.decode_image(f, channels=3)` (vision_transformer_utilities.py:431) for a batch
    of JPEG, PNG and BMP files (by their signature), decoded on the device (vtd_jpeg_decode /
    vtd_png_decode / vtd_bmp_decode) into one packed RGB uint8 buffer -> (pixels, per-image byte offsets,
    [(height, width), ...]) as `decode_jpegs`."""
    import ctypes
    if len(files) == 0:
        raise ValueError("decode_images: empty file list")
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError(f"decode_images runs on a HIP device, got {dev}")
    files = [bytes(f) for f in files]
    kinds = [_kind(f) for f in files]
    sizes = []
    for f, k in zip(files, kinds):
        h, w, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = getattr(L.lib, f"vtd_{k}_info")(f, len(f), ctypes.byref(h), ctypes.byref(w),
                                            ctypes.byref(c))
        if rc != 0:
            raise ValueError(L.lib.vtd_last_error().decode())
        sizes.append((h.value, w.value))
    n = len(files)
    offsets = np.zeros(n, np.int64)
    offsets[1:] = np.cumsum([h * w * 3 for h, w in sizes])[:-1]
    total = int(offsets[-1]) + sizes[-1][0] * sizes[-1][1] * 3
    pixels = torch.empty(total, dtype=torch.uint8, device=dev)
    for kind in ("jpeg", "png", "bmp"):
        idx = [i for i in range(n) if kinds[i] == kind]
        if idx:
            _decode_with(kind, [files[i] for i in idx], pixels, [offsets[i] for i in idx], dev,
                         stream)
    return pixels, offsets, sizes


def _on_stream(stream, dev, *tensors):
    """Before launching on a caller-given `stream` that is not the current one: order it after
    the current stream's work (the allocations and host-to-device copies of the inputs were
    made there), and tell the caching allocator that the tensors are used on `stream`, so a
    tensor freed at return is not handed out again before `stream`'s kernels have run."""
    if stream is None:
        return
    cur = torch.cuda.current_stream(dev)
    if stream != cur:
        stream.wait_stream(cur)
    for t in tensors:
        t.record_stream(stream)


def get_image_tensors_from_files(paths_or_bytes, target_height: int = MODEL_IMAGE_HEIGHT,
                                 target_width: int = MODEL_IMAGE_WIDTH, device="cuda",
                                 stream=None):
    """`_get_image_tensor_coco` for a batch of JPEG / PNG files (paths or bytes): read, decode
    on the device (decode_images), resize_with_pad / clip / normalise on the device ->
    (images (B, target_height, target_width, 3) fp32 in [-1, 1], original sizes)."""
    files = []
    for p in paths_or_bytes:
        if isinstance(p, (bytes, bytearray, memoryview)):
            files.append(bytes(p))
        else:
            with open(p, "rb") as f:
                files.append(f.read())
    pixels, offsets, sizes = decode_images(files, device=device, stream=stream)
    dev = torch.device(device)
    for h, w in sizes:
        if not _resized_side_positive(h, w, target_height, target_width):
            raise ValueError(f"image {h}x{w} cannot be resized with pad to "
                             f"{target_height}x{target_width} (a resized side would be 0)")
    offs = torch.from_numpy(offsets).to(dev)
    szs = torch.tensor(sizes, dtype=torch.int32).to(dev)
    out = torch.empty(len(files), target_height, target_width, 3, dtype=torch.float32, device=dev)
    _on_stream(stream, dev, pixels, offs, szs, out)
    with torch.cuda.device(dev):
        L.check(L.lib.vtd_resize_with_pad(L.ptr(pixels), L.ptr(offs), L.ptr(szs), len(files),
                                          target_height, target_width, L.ptr(out),
                                          L.stream_ptr(stream)), "resize_with_pad")
    return out, sizes
