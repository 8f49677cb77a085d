"""Device JPEG decode (vtd_jpeg_decode; SURVEY §8f rank 4: `tf.image.decode_image(file,
channels=3)`, vision_transformer_utilities.py:431) against libjpeg-turbo -- the library TF's
decode_jpeg uses -- as bundled with Pillow (default ISLOW IDCT + fancy upsampling, the TF
defaults).  Bit-exact on every pixel, over synthetic photos-like images JPEG-encoded by Pillow
at several sizes (odd, 1x1, MCU-unaligned), qualities, 4:4:4 / 4:2:2 / 4:2:0 subsampling,
grayscale and restart intervals, decoded in one ragged batch.  Parity against TF itself is
unpinned (TF is not importable); both decode with libjpeg-turbo."""
import io

import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu


def _image(h, w, seed):
    """Smooth gradients + texture + a few hard edges (JPEG-typical content, all 8x8 blocks
    carrying AC energy)."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    base = np.stack([127 + 100 * np.sin(x / (5 + 7 * c) + y / (9 + 3 * c) + c) for c in range(3)], -1)
    noise = rng.normal(0, 18, (h, w, 3))
    img = base + noise
    img[(x // 13 + y // 11) % 5 == 0] = rng.uniform(0, 255, 3)
    return np.clip(img, 0, 255).astype(np.uint8)


def _encode(img, mode="RGB", **kw):
    b = io.BytesIO()
    Image.fromarray(img).convert(mode).save(b, format="JPEG", **kw)
    return b.getvalue()


def _pil_rgb(data):
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))


CASES = [  # (h, w, mode, encoder kwargs)
    (37, 53, "RGB", dict(quality=90, subsampling=0)),
    (37, 53, "RGB", dict(quality=75, subsampling=1)),
    (37, 53, "RGB", dict(quality=75, subsampling=2)),
    (480, 640, "RGB", dict(quality=85, subsampling=2)),     # the COCO shape
    (427, 640, "RGB", dict(quality=95, subsampling=2)),
    (1, 1, "RGB", dict(quality=80, subsampling=2)),
    (2, 3, "RGB", dict(quality=80, subsampling=2)),
    (17, 4, "RGB", dict(quality=60, subsampling=1)),
    (64, 64, "L", dict(quality=90)),
    (33, 70, "L", dict(quality=50)),
    (100, 120, "RGB", dict(quality=100, subsampling=0)),
    (31, 47, "RGB", dict(quality=10, subsampling=2)),
    (96, 80, "RGB", dict(quality=85, subsampling=2, optimize=True)),
    (1200, 1600, "RGB", dict(quality=100, subsampling=0)),  # ~MBs of scan: many LDS chunks
]


def _restart_case(h=72, w=88, rows=2):
    # restart markers every `rows` MCU rows (Pillow's restart_marker_rows, libjpeg
    # restart_in_rows)
    img = _image(h, w, 99)
    try:
        return _encode(img, quality=85, subsampling=2, restart_marker_rows=rows)
    except TypeError:
        return None


@pytest.mark.parametrize("chunk_bits", [None, "64", "256"])
def test_jpeg_decode_bit_exact_vs_libjpeg_turbo(cuda, monkeypatch, chunk_bits):
    """chunk_bits: the smallest entropy-decode chunk (default 1024 bits); 64 cuts even the
    small images into many chunks, so nearly every chunk starts at a guessed decoder state
    and must resynchronise."""
    from vision_transformer_detector_amd import _lib as L
    from vision_transformer_detector_amd.preprocess import decode_jpegs
    files = [_encode(_image(h, w, i), mode, **kw) for i, (h, w, mode, kw) in enumerate(CASES)]
    for rst in (_restart_case(), _restart_case(720, 960, 1)):   # the second spans chunks
        if rst is not None:
            files.append(rst)
    with L.knob(L.KNOB_JPEG_CHUNK_BITS, int(chunk_bits) if chunk_bits else -1):
        pixels, offsets, sizes = decode_jpegs(files, device=cuda)
        torch.cuda.synchronize()
    got = pixels.cpu().numpy()
    for i, f in enumerate(files):
        ref = _pil_rgb(f)
        h, w = sizes[i]
        assert (h, w) == ref.shape[:2]
        mine = got[offsets[i]:offsets[i] + h * w * 3].reshape(h, w, 3)
        bad = np.argwhere(mine != ref)
        assert bad.size == 0, (f"image {i} {CASES[i] if i < len(CASES) else 'restart'}: "
                               f"{len(bad)} differing values, first at {bad[0].tolist()}: "
                               f"{mine[tuple(bad[0])]} vs {ref[tuple(bad[0])]}")


PROG_CASES = [  # progressive (SOF2; libjpeg's simple progression script: DC / AC spectral
    # selection and successive approximation, every scan with its own Huffman tables)
    (37, 53, "RGB", dict(quality=75, subsampling=2)),
    (480, 640, "RGB", dict(quality=85, subsampling=2)),
    (100, 120, "RGB", dict(quality=95, subsampling=0)),
    (17, 4, "RGB", dict(quality=60, subsampling=1)),
    (33, 70, "L", dict(quality=50)),
    (1, 1, "RGB", dict(quality=80)),
    (64, 48, "RGB", dict(quality=100, subsampling=1)),
]


def test_jpeg_progressive_bit_exact_vs_libjpeg_turbo(cuda):
    """Progressive JPEGs decode to libjpeg-turbo's pixels exactly (its jdphuff.c first /
    refinement scans rebuild the same quantized coefficients; IDCT and colour are shared),
    batched together with baseline files; and with restart markers (segments decoded in
    parallel lanes)."""
    from vision_transformer_detector_amd.preprocess import decode_jpegs
    files = [_encode(_image(h, w, 50 + i), mode, progressive=True, **kw)
             for i, (h, w, mode, kw) in enumerate(PROG_CASES)]
    files.append(_encode(_image(40, 56, 7), quality=85, subsampling=2))       # baseline
    try:
        files.append(_encode(_image(72, 88, 8), quality=85, subsampling=2, progressive=True,
                             restart_marker_rows=1))
    except TypeError:
        pass
    assert all(b"\xff\xc2" in f for f in files[:len(PROG_CASES)])
    pixels, offsets, sizes = decode_jpegs(files, device=cuda)
    torch.cuda.synchronize()
    got = pixels.cpu().numpy()
    for i, f in enumerate(files):
        ref = _pil_rgb(f)
        h, w = sizes[i]
        assert (h, w) == ref.shape[:2]
        mine = got[offsets[i]:offsets[i] + h * w * 3].reshape(h, w, 3)
        bad = np.argwhere(mine != ref)
        assert bad.size == 0, (f"file {i}: {len(bad)} differing values, first at "
                               f"{bad[0].tolist()}: {mine[tuple(bad[0])]} vs {ref[tuple(bad[0])]}")


def test_jpeg_restart_markers_present():
    data = _restart_case()
    if data is None:
        pytest.skip("this Pillow cannot write restart markers")
    assert b"\xff\xdd" in data and any(bytes([0xFF, 0xD0 + k]) in data for k in range(8))


def test_jpeg_decode_then_resize_matches_host_pipeline(cuda):
    """decode on the device -> resize_with_pad -> [-1, 1]  ==  PIL decode -> the same
    resize_with_pad (bit-exact device kernel, tests/test_gpu_preprocess.py)."""
    from vision_transformer_detector_amd.preprocess import (get_image_tensors,
                                                            get_image_tensors_from_files)
    files = [_encode(_image(480, 640, 3), quality=85, subsampling=2),
             _encode(_image(333, 500, 4), quality=90, subsampling=0)]
    a, sa = get_image_tensors_from_files(files, device=cuda)
    b, sb = get_image_tensors([_pil_rgb(f) for f in files], device=cuda)
    torch.cuda.synchronize()
    assert sa == sb
    assert torch.equal(a, b)


def test_jpeg_unsupported_raises(cuda):
    from vision_transformer_detector_amd.preprocess import decode_jpegs
    rgb = _encode(_image(40, 40, 1), quality=80)
    i = rgb.index(b"\xff\xc0")
    two = rgb[:i + 9] + b"\x02" + rgb[i + 10:]          # Nf = 2: no such colour space
    with pytest.raises(ValueError, match="component"):
        decode_jpegs([two], device=cuda)
    with pytest.raises(ValueError):
        decode_jpegs([b"\x00\x01not a jpeg"], device=cuda)


def _cmyk_image(h, w, seed):
    """Four independent smooth + noisy channels (K not derived from C, M, Y)."""
    rgb = _image(h, w, seed)
    k = _image(h, w, seed + 1000)[..., 0]
    return np.concatenate([rgb, k[..., None]], -1)


def _cmyk_file(h, w, seed, **kw):
    b = io.BytesIO()
    Image.fromarray(_cmyk_image(h, w, seed), mode="CMYK").save(b, format="JPEG", **kw)
    return b.getvalue()


def _adobe_transform(data, t):
    """The same file with its Adobe APP14 transform byte set to t (2: YCCK -- libjpeg then
    converts the first three planes from YCbCr; the coefficients stay valid)."""
    i = data.index(b"Adobe") - 4
    assert data[i:i + 2] == b"\xff\xee"
    return data[:i + 4 + 11] + bytes([t]) + data[i + 4 + 12:]


def _without_adobe(data):
    i = data.index(b"Adobe") - 4
    ln = int.from_bytes(data[i + 2:i + 4], "big")
    return data[:i] + data[i + 2 + ln:]


def _tf_cmyk_rgb(data):
    """Expected `decode_image(f, channels=3)` of a 4-component JPEG: libjpeg-turbo's CMYK
    output (Pillow's CMYK pixels are its inversion, rawmode "CMYK;I"), then TF's
    jpeg_mem.cc CMYK -> RGB (integer division; Adobe marker: R = K C / 255, otherwise
    R = (255 - K)(255 - C) / 255)."""
    im = Image.open(io.BytesIO(data))
    assert im.mode == "CMYK"
    raw = 255 - np.asarray(im).astype(np.int64)
    c, m, y, k = (raw[..., i] for i in range(4))
    if b"Adobe" in data:
        out = np.stack([k * c // 255, k * m // 255, k * y // 255], -1)
    else:
        out = np.stack([(255 - k) * (255 - c) // 255, (255 - k) * (255 - m) // 255,
                        (255 - k) * (255 - y) // 255], -1)
    return out.astype(np.uint8)


def test_jpeg_cmyk_and_ycck_vs_libjpeg_turbo(cuda):
    """4-component JPEGs: the CMYK planes are libjpeg-turbo's bit for bit
    (Pillow's decode: baseline, progressive, 4:2:0-sampled first plane, an Adobe transform 2
    file that libjpeg decodes as YCCK through jdcolor.c ycck_cmyk_convert, a file without the
    Adobe marker), and the RGB is TF's CMYK -> RGB of those planes (restated from TF's
    jpeg_mem.cc; TF itself is not importable, so that last integer step is unpinned)."""
    from vision_transformer_detector_amd.preprocess import decode_jpegs
    base = _cmyk_file(37, 53, 1, quality=90)
    files = [base, _cmyk_file(48, 64, 2, quality=75, subsampling=2),
             _cmyk_file(61, 45, 3, quality=85, progressive=True),
             _cmyk_file(1, 1, 4, quality=80),
             _adobe_transform(base, 2), _without_adobe(base),
             _encode(_image(20, 24, 5), quality=85, subsampling=2)]     # + an RGB file
    assert b"Adobe" in base and b"\xff\xc2" in files[2]
    pixels, offsets, sizes = decode_jpegs(files, device=cuda)
    torch.cuda.synchronize()
    got = pixels.cpu().numpy()
    for i, f in enumerate(files):
        ref = _tf_cmyk_rgb(f) if i < len(files) - 1 else _pil_rgb(f)
        h, w = sizes[i]
        assert (h, w) == ref.shape[:2]
        mine = got[offsets[i]:offsets[i] + h * w * 3].reshape(h, w, 3)
        bad = np.argwhere(mine != ref)
        assert bad.size == 0, (f"file {i}: {len(bad)} differing values, first at "
                               f"{bad[0].tolist()}: {mine[tuple(bad[0])]} vs {ref[tuple(bad[0])]}")
