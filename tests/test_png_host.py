"""PNG host side (vtd_png_info / vtd_png_workspace_bytes; no GPU): header walk over every
colour type / bit depth Pillow writes, Adam7, and the refusals libpng makes (bad signature,
critical-chunk CRC, truncation, palette without PLTE)."""
import ctypes
import io
import struct
import zlib

import numpy as np
import pytest
from PIL import Image


@pytest.fixture(scope="module")
def L():
    from vision_transformer_detector_amd import _lib
    return _lib


def _png(arr, mode, **kw):
    b = io.BytesIO()
    Image.fromarray(arr, mode=mode).save(b, format="PNG", **kw)
    return b.getvalue()


def _info(L, f):
    h, w, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = L.lib.vtd_png_info(f, len(f), ctypes.byref(h), ctypes.byref(w), ctypes.byref(c))
    return rc, (h.value, w.value, c.value)


def _ws(L, files):
    n = len(files)
    ptrs = (ctypes.c_char_p * n)(*files)
    lens = (ctypes.c_size_t * n)(*[len(f) for f in files])
    dims = np.zeros((n, 2), np.int32)
    b = ctypes.c_size_t()
    rc = L.lib.vtd_png_workspace_bytes(ptrs, lens, n, dims.ctypes.data, ctypes.byref(b))
    return rc, dims, b.value


def _chunk(t, body):
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body))


def test_png_header_walk(L):
    rng = np.random.default_rng(0)
    rgb = rng.integers(0, 256, (9, 13, 3), dtype=np.uint8)
    cases = [(_png(rgb, "RGB"), 3), (_png(rgb[..., 0], "L"), 1),
             (_png(np.dstack([rgb, rgb[..., :1]]), "RGBA"), 4),
             (_png(rgb, "RGB", optimize=True), 3),
             (_png((rgb[..., 0] > 127), "1"), 1)]
    pal = Image.fromarray(rgb).convert("P", palette=Image.ADAPTIVE, colors=16)
    b = io.BytesIO()
    pal.save(b, format="PNG")
    cases.append((b.getvalue(), 1))
    for f, comps in cases:
        rc, dims = _info(L, f)
        assert rc == 0 and dims == (9, 13, comps), (dims, L.lib.vtd_last_error())
    rc, dims, ws = _ws(L, [c[0] for c in cases])
    assert rc == 0 and ws > 0 and (dims == [9, 13]).all()


def test_png_refusals_name_the_reason(L):
    f = _png(np.zeros((4, 5, 3), np.uint8), "RGB")
    assert _info(L, b"GIF89a" + f[6:])[0] != 0 and b"not a PNG" in L.lib.vtd_last_error()
    i = f.index(b"IHDR")
    bad = f[:i + 5] + bytes([f[i + 5] ^ 1]) + f[i + 6:]          # IHDR body changed, CRC not
    assert _info(L, bad)[0] != 0 and b"CRC" in L.lib.vtd_last_error()
    assert _info(L, f[:-12])[0] != 0 and b"IEND" in L.lib.vtd_last_error()
    sig = b"\x89PNG\r\n\x1a\n"
    ihdr = _chunk(b"IHDR", struct.pack(">IIBBBBB", 4, 4, 8, 3, 0, 0, 0))
    nopal = sig + ihdr + _chunk(b"IDAT", zlib.compress(bytes(4 * 5))) + _chunk(b"IEND", b"")
    assert _info(L, nopal)[0] != 0 and b"PLTE" in L.lib.vtd_last_error()
    rc, _, _ = _ws(L, [f, nopal])
    assert rc != 0 and b"image 1" in L.lib.vtd_last_error()


def _bmp(arr, mode):
    b = io.BytesIO()
    Image.fromarray(arr).convert(mode).save(b, format="BMP")
    return b.getvalue()


def test_bmp_header_and_refusals(L):
    """BMP as TF 2.x's decode_image (DecodeImageV2, decode_image_op.cc): 8-, 24- and 32-bit files
    pass (channels = bpp / 8 in 1, 3, 4); other depths and RLE compression are refused by name;
    truncation is refused."""
    rng = np.random.default_rng(1)
    rgb = rng.integers(0, 256, (7, 11, 3), dtype=np.uint8)
    h, w, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    for mode in ("RGB", "RGBA", "L", "P"):
        f = _bmp(rgb, mode)
        assert L.lib.vtd_bmp_info(f, len(f), ctypes.byref(h), ctypes.byref(w), ctypes.byref(c)) == 0, \
            (mode, L.lib.vtd_last_error())
        assert (h.value, w.value, c.value) == (7, 11, 3)
    f = _bmp(rgb, "RGB")
    g = bytearray(f)
    g[28:30] = (16).to_bytes(2, "little")
    assert L.lib.vtd_bmp_info(bytes(g), len(g), ctypes.byref(h), ctypes.byref(w), ctypes.byref(c)) != 0
    assert b"16-bit" in L.lib.vtd_last_error()
    g = bytearray(_bmp(rgb, "L"))
    g[30:34] = (1).to_bytes(4, "little")                       # BI_RLE8
    assert L.lib.vtd_bmp_info(bytes(g), len(g), ctypes.byref(h), ctypes.byref(w), ctypes.byref(c)) != 0
    assert b"RLE" in L.lib.vtd_last_error()
    for comp in (4, 5, 6):                                     # BI_JPEG, BI_PNG, other
        g = bytearray(f)
        g[30:34] = comp.to_bytes(4, "little")
        assert L.lib.vtd_bmp_info(bytes(g), len(g), ctypes.byref(h), ctypes.byref(w),
                                  ctypes.byref(c)) != 0, comp
        assert b"compression" in L.lib.vtd_last_error()
    g = bytearray(f)
    g[30:34] = (3).to_bytes(4, "little")                       # BI_BITFIELDS decodes
    assert L.lib.vtd_bmp_info(bytes(g), len(g), ctypes.byref(h), ctypes.byref(w), ctypes.byref(c)) == 0
    assert L.lib.vtd_bmp_info(f[:60], 60, ctypes.byref(h), ctypes.byref(w), ctypes.byref(c)) != 0
    assert b"truncated" in L.lib.vtd_last_error()


def test_png_wide_rows_accepted(L):
    """Rows wider than the decoder's LDS row buffer (16 KiB of filtered bytes: RGB8 wider than
    5461 px, RGBA16 wider than 2048 px) are accepted by the header walk (they are unfiltered in
    place on the device); only the 2^28-pixel cap remains."""
    sig = b"\x89PNG\r\n\x1a\n"
    for w, depth, ctype in ((6000, 8, 2), (2100, 16, 6), (20000, 1, 0)):
        ihdr = _chunk(b"IHDR", struct.pack(">IIBBBBB", w, 2, depth, ctype, 0, 0, 0))
        f = sig + ihdr + _chunk(b"IDAT", zlib.compress(b"")) + _chunk(b"IEND", b"")
        rc, dims = _info(L, f)
        assert rc == 0 and dims[:2] == (2, w), L.lib.vtd_last_error()
    ihdr = _chunk(b"IHDR", struct.pack(">IIBBBBB", 1 << 15, (1 << 13) + 1, 8, 2, 0, 0, 0))
    f = sig + ihdr + _chunk(b"IEND", b"")
    assert _info(L, f)[0] != 0 and b"2^28" in L.lib.vtd_last_error()
    # a one-row RGBA16 image of 2^28 pixels: 2^31 bytes per row (the unfilter kernel's int
    # row index would wrap) -- refused, not decoded
    ihdr = _chunk(b"IHDR", struct.pack(">IIBBBBB", 1 << 28, 1, 16, 6, 0, 0, 0))
    f = sig + ihdr + _chunk(b"IEND", b"")
    assert _info(L, f)[0] != 0 and b"2^31" in L.lib.vtd_last_error()


def test_decode_images_routes_by_signature():
    """decode_images picks the decoder by file signature (no GPU needed for the routing)."""
    from vision_transformer_detector_amd.preprocess import _kind
    rgb = np.zeros((4, 4, 3), np.uint8)
    for fmt, kind in (("JPEG", "jpeg"), ("PNG", "png"), ("BMP", "bmp")):
        b = io.BytesIO()
        Image.fromarray(rgb).save(b, format=fmt)
        assert _kind(b.getvalue()) == kind
    b = io.BytesIO()
    Image.fromarray(rgb).save(b, format="GIF")
    with pytest.raises(ValueError, match="GIF"):
        _kind(b.getvalue())
