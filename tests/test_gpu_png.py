"""Device PNG decode (vtd_png_decode; `tf.image.decode_image(file, channels=3)` on PNG files,
vision_transformer_utilities.py:431) against the PNG specification's pixel arithmetic.  Files
come from a small encoder in this test that controls every field -- colour type, bit depth
1-16, palette, Adam7, and the filter type of every row (None / Sub / Up / Average / Paeth,
cycled, so each appears after each) -- with the expected RGB8 computed as TF's libpng path
does (gray expanded x 255 / (2^d - 1), 16-bit -> high byte, alpha dropped, palette looked up),
and from Pillow's encoder, checked against Pillow's decoder.  TF itself is not importable."""
import io
import struct
import zlib

import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu

A7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)


def _filter_rows(raw_rows, bpp, first_type):
    out, prev = [], bytes(len(raw_rows[0]))
    for r, row in enumerate(raw_rows):
        ft = (first_type + r) % 5
        f = bytearray(len(row))
        for i, x in enumerate(row):
            a = row[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            pred = [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]
            f[i] = (x - pred) & 0xFF
        out.append(bytes([ft]) + bytes(f))
        prev = row
    return b"".join(out)


def _pack_rows(samples, depth):
    """samples (h, w*ch) ints -> list of packed row bytes (big-endian for 16-bit)."""
    rows = []
    for r in samples:
        if depth == 16:
            rows.append(b"".join(struct.pack(">H", int(v)) for v in r))
        elif depth == 8:
            rows.append(bytes(int(v) for v in r))
        else:
            bits = "".join(format(int(v), f"0{depth}b") for v in r)
            bits += "0" * (-len(bits) % 8)
            rows.append(bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8)))
    return rows


def _chunk(t, body):
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body))


def encode_png(samples, ctype, depth, palette=None, interlace=False, first_type=0):
    """samples: (h, w, ch) ints (palette: indices)."""
    h, w, ch = samples.shape
    bpp = max(1, ch * depth // 8)
    if interlace:
        data = b""
        for p, (x0, y0, dx, dy) in enumerate(A7):
            sub = samples[y0::dy, x0::dx]
            if sub.size == 0:
                continue
            data += _filter_rows(_pack_rows(sub.reshape(sub.shape[0], -1), depth), bpp,
                                 first_type + p)
    else:
        data = _filter_rows(_pack_rows(samples.reshape(h, -1), depth), bpp, first_type)
    f = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0,
                                                           1 if interlace else 0))
    if palette is not None:
        f += _chunk(b"PLTE", bytes(palette.reshape(-1).tolist()))
    comp = zlib.compress(data, 6)
    f += _chunk(b"IDAT", comp[:len(comp) // 2]) + _chunk(b"IDAT", comp[len(comp) // 2:])
    return f + _chunk(b"IEND", b"")


def expected_rgb(samples, ctype, depth, palette=None):
    s = samples.astype(np.int64)
    if depth == 16:
        s = s >> 8
    if ctype == 3:
        return palette[samples[..., 0]].astype(np.uint8)
    if ctype in (0, 4):
        g = s[..., 0]
        if depth < 8:
            g = g * 255 // ((1 << depth) - 1)
        return np.stack([g, g, g], -1).astype(np.uint8)
    return s[..., :3].astype(np.uint8)


CASES = [  # (h, w, ctype, depth, interlace)
    (17, 23, 2, 8, False), (17, 23, 2, 16, False), (9, 31, 6, 8, False), (9, 31, 6, 16, False),
    (12, 19, 0, 1, False), (12, 19, 0, 2, False), (12, 19, 0, 4, False), (12, 19, 0, 8, False),
    (12, 19, 0, 16, False), (11, 7, 4, 8, False), (11, 7, 4, 16, False),
    (13, 29, 3, 1, False), (13, 29, 3, 2, False), (13, 29, 3, 4, False), (13, 29, 3, 8, False),
    (1, 1, 2, 8, False), (33, 41, 2, 8, True), (21, 18, 3, 4, True), (19, 26, 0, 1, True),
    (5, 3, 6, 16, True), (2, 2, 0, 8, True), (64, 300, 2, 8, False)]


def _case(i, h, w, ctype, depth, interlace):
    rng = np.random.default_rng(100 + i)
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    hi = (1 << depth) if ctype != 3 else min(1 << depth, 200)
    y, x = np.mgrid[0:h, 0:w]
    smooth = ((x * 7 + y * 3) % hi)[..., None] * np.ones(ch, np.int64)   # filters predict well
    noise = rng.integers(0, hi, (h, w, ch))
    samples = np.where(rng.random((h, w, 1)) < 0.5, smooth, noise)
    pal = rng.integers(0, 256, (hi, 3)) if ctype == 3 else None
    return encode_png(samples, ctype, depth, pal, interlace, first_type=i % 5), \
        expected_rgb(samples, ctype, depth, pal)


def test_png_decode_bit_exact(cuda):
    """Every colour type x bit depth, Adam7, every filter type, in one ragged batch."""
    from vision_transformer_detector_amd.preprocess import decode_images
    files, refs = [], []
    for i, c in enumerate(CASES):
        f, ref = _case(i, *c)
        files.append(f)
        refs.append(ref)
    pixels, offsets, sizes = decode_images(files, device=cuda)
    torch.cuda.synchronize()
    got = pixels.cpu().numpy()
    for i, ref in enumerate(refs):
        h, w = sizes[i]
        assert (h, w) == ref.shape[:2]
        mine = got[offsets[i]:offsets[i] + h * w * 3].reshape(h, w, 3)
        bad = np.argwhere(mine != ref)
        assert bad.size == 0, (f"case {i} {CASES[i]}: {len(bad)} differing, first {bad[0].tolist()}: "
                               f"{mine[tuple(bad[0])]} vs {ref[tuple(bad[0])]}")


def test_png_pillow_files_and_mixed_batch(cuda):
    """Files from Pillow's encoder (its own filter choices) decode to Pillow's pixels; a batch
    mixing JPEG and PNG files goes through decode_images in one packed buffer."""
    from vision_transformer_detector_amd.preprocess import decode_images
    rng = np.random.default_rng(7)
    y, x = np.mgrid[0:45, 0:61]
    rgb = np.clip(np.stack([x * 4, y * 5, (x + y) * 2], -1) + rng.integers(-20, 20, (45, 61, 3)),
                  0, 255).astype(np.uint8)
    ims = [Image.fromarray(rgb), Image.fromarray(rgb[..., 0]),
           Image.fromarray(np.dstack([rgb, rgb[..., 1:2]])),
           Image.fromarray(rgb).convert("P", palette=Image.ADAPTIVE, colors=37),
           Image.fromarray(rgb[..., 0] > 100)]
    files = []
    for k, im in enumerate(ims):
        b = io.BytesIO()
        im.save(b, format="PNG", optimize=bool(k & 1))
        files.append(b.getvalue())
    b = io.BytesIO()
    ims[0].save(b, format="JPEG", quality=90)
    files.insert(2, b.getvalue())
    pixels, offsets, sizes = decode_images(files, device=cuda)
    torch.cuda.synchronize()
    got = pixels.cpu().numpy()
    for i, f in enumerate(files):
        ref = np.asarray(Image.open(io.BytesIO(f)).convert("RGB"))
        h, w = sizes[i]
        mine = got[offsets[i]:offsets[i] + h * w * 3].reshape(h, w, 3)
        assert np.array_equal(mine, ref), i


def test_png_wide_rows_bit_exact(cuda):
    """Rows wider than the LDS row buffer (16 KiB of filtered bytes) are unfiltered in place in
    the workspace: RGB8 6000 px (18,000 B rows), RGBA16 2100 px interlaced (Adam7's last passes
    are the wide ones), gray 1-bit 150,000 px, next to a narrow file in the same batch; every
    filter type on every row."""
    from vision_transformer_detector_amd.preprocess import decode_images
    files, refs = [], []
    for i, (h, w, ctype, depth, il) in enumerate([(6, 6000, 2, 8, False), (9, 2100, 6, 16, True),
                                                  (5, 150000, 0, 1, False), (17, 23, 2, 8, False)]):
        f, ref = _case(40 + i, h, w, ctype, depth, il)
        files.append(f)
        refs.append(ref)
    pixels, offsets, sizes = decode_images(files, device=cuda)
    torch.cuda.synchronize()
    got = pixels.cpu().numpy()
    for i, ref in enumerate(refs):
        h, w = sizes[i]
        mine = got[offsets[i]:offsets[i] + h * w * 3].reshape(h, w, 3)
        assert np.array_equal(mine, ref), i


def test_png_bad_filter_type_raises(cuda):
    """A row filter byte above 4 is an error (libpng: bad adaptive filter value), not a row
    decoded as None."""
    from vision_transformer_detector_amd.preprocess import decode_images
    samples = np.arange(4 * 5 * 3).reshape(4, 5, 3) % 256
    raw = bytearray(zlib.decompress(zlib.compress(
        _filter_rows(_pack_rows(samples.reshape(4, -1), 8), 3, 0))))
    raw[2 * (1 + 15)] = 7                                       # row 2's filter byte
    f = (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", 5, 4, 8, 2, 0, 0, 0)) +
         _chunk(b"IDAT", zlib.compress(bytes(raw))) + _chunk(b"IEND", b""))
    with pytest.raises((ValueError, RuntimeError), match="filter"):
        decode_images([f], device=cuda)


def test_png_corrupt_stream_raises(cuda):
    from vision_transformer_detector_amd.preprocess import decode_images
    f, _ = _case(0, *CASES[0])
    i = f.index(b"IDAT")
    ln = int.from_bytes(f[i - 4:i], "big")
    body = bytes([f[i + 4] ^ 0xFF]) + f[i + 5:i + 4 + ln]       # zlib header broken
    bad = f[:i - 4] + _chunk(b"IDAT", body) + f[i + 8 + ln:]
    with pytest.raises((ValueError, RuntimeError), match="zlib|truncated"):
        decode_images([bad], device=cuda)


def test_bmp_decode_bottom_up_and_top_down(cuda):
    """24-bit BMP (TF decode_image): bottom-up rows from Pillow's encoder and the same file made
    top-down (negative height, rows reversed), widths with 4-byte row padding."""
    from vision_transformer_detector_amd.preprocess import decode_images
    files, refs = [], []
    for k, (h, w) in enumerate([(7, 11), (16, 16), (1, 1), (33, 50)]):
        rgb = np.random.default_rng(k).integers(0, 256, (h, w, 3), dtype=np.uint8)
        b = io.BytesIO()
        Image.fromarray(rgb).save(b, format="BMP")
        f = b.getvalue()
        files.append(f)
        refs.append(rgb)
        off = int.from_bytes(f[10:14], "little")
        row = (24 * w + 31) // 32 * 4
        rows = [f[off + r * row:off + (r + 1) * row] for r in range(h)]
        td = bytearray(f[:off] + b"".join(rows[::-1]))
        td[22:26] = (-h).to_bytes(4, "little", signed=True)
        files.append(bytes(td))
        refs.append(rgb)
    pixels, offsets, sizes = decode_images(files, device=cuda)
    torch.cuda.synchronize()
    got = pixels.cpu().numpy()
    for i, ref in enumerate(refs):
        h, w = sizes[i]
        assert np.array_equal(got[offsets[i]:offsets[i] + h * w * 3].reshape(h, w, 3), ref), i


def test_bmp_decode_8_and_32_bit(cuda):
    """8- and 32-bit BMP as TF 2.x decode_image (decode_image_op.cc DecodeBmpV2) converts them to
    channels = 3: 32-bit BGRA -> RGB (alpha dropped); 8-bit -> the stored byte replicated into
    R, G, B -- the palette is not applied (a Pillow "P" file with a non-identity palette
    decodes to its indices), which is what TF's decoder does.  Parity against TF itself is
    unpinned (not importable here)."""
    from vision_transformer_detector_amd.preprocess import decode_images
    rng = np.random.default_rng(5)
    files, refs = [], []
    for k, (h, w) in enumerate([(7, 13), (5, 3), (20, 31)]):
        rgba = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
        b = io.BytesIO()
        Image.fromarray(rgba, mode="RGBA").save(b, format="BMP")
        files.append(b.getvalue())
        refs.append(rgba[..., :3])
        gray = rng.integers(0, 256, (h, w), dtype=np.uint8)
        b = io.BytesIO()
        Image.fromarray(gray, mode="L").save(b, format="BMP")
        files.append(b.getvalue())
        refs.append(np.repeat(gray[..., None], 3, -1))
        idx = rng.integers(0, 16, (h, w), dtype=np.uint8)
        im = Image.fromarray(idx, mode="P")
        im.putpalette(list(rng.integers(0, 256, 16 * 3).astype(int)))
        b = io.BytesIO()
        im.save(b, format="BMP")
        files.append(b.getvalue())
        refs.append(np.repeat(idx[..., None], 3, -1))
    pixels, offsets, sizes = decode_images(files, device=cuda)
    torch.cuda.synchronize()
    got = pixels.cpu().numpy()
    for i, ref in enumerate(refs):
        h, w = sizes[i]
        assert np.array_equal(got[offsets[i]:offsets[i] + h * w * 3].reshape(h, w, 3), ref), i
