"""CPU tests of the JPEG decoder's host side (vtd_jpeg_info / vtd_jpeg_workspace_bytes: the
marker walk that feeds the device decoder; no GPU calls): image sizes agree with Pillow's
header parse over the supported flavours, unsupported flavours come back as
VTD_ERR_UNSUPPORTED naming the reason, and malformed input fails cleanly."""
import ctypes
import io

import numpy as np
import pytest
from PIL import Image


@pytest.fixture(scope="module")
def L():
    from vision_transformer_detector_amd import _lib
    return _lib


def _jpeg(h, w, mode="RGB", **kw):
    rng = np.random.default_rng(h * 1000 + w)
    img = Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).convert(mode)
    b = io.BytesIO()
    img.save(b, format="JPEG", **kw)
    return b.getvalue()


def _plan(L, files):
    n = len(files)
    ptrs = (ctypes.c_char_p * n)(*files)
    lens = (ctypes.c_size_t * n)(*[len(f) for f in files])
    dims = np.zeros((n, 2), np.int32)
    ws = ctypes.c_size_t()
    rc = L.lib.vtd_jpeg_workspace_bytes(ptrs, lens, n, dims.ctypes.data, ctypes.byref(ws))
    return rc, dims, ws.value


def _info(L, f):
    h, w, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = L.lib.vtd_jpeg_info(f, len(f), ctypes.byref(h), ctypes.byref(w), ctypes.byref(c))
    return rc, (h.value, w.value, c.value)


SUPPORTED = [
    (480, 640, "RGB", dict(quality=85, subsampling=2)),
    (37, 53, "RGB", dict(quality=90, subsampling=0)),
    (17, 4, "RGB", dict(quality=60, subsampling=1)),
    (1, 1, "RGB", dict(quality=80)),
    (33, 70, "L", dict(quality=50)),
    (96, 80, "RGB", dict(quality=85, optimize=True)),
    (72, 88, "RGB", dict(quality=85, restart_marker_rows=2)),
]


@pytest.mark.parametrize("h,w,mode,kw", SUPPORTED)
def test_info_matches_pillow_header(L, h, w, mode, kw):
    try:
        f = _jpeg(h, w, mode, **kw)
    except TypeError:
        pytest.skip("this Pillow lacks an encoder option")
    rc, (hh, ww, c) = _info(L, f)
    assert rc == 0, L.lib.vtd_last_error()
    im = Image.open(io.BytesIO(f))
    assert (hh, ww) == (im.height, im.width)
    assert c == (1 if mode == "L" else 3)


def test_workspace_plan_dims_and_growth(L):
    files = [_jpeg(h, w, m, **kw) for h, w, m, kw in SUPPORTED if "restart_marker_rows" not in kw]
    rc, dims, ws = _plan(L, files)
    assert rc == 0
    assert [tuple(d) for d in dims] == [(h, w) for h, w, m, kw in SUPPORTED
                                        if "restart_marker_rows" not in kw]
    # the workspace holds at least the coefficients (2 B each) of every image's blocks
    assert ws >= sum(((h + 15) // 16) * ((w + 15) // 16) * 6 * 128 for h, w in dims) // 2
    rc2, _, ws2 = _plan(L, files + files)
    assert rc2 == 0 and ws2 > ws


def test_unsupported_flavours_name_the_reason(L):
    # two components: the RGB file's frame header with Nf = 2
    rgb = _jpeg(16, 16, quality=80)
    i = rgb.index(b"\xff\xc0")
    assert rgb[i + 9] == 3
    two = rgb[:i + 9] + b"\x02" + rgb[i + 10:]
    rc, _ = _info(L, two)
    assert rc != 0 and b"component" in L.lib.vtd_last_error()
    rc, _, _ = _plan(L, [_jpeg(8, 8), two])
    assert rc != 0 and b"image 1" in L.lib.vtd_last_error()
    # arithmetic coding (SOF9): the same file with its SOF0 marker byte changed
    base = _jpeg(16, 16, quality=80)
    i = base.index(b"\xff\xc0")
    arith = base[:i + 1] + b"\xc9" + base[i + 2:]
    rc, _ = _info(L, arith)
    assert rc != 0 and b"arithmetic" in L.lib.vtd_last_error()


@pytest.mark.parametrize("mode,kw", [("RGB", dict(quality=80, subsampling=2)),
                                     ("RGB", dict(quality=95, subsampling=0)), ("L", {})])
def test_progressive_header_walk(L, mode, kw):
    """Progressive JPEGs (SOF2, several scans with their own Huffman tables) pass the header
    walk: the dimensions are Pillow's, and the workspace plan grows with the scans."""
    f = _jpeg(45, 61, mode, progressive=True, **kw)
    assert f.count(b"\xff\xda") > 1 and b"\xff\xc2" in f
    rc, dims = _info(L, f)
    assert rc == 0 and dims[:2] == (45, 61), dims
    rc, pd, ws = _plan(L, [f, _jpeg(45, 61, mode, **kw)])
    assert rc == 0 and ws > 0


def test_progressive_dqt_redefined_after_its_scan_is_refused(L):
    """libjpeg-turbo latches a component's quantization table at its first scan; a DQT that
    redefines a latched table with other values between scans is refused by name,
    one that repeats the same values is accepted."""
    f = _jpeg(40, 48, "RGB", progressive=True, quality=75)
    i = f.index(b"\xff\xdb")
    ln = int.from_bytes(f[i + 2:i + 4], "big")
    first = f[i + 4:i + 4 + 65]                 # Pq/Tq byte + 64 8-bit entries of table 0
    assert first[0] >> 4 == 0
    second_sos = f.index(b"\xff\xda", f.index(b"\xff\xda") + 2)
    same = f[:second_sos] + _segment(0xDB, first) + f[second_sos:]
    other = f[:second_sos] + _segment(0xDB, bytes([first[0]]) + bytes([1] * 64)) + f[second_sos:]
    assert ln >= 67
    rc, dims = _info(L, same)
    assert rc == 0 and dims[:2] == (40, 48)
    rc, _ = _info(L, other)
    assert rc != 0 and b"latched" in L.lib.vtd_last_error()


def _with_sof_sampling(f, comp0):
    """A copy of baseline JPEG f with component 0's sampling byte of the SOF0 replaced."""
    i = f.index(b"\xff\xc0")
    b = bytearray(f)
    b[i + 2 + 2 + 6 + 1] = comp0         # marker, length, P/Y/X/Nf, then C1 id, H1V1
    return bytes(b)


def test_440_subsampling_is_refused(L):
    """4:4:0 (luma 1 x 2, chroma 1 x 1) would need libjpeg-turbo's h1v2 upsampling, which the
    colour pass does not implement: the header walk refuses it by name."""
    f = _with_sof_sampling(_jpeg(32, 32, quality=80, subsampling=0), 0x12)
    rc, _ = _info(L, f)
    assert rc != 0 and b"4:4:0" in L.lib.vtd_last_error()


def _segment(marker, payload):
    return b"\xff" + bytes([marker]) + (len(payload) + 2).to_bytes(2, "big") + payload


@pytest.mark.parametrize("marker", [0xDD, 0xDA])
def test_short_dri_sos_at_the_end_of_the_file(L, marker):
    """A DRI / SOS segment whose declared length leaves no payload, placed so that the
    segment ends the buffer: refused before any payload byte is read (ASan host check too)."""
    f = _jpeg(16, 16, quality=80)
    head = f[:f.index(b"\xff\xda")]    # everything before the scan
    rc, _ = _info(L, head + _segment(marker, b""))
    assert rc != 0 and b"truncated" in L.lib.vtd_last_error()


@pytest.mark.parametrize("data", [b"", b"\x00\x01not a jpeg", b"\xff\xd8", b"\xff\xd8\xff\xd9",
                                  b"\xff\xd8\xff\xdb\x00\x43\x00"])
def test_malformed_input_fails_cleanly(L, data):
    if not data:
        rc = L.lib.vtd_jpeg_info(b"\0", 0, None, None, None)
    else:
        rc, _ = _info(L, data)
    assert rc != 0 and L.lib.vtd_last_error()


def test_truncations_of_a_valid_file_never_crash(L):
    f = _jpeg(24, 24, quality=75)
    for cut in range(1, len(f), 7):
        rc, _ = _info(L, f[:cut])        # a header cut short fails; a cut scan still parses
        assert rc in (0,) or L.lib.vtd_last_error()


def test_decode_requires_a_hip_device():
    from vision_transformer_detector_amd.preprocess import decode_jpegs
    with pytest.raises(ValueError, match="HIP device"):
        decode_jpegs([_jpeg(8, 8)], device="cpu")


def test_cmyk_header_walk(L):
    """4-component (CMYK; Adobe APP14) JPEGs pass the header walk with comps = 4."""
    cmyk = _jpeg(16, 24, "CMYK", quality=80)
    assert b"Adobe" in cmyk
    rc, dims = _info(L, cmyk)
    assert rc == 0 and dims == (16, 24, 4), dims
    rc, pd, ws = _plan(L, [_jpeg(8, 8), cmyk])
    assert rc == 0 and ws > 0
