"""CPU: the image-transform restatement (oracle/preprocess.py, utils.py:438-447) against
hand-derived known answers of TF's resize_with_pad / ResizeBilinear(half_pixel_centers)
algorithm, and the host shim's argument checks (no GPU needed)."""
import numpy as np
import pytest

from oracle import preprocess as P

F = np.float32


def test_geometry_coco_landscape_and_portrait():
    # 640x480 (w x h) -> 608: ratio = fl(640/608); fl(640/ratio) and fl(480/ratio) as
    # float32 division gives; pad = floor((608 - side/ratio) / 2)
    ratio = F(640) / F(608)
    rw, rh = F(640) / ratio, F(480) / ratio
    exp = (int(np.floor(rh)), int(np.floor(rw)),
           int(np.floor((F(608) - rh) / F(2))), int(np.floor((F(608) - rw) / F(2))))
    # in real arithmetic 480 * 608 / 640 = 456; in float32 ratio = 1.0526316 (rounded up)
    # and 480 / ratio = 455.99997, so TF's floor gives 455 (pad 76, bottom pad 77)
    assert ratio == F(1.0526316) and rh == F(455.99997) and rw == F(608)
    assert exp[0] == 455 and exp[2] == 76
    assert exp[1] == 608 and exp[3] == 0
    assert P.geometry(480, 640, 608, 608) == exp
    assert P.geometry(640, 480, 608, 608) == (exp[1], exp[0], exp[3], exp[2])


def test_geometry_exact_fit_and_small_images():
    assert P.geometry(608, 608, 608, 608) == (608, 608, 0, 0)
    assert P.geometry(304, 304, 608, 608) == (608, 608, 0, 0)      # upscaled to fill
    assert P.geometry(2, 4, 4, 4) == (2, 4, 1, 0)                  # pad top 1, bottom 1


def test_half_pixel_upsample_weights():
    # in 2 -> out 4: scale 0.5, in = -0.25, 0.25, 0.75, 1.25 -> (lo, hi, lerp) =
    # (0,0,.75) (0,1,.25) (0,1,.75) (1,1,.25): [a, a + (b-a)/4, a + 3(b-a)/4, b]
    img = np.array([[[0, 0, 0], [100, 200, 40]]], np.uint8)        # 1 x 2 x 3
    out = P.resize_bilinear(img, 1, 4)
    np.testing.assert_array_equal(out[0, :, 0], F([0, 25, 75, 100]))
    np.testing.assert_array_equal(out[0, :, 1], F([0, 50, 150, 200]))
    np.testing.assert_array_equal(out[0, :, 2], F([0, 10, 30, 40]))


def test_half_pixel_downsample_averages_pairs():
    # in 4 -> out 2: scale 2, in = 0.5, 2.5 -> mean of pixels (0,1) and (2,3)
    img = np.array([[[10] * 3, [20] * 3, [30] * 3, [50] * 3]], np.uint8)
    out = P.resize_bilinear(img, 1, 2)
    np.testing.assert_array_equal(out[0, :, 0], F([15, 40]))


def test_identity_size_and_pad_value():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (2, 4, 3), dtype=np.uint8)
    out = P.get_image_tensor(img, 4, 4)
    np.testing.assert_array_equal(out[0], np.full((4, 3), -1, F))  # pad rows: 0/127.5 - 1
    np.testing.assert_array_equal(out[3], np.full((4, 3), -1, F))
    np.testing.assert_array_equal(out[1:3], img.astype(F) / F(127.5) - F(1))
    assert out.min() >= -1 and out.max() <= 1


def test_extreme_aspect_raises_like_tf():
    with pytest.raises(ValueError):
        P.resize_with_pad(np.zeros((1, 2000, 3), np.uint8), 608, 608)


def test_host_shim_rejects_bad_images_before_any_launch():
    L = pytest.importorskip("vision_transformer_detector_amd")
    from vision_transformer_detector_amd import preprocess as pre
    with pytest.raises(ValueError):
        pre.get_image_tensors([np.zeros((1, 2000, 3), np.uint8)], device="cuda")
    with pytest.raises(ValueError):
        pre.get_image_tensors([np.zeros((8, 8, 4), np.uint8)], device="cuda")
    with pytest.raises(ValueError):
        pre.get_image_tensors([np.zeros((8, 8, 3), np.float32)], device="cuda")
    with pytest.raises(ValueError):
        pre.get_image_tensors([], device="cuda")
    with pytest.raises(ValueError):
        pre.get_image_tensors([np.zeros((8, 8, 3), np.uint8)], device="cpu")
    assert L is not None
