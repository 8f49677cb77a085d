"""GPU: vtd_resize_with_pad (the image transform of utils.py:438-447) against the float32
restatement oracle/preprocess.py, bit for bit, over ragged batches of image sizes
(landscape / portrait / exact fit / upscaled / 1-pixel rows), odd target planes (the
unaligned-store and tail paths), and end to end into the model."""
import numpy as np
import pytest
import torch

from oracle import preprocess as P
from oracle import vtd_numpy as ref

pytestmark = pytest.mark.gpu

SIZES = [(480, 640), (640, 480), (608, 608), (427, 640), (100, 37), (1, 5), (5, 1),
         (333, 333), (17, 1000), (2, 2)]


@pytest.fixture(scope="module")
def pre(cuda):
    from vision_transformer_detector_amd import preprocess as m
    return m


def _images(sizes, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in sizes]


@pytest.mark.parametrize("target", [(608, 608), (224, 224), (223, 97), (40, 36)])
def test_resize_with_pad_bit_exact(pre, cuda, target):
    # TF raises for an image whose resized side floors to 0 (17x1000 into 40x36)
    imgs = [i for i in _images(SIZES, seed=1)
            if min(P.geometry(i.shape[0], i.shape[1], *target)[:2]) > 0]
    got, sizes = pre.get_image_tensors(imgs, *target, device=cuda)
    got = got.cpu().numpy()
    assert sizes == [tuple(i.shape[:2]) for i in imgs]
    assert got.shape == (len(imgs), target[0], target[1], 3)
    for b, img in enumerate(imgs):
        exp = P.get_image_tensor(img, *target)
        np.testing.assert_array_equal(got[b], exp, err_msg=f"image {b} {img.shape}")


def test_resize_with_pad_single_and_torch_input(pre, cuda):
    img = torch.from_numpy(_images([(480, 640)], seed=2)[0])
    got, _ = pre.get_image_tensors([img], device=cuda)
    np.testing.assert_array_equal(got[0].cpu().numpy(), P.get_image_tensor(img.numpy()))


def test_preprocessed_batch_feeds_the_model(pre, cuda):
    """get_image_tensors -> Model.__call__ equals the oracle forward of the oracle's
    preprocessed images (float32 mode, north_star tolerance)."""
    import vision_transformer_detector_amd as vtd
    kw = dict(input_shape=(40, 36, 3), patch_size=8, embedding_dim=24, encoder_num_heads=3,
              encoder_key_dim=10, encoder_mlp_quantities=3, encoder_repeat_times=2,
              mlp_head_last_units=8, mlp_head_dense_layers_quantity=3)
    imgs = _images([(48, 64), (30, 20), (40, 36)], seed=3)
    x, _ = pre.get_image_tensors(imgs, 40, 36, device=cuda)
    xr = np.stack([P.get_image_tensor(i, 40, 36) for i in imgs]).astype(np.float64)
    w = ref.init_weights(seed=5, **kw)
    expect = ref.forward(w, xr, **kw)
    model = vtd.create_vision_transformer_detector(**kw, dtype="float32", device=cuda)
    model.set_weights(w)
    got = model(x, training=False).cpu().numpy()
    bound = 1e-3 * np.abs(expect) + 1e-3 * np.abs(expect).max()
    assert np.all(np.abs(got - expect) <= bound)
