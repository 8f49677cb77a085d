"""CPU tests of the oracle itself (no GPU): the hand-derived known-answer tests of
SURVEY.md Appendix A, the reference's layer-shape fixture (notebook plot_model diagram),
agreement of the two independent restatements, and reproducibility of the golden files.
"""
import hashlib
import json
import math
import os

import numpy as np
import pytest
import torch

from oracle import vtd_numpy as V
from oracle import vtd_torch_cpu as T

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_patch_order_and_same_padding_kat():
    """App. A.1: H = W = 5, p = 2 -> 3x3 patches, pad 1 -> 0 before / 1 after; patch
    (0,0) = pixels (0..1, 0..1) flattened (kh, kw, c)."""
    img = np.arange(5 * 5 * 3, dtype=np.float64).reshape(1, 5, 5, 3)
    p = V.extract_patches_same(img, 2)
    assert p.shape == (1, 9, 12)
    np.testing.assert_array_equal(p[0, 0], [0, 1, 2, 3, 4, 5, 15, 16, 17, 18, 19, 20])
    # patch (2, 2): only pixel (4, 4) is inside the image
    np.testing.assert_array_equal(p[0, 8], [72, 73, 74] + [0] * 9)
    # 608 / 17: 36 patches, pad total 4 -> 2 rows / cols of zeros at the top / left
    img = np.ones((1, 608, 608, 3))
    p = V.extract_patches_same(img, 17)
    assert p.shape == (1, 1296, 867)
    first = p[0, 0].reshape(17, 17, 3)
    assert (first[:2] == 0).all() and (first[:, :2] == 0).all() and (first[2:, 2:] == 1).all()
    last = p[0, -1].reshape(17, 17, 3)
    assert (last[-2:] == 0).all() and (last[:-2, :-2] == 1).all()


def test_reshape_not_transpose_kat():
    """App. A.2: Dense(17) output t[b,n,k] = n*17+k (N = 196) -> head input
    u[b,i,j] = i*196+j, which is not t transposed."""
    n = 196
    t = np.arange(n * 17, dtype=np.float64).reshape(1, n, 17)
    u = t.reshape(1, 17, n)
    np.testing.assert_array_equal(u[0], np.arange(17 * n).reshape(17, n))
    assert not np.array_equal(u[0], t[0].T)


def test_layernorm_epsilon_kat():
    """App. A.3: a row with variance 1e-3 is scaled by 1/sqrt(2e-3)."""
    x = np.array([[(-1) ** i * math.sqrt(1e-3) for i in range(64)]])
    y = V.layer_norm(x, np.ones(64), np.zeros(64))
    assert abs(y[0, 0] - math.sqrt(1e-3) / math.sqrt(2e-3)) < 1e-12


def test_mha_uniform_softmax_kat():
    """App. A.4: Wq = 0, bq = 0 -> uniform softmax -> O = mean_k(V); I != D."""
    rng = np.random.default_rng(0)
    D, H, dk, N = 6, 2, 5, 7
    w = {"m/query/kernel": np.zeros((D, H, dk)), "m/query/bias": np.zeros((H, dk)),
         "m/key/kernel": rng.normal(size=(D, H, dk)), "m/key/bias": rng.normal(size=(H, dk)),
         "m/value/kernel": rng.normal(size=(D, H, dk)), "m/value/bias": rng.normal(size=(H, dk)),
         "m/attention_output/kernel": np.eye(H * dk, D).reshape(H, dk, D),
         "m/attention_output/bias": np.zeros(D)}
    x = rng.normal(size=(1, N, D))
    out = V.multi_head_attention(x, w, "m", dk)
    v = np.einsum("abc,cde->abde", x, w["m/value/kernel"]) + w["m/value/bias"]
    expect = np.einsum("abcd,cde->abe", np.broadcast_to(v.mean(1, keepdims=True), v.shape),
                       w["m/attention_output/kernel"])
    np.testing.assert_allclose(out, expect, atol=1e-12)


def test_position_embedding_width_one_kat():
    """App. A.5: the position embedding is (N, 1) and raises every channel equally."""
    kw = dict(input_shape=(16, 16, 3), patch_size=8, embedding_dim=4, encoder_num_heads=1,
              encoder_key_dim=4, encoder_mlp_quantities=1, encoder_repeat_times=1,
              mlp_head_last_units=2, mlp_head_dense_layers_quantity=1)
    assert V.weight_shapes(**kw)["position_encoding/position_embedding/embeddings"] == (4, 1)


def test_activation_kats():
    """App. A.6 (tfa mish / GELU(approximate=True) published values)."""
    assert V.mish(0.0) == 0.0
    assert abs(V.mish(1.0) - 0.8650983882673103) < 1e-15
    assert abs(V.mish(-1.0) - (-0.30340146137410895)) < 1e-15
    assert abs(V.mish(50.0) - 50.0) < 1e-12
    assert abs(V.gelu_tanh(1.0) - 0.8411919906082768) < 1e-15


def test_decode_kat():
    """App. A.7: a zero logit decodes to [0.5, 39.5, 304, 304, 304, 304]."""
    np.testing.assert_allclose(V.transform_predictions(np.zeros((1, 1, 6)))[0, 0],
                               [0.5, 39.5, 304, 304, 304, 304])


def test_layer_shapes_match_notebook_plot_model_fixture():
    """App. A.8: every layer the reference's plot_model diagram shows (default config)
    has the oracle's output shape."""
    fixture = json.load(open(os.path.join(GOLD, "plot_model_shapes.json")))
    shapes = V.layer_output_shapes()
    checked = 0
    dense_widths = {s[-1] for n, s in shapes.items() if n.startswith(("MLP_", "dense_"))}
    for name, shp in fixture.items():
        if name.startswith("_"):
            continue
        if name.startswith(("layer_normalization", "multi_head")):
            # LN / MHA keep the embedding shape (MHA projects back to D, vtd.py:364-369)
            assert tuple(shp) == tuple(shapes["embedded_patches"]), name
        elif name.startswith("mish_activation"):
            assert shp[-1] in dense_widths, name     # elementwise on a Dense output
        else:
            assert tuple(shapes[name]) == tuple(shp), name
        checked += 1
    assert checked >= 60
    # activation after EVERY MLP Dense incl. the last: 8 per block x 8 blocks + 7 head
    # activations -> the head's mish layers are numbered 64..70
    assert "mish_activation_63" in fixture and "mish_activation_70" in fixture


def test_param_counts():
    """C1 131.48 M params, C2 (ViT-B/16 preset) 180.36 M."""
    n1 = sum(int(np.prod(s)) for s in V.weight_shapes().values())
    assert abs(n1 / 1e6 - 131.48) < 0.01
    c2 = dict(input_shape=(224, 224, 3), patch_size=16, embedding_dim=768,
              encoder_num_heads=12, encoder_key_dim=64, encoder_repeat_times=12,
              encoder_mlp_quantities=3, use_mish=False)
    n2 = sum(int(np.prod(s)) for s in V.weight_shapes(**c2).values())
    assert abs(n2 / 1e6 - 180.36) < 0.01


@pytest.mark.parametrize("kw", [
    dict(input_shape=(40, 36, 3), patch_size=8, embedding_dim=24, encoder_num_heads=3,
         encoder_key_dim=10, encoder_mlp_quantities=3, encoder_repeat_times=2,
         mlp_head_last_units=8, mlp_head_dense_layers_quantity=3),
    dict(input_shape=(33, 50, 3), patch_size=7, embedding_dim=20, encoder_num_heads=2,
         encoder_key_dim=12, encoder_mlp_quantities=2, encoder_repeat_times=1,
         mlp_head_last_units=4, mlp_head_dense_layers_quantity=5,
         mlp_head_dense_mish_block_repeats=2, use_mish=False)])
def test_two_restatements_agree(kw):
    w = V.init_weights(seed=5, **kw)
    x = V.synthetic_images(2, V.resolve_kwargs(**kw)["input_shape"], seed=6)
    a = V.forward(w, x, **kw)
    b = T.TorchCpuDetector(w, dtype=torch.float64, **kw)(x).numpy()
    c = T.TorchCpuDetector(w, **kw)(x).numpy()
    assert np.abs(a - b).max() < 1e-12
    assert np.abs(a - c).max() < 1e-5 * max(1.0, np.abs(a).max())


@pytest.mark.parametrize("name", ["tiny_mish", "tiny_gelu", "tiny_seq400"])
def test_golden_files_reproduce(name):
    z = np.load(os.path.join(GOLD, f"{name}.npz"))
    kw = json.loads(str(z["kwargs"]))
    kw["input_shape"] = tuple(kw["input_shape"])
    w = {k[2:]: z[k] for k in z.files if k.startswith("w:")}
    y = V.forward(w, z["images"], **kw)
    np.testing.assert_allclose(y, z["logits"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(V.transform_predictions(y), z["dets"], atol=1e-9)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


def test_seeded_inputs_are_platform_stable():
    """The GPU box regenerates C1/C2 weights and images from seeds: their hashes must
    match the ones recorded when the expected logits were computed."""
    spec = json.load(open(os.path.join(GOLD, "seeded_forward.json")))
    for name, s in spec.items():
        kw = dict(s["kwargs"])
        if "input_shape" in kw:
            kw["input_shape"] = tuple(kw["input_shape"])
        shape = V.resolve_kwargs(**kw)["input_shape"]
        x = V.synthetic_images(s["batch"], shape, seed=s["image_seed"], letterbox=s["letterbox"])
        assert _sha(x) == s["images_sha256"], name
        w = V.init_weights(seed=s["weight_seed"], perturb=s["perturb"], **kw)
        assert _sha(np.concatenate([v.ravel() for v in w.values()])) == s["weights_sha256"]


def test_detection_mask_kat():
    """vtd.py:1367-1384 on decoded predictions: tf.round is half-to-even; confidence
    (0.5 - |c - round(c)|)/0.5 must exceed 0.5, i.e. |c - round(c)| < 0.25."""
    d = np.zeros((1, 6, 6))
    d[0, :, 0] = [0.9, 0.9, 0.9, 0.9, 0.5, 0.51]
    d[0, :, 1] = [2.0, 2.5, 3.5, 2.24, 7.0, 7.2]
    cat, valid = V.detection_mask(d)
    np.testing.assert_array_equal(cat[0], [2, 2, 4, 2, 7, 7])
    np.testing.assert_array_equal(valid[0], [True, False, False, True, False, True])


def test_mx8_format_kats():
    """MX-fp8 restatement (oracle/mx8.py) against the OCP MX / e4m3 definitions: byte
    decoding, round-to-nearest-even ties, the e4m3 range, and the block-scale rule."""
    from oracle import mx8 as MX
    dec = MX.decode_e4m3(np.array([0x7e, 0x38, 0x08, 0x01, 0x00, 0x80, 0xb8, 0x7f], np.uint8))
    np.testing.assert_array_equal(dec[:7], [448.0, 1.0, 2.0 ** -6, 2.0 ** -9, 0.0, -0.0, -1.0])
    assert np.isnan(dec[7])
    # ties to even: 1.0625 is halfway between 1.0 (mantissa 0) and 1.125 (1) -> 1.0;
    # 1.1875 halfway between 1.125 (1) and 1.25 (2) -> 1.25; subnormal 1.5 * 2^-9 -> 2^-8
    np.testing.assert_array_equal(MX.round_e4m3([1.0625, 1.1875, 1.5 * 2.0 ** -9, 448.0, -3.3]),
                                  [1.0, 1.25, 2.0 ** -8, 448.0, -3.25])
    # least E with amax <= 448 * 2^E
    np.testing.assert_array_equal(MX.block_exponent([448.0, 449.0, 56.0, 56.5, 0.0, 1e30]),
                                  [0, 1, -3, -2, -126, 91])
    x = np.random.default_rng(0).normal(size=(6, 100)) * np.exp2(np.arange(6) * 7 - 20)[:, None]
    vals, E = MX.quantize(x, 128)
    deq = (vals.reshape(6, 4, 32) * np.exp2(E)[..., None]).reshape(6, 128)[:, :100]
    assert np.all(np.abs(deq - x) <= np.abs(x) / 16 + np.exp2(E.max(axis=1) - 10)[:, None])
    assert np.all(np.abs(vals) <= 448)
