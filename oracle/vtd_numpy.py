"""TEST INFRASTRUCTURE ONLY — float64 NumPy restatement of the reference forward pass.

Follows `/root/reference/vision_transformer_detector.py` (cited as `vtd.py:N`) and the
upstream TF 2.9.1 / Keras 2.9 / tensorflow-addons semantics catalogued in SURVEY.md
Appendix B.  Parity against executed reference output is UNPINNED (TF not importable,
no reference vectors exist); see `oracle/__init__.py` for what pins it instead.

Weights are a dict keyed by Keras weight names, e.g.
`linear_projection/kernel`, `multi_head_attention_3/query/kernel`, `MLP_2_1/bias`.
"""
from __future__ import annotations

import math

import numpy as np

MAX_DETECT_OBJECTS_QUANTITY = 17          # vtd.py:28
CLASSES = 80                              # vtd.py:20
MODEL_IMAGE_SIZE = (608, 608)             # vtd.py:22
LAYER_NORM_EPSILON = 1e-3                 # keras.layers.LayerNormalization default [upstream]

DEFAULT_KWARGS = dict(                    # vtd.py:498-506
    input_shape=None, patch_size=17, embedding_dim=28, encoder_num_heads=8,
    encoder_key_dim=40, dropout=None, encoder_mlp_quantities=8,
    encoder_repeat_times=8, mlp_head_last_units=136,
    mlp_head_dense_layers_quantity=7, mlp_head_dense_mish_block_repeats=1,
    use_mish=True, max_weight=10, clip_weight=True, training=None)


def resolve_kwargs(**kw):
    out = dict(DEFAULT_KWARGS)
    for k, v in kw.items():
        if k not in out:
            raise TypeError(f"unexpected keyword argument {k!r}")
        out[k] = v
    if out["input_shape"] is None:                       # vtd.py:550-551
        out["input_shape"] = (*MODEL_IMAGE_SIZE, 3)
    return out


def token_grid(h, w, p):
    """SAME padding: out = ceil(in / stride) (tf.image.extract_patches) [upstream]."""
    return -(-h // p), -(-w // p)


# ----------------------------------------------------------------------------- shapes
def weight_shapes(**kw):
    """Keras weight name -> shape, in layer-creation order."""
    k = resolve_kwargs(**kw)
    h, w, c = k["input_shape"]
    p = k["patch_size"]
    gh, gw = token_grid(h, w, p)
    n_tok, n_in = gh * gw, p * p * c
    d, nh, dk = k["embedding_dim"], k["encoder_num_heads"], k["encoder_key_dim"]
    shapes = {}
    shapes["position_encoding/position_embedding/embeddings"] = (n_tok, 1)   # vtd.py:291-293
    shapes["linear_projection/kernel"] = (n_in, d)                          # vtd.py:297-301
    shapes["linear_projection/bias"] = (d,)
    q = k["encoder_mlp_quantities"]
    units = [d * 2 ** e for e in range(q - 1, -1, -1)]                     # vtd.py:385-386
    for i in range(1, k["encoder_repeat_times"] + 1):
        ln1 = "layer_normalization" + ("" if i == 1 else f"_{2 * (i - 1)}")
        ln2 = f"layer_normalization_{2 * (i - 1) + 1}"
        mha = "multi_head_attention" + ("" if i == 1 else f"_{i - 1}")
        shapes[f"{ln1}/gamma"] = (d,)
        shapes[f"{ln1}/beta"] = (d,)
        for nm in ("query", "key", "value"):
            shapes[f"{mha}/{nm}/kernel"] = (d, nh, dk)
            shapes[f"{mha}/{nm}/bias"] = (nh, dk)
        shapes[f"{mha}/attention_output/kernel"] = (nh, dk, d)
        shapes[f"{mha}/attention_output/bias"] = (d,)
        shapes[f"{ln2}/gamma"] = (d,)
        shapes[f"{ln2}/beta"] = (d,)
        fan_in = d
        for j in range(q):
            shapes[f"MLP_{i}_{j + 1}/kernel"] = (fan_in, units[j])
            shapes[f"MLP_{i}_{j + 1}/bias"] = (units[j],)
            fan_in = units[j]
    shapes["dense/kernel"] = (d, MAX_DETECT_OBJECTS_QUANTITY)                 # vtd.py:454-458
    shapes["dense/bias"] = (MAX_DETECT_OBJECTS_QUANTITY,)
    head_units = [k["mlp_head_last_units"] * 2 ** e
                  for e in range(k["mlp_head_dense_layers_quantity"])]      # vtd.py:465-466
    fan_in, idx = n_tok, 1
    for u in reversed(head_units):                                          # vtd.py:468-476
        for _ in range(k["mlp_head_dense_mish_block_repeats"]):
            shapes[f"dense_{idx}/kernel"] = (fan_in, u)
            shapes[f"dense_{idx}/bias"] = (u,)
            fan_in, idx = u, idx + 1
    shapes["MLP_Head_no_Sigmoid/kernel"] = (fan_in, 6)                       # vtd.py:489-493
    shapes["MLP_Head_no_Sigmoid/bias"] = (6,)
    return shapes


def layer_output_shapes(**kw):
    """Per-layer output shapes with the batch dim as None, as drawn by keras plot_model."""
    k = resolve_kwargs(**kw)
    h, w, c = k["input_shape"]
    p = k["patch_size"]
    gh, gw = token_grid(h, w, p)
    n_tok, n_in, d = gh * gw, p * p * c, k["embedding_dim"]
    out = {"images": (None, h, w, c),
           "split_image_into_patches": (None, gh, gw, n_in),
           "flatten_patches": (None, n_tok, n_in),
           "linear_projection": (None, n_tok, d),
           "position_encoding": (1, n_tok, 1),
           "embedded_patches": (None, n_tok, d)}
    q = k["encoder_mlp_quantities"]
    units = [d * 2 ** e for e in range(q - 1, -1, -1)]
    for i in range(1, k["encoder_repeat_times"] + 1):
        out[f"residual_connection_{i}_1"] = (None, n_tok, d)
        for j in range(q):
            out[f"MLP_{i}_{j + 1}"] = (None, n_tok, units[j])
        out["encoded_images" if i == k["encoder_repeat_times"]
            else f"residual_connection_{i}_2"] = (None, n_tok, d)
    out["dense"] = (None, n_tok, MAX_DETECT_OBJECTS_QUANTITY)
    out["reshape"] = (None, MAX_DETECT_OBJECTS_QUANTITY, n_tok)
    names = [nm[:-len("/kernel")] for nm in weight_shapes(**kw) if nm.startswith("dense_")
             and nm.endswith("/kernel")]
    for nm in names:
        out[nm] = (None, MAX_DETECT_OBJECTS_QUANTITY, weight_shapes(**kw)[nm + "/kernel"][1])
    out["MLP_Head_no_Sigmoid"] = (None, MAX_DETECT_OBJECTS_QUANTITY, 6)
    return out


# ------------------------------------------------------------------------------- ops
def extract_patches_same(images, p):
    """`tf.image.extract_patches(sizes=strides=[1,p,p,1], rates=1, padding='SAME')`
    (vtd.py:195-197) + Reshape((-1, p*p*C)) (vtd.py:279-280).

    SAME: pad_total = max((out-1)*s + k - in, 0), pad_before = pad_total // 2, zeros;
    each patch flattened in (row, col, depth) order [upstream]."""
    b, h, w, c = images.shape
    gh, gw = token_grid(h, w, p)
    pad_h = max((gh - 1) * p + p - h, 0)
    pad_w = max((gw - 1) * p + p - w, 0)
    top, left = pad_h // 2, pad_w // 2
    padded = np.zeros((b, gh * p, gw * p, c), dtype=images.dtype)
    padded[:, top:top + h, left:left + w, :] = images
    x = padded.reshape(b, gh, p, gw, p, c).transpose(0, 1, 3, 2, 4, 5)
    return x.reshape(b, gh * gw, p * p * c)


def softplus(x):
    return np.logaddexp(0.0, x)


def mish(x):
    """tfa.activations.mish: x * tanh(softplus(x)) (vtd.py:128-129) [upstream]."""
    return x * np.tanh(softplus(x))


def gelu_tanh(x):
    """tfa.layers.GELU() default approximate=True (vtd.py:402, 483) [upstream]."""
    return 0.5 * x * (1.0 + np.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x ** 3)))


def layer_norm(x, gamma, beta, eps=LAYER_NORM_EPSILON):
    """keras LayerNormalization(axis=-1): biased variance, eps 1e-3 (vtd.py:353-357)."""
    mu = x.mean(axis=-1, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * gamma + beta


def softmax(x, axis=-1):
    e = np.exp(x - x.max(axis=axis, keepdims=True))
    return e / e.sum(axis=axis, keepdims=True)


def multi_head_attention(x, wts, prefix, key_dim):
    """keras MultiHeadAttention(query=x, value=x) (vtd.py:364-369): key = value,
    EinsumDense projections with bias, Q scaled by 1/sqrt(key_dim), softmax over keys,
    output EinsumDense back to D [upstream]."""
    g = lambda n: wts[f"{prefix}/{n}"]
    q = np.einsum("abc,cde->abde", x, g("query/kernel")) + g("query/bias")
    k = np.einsum("abc,cde->abde", x, g("key/kernel")) + g("key/bias")
    v = np.einsum("abc,cde->abde", x, g("value/kernel")) + g("value/bias")
    q = q * (1.0 / math.sqrt(float(key_dim)))
    scores = np.einsum("aecd,abcd->acbe", k, q)           # (B, H, Nq, Nk)
    probs = softmax(scores, axis=-1)
    o = np.einsum("acbe,aecd->abcd", probs, v)            # (B, Nq, H, dk)
    return np.einsum("abcd,cde->abe", o, g("attention_output/kernel")) + \
        g("attention_output/bias")


def dense(x, wts, name):
    return x @ wts[f"{name}/kernel"] + wts[f"{name}/bias"]


# --------------------------------------------------------------------------- forward
def forward(weights, images, **kw):
    """Logits (B, 17, 6) of `model(images, training=False)` (vtd.py:498-583)."""
    k = resolve_kwargs(**kw)
    if k["dropout"] not in (None, 0, 0.0):
        raise ValueError("forward oracle covers dropout=None / 0 only")
    wts = {n: np.asarray(v, dtype=np.float64) for n, v in weights.items()}
    x = np.asarray(images, dtype=np.float64)
    act = mish if k["use_mish"] else gelu_tanh
    p = k["patch_size"]
    patches = extract_patches_same(x, p)
    n_tok = patches.shape[1]
    pos = wts["position_encoding/position_embedding/embeddings"][np.arange(n_tok)]  # (N,1)
    e = dense(patches, wts, "linear_projection") + pos[None, :, :]       # vtd.py:305-307
    d = e.shape[-1]
    q = k["encoder_mlp_quantities"]
    for i in range(1, k["encoder_repeat_times"] + 1):                     # vtd.py:350-412
        ln1 = "layer_normalization" + ("" if i == 1 else f"_{2 * (i - 1)}")
        ln2 = f"layer_normalization_{2 * (i - 1) + 1}"
        mha = "multi_head_attention" + ("" if i == 1 else f"_{i - 1}")
        h = layer_norm(e, wts[f"{ln1}/gamma"], wts[f"{ln1}/beta"])
        e = e + multi_head_attention(h, wts, mha, k["encoder_key_dim"])
        h = layer_norm(e, wts[f"{ln2}/gamma"], wts[f"{ln2}/beta"])
        for j in range(q):
            h = act(dense(h, wts, f"MLP_{i}_{j + 1}"))
        e = e + h
    t = dense(e, wts, "dense")                                            # (B, N, 17)
    b = t.shape[0]
    u = t.reshape(b, MAX_DETECT_OBJECTS_QUANTITY, n_tok)                  # vtd.py:461-463
    idx = 1
    while f"dense_{idx}/kernel" in wts:                                   # vtd.py:468-486
        u = act(dense(u, wts, f"dense_{idx}"))
        idx += 1
    return dense(u, wts, "MLP_Head_no_Sigmoid")                           # vtd.py:489-493


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def transform_predictions(inputs):
    """vtd.py:586-647: sigmoid, clip boxes to [0,1], class*(CLASSES-1),
    cx,w * MODEL_IMAGE_SIZE[1], cy,h * MODEL_IMAGE_SIZE[0] (the constant 608)."""
    s = sigmoid(np.asarray(inputs, dtype=np.float64))
    s[..., -4:] = np.clip(s[..., -4:], 0.0, 1.0)
    out = s.copy()
    out[..., 1] = s[..., 1] * (CLASSES - 1)
    out[..., 2] = s[..., 2] * MODEL_IMAGE_SIZE[1]
    out[..., 3] = s[..., 3] * MODEL_IMAGE_SIZE[0]
    out[..., 4] = s[..., 4] * MODEL_IMAGE_SIZE[0]
    out[..., 5] = s[..., 5] * MODEL_IMAGE_SIZE[1]
    return out


# --------------------------------------------------------------------------- weights
def _fans(shape):
    """keras initializers._compute_fans [upstream]."""
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    rf = int(np.prod(shape[:-2]))
    return shape[-2] * rf, shape[-1] * rf


def init_weights(seed=0, perturb=0.02, **kw):
    """Keras-default-like init: glorot_uniform kernels, zero bias, LN gamma=1/beta=0,
    Embedding U(-0.05,0.05) [upstream].  `perturb` adds N(0, perturb) to biases, gamma
    and beta so parity runs exercise every term."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in weight_shapes(**kw).items():
        if name.endswith("/embeddings"):
            v = rng.uniform(-0.05, 0.05, size=shape)
        elif name.endswith("/kernel"):
            fi, fo = _fans(shape)
            lim = math.sqrt(6.0 / (fi + fo))
            v = rng.uniform(-lim, lim, size=shape)
        elif name.endswith("/gamma"):
            v = np.ones(shape) + (rng.normal(0, perturb, size=shape) if perturb else 0)
        else:  # bias / beta
            v = rng.normal(0, perturb, size=shape) if perturb else np.zeros(shape)
        out[name] = v.astype(np.float32)
    return out


def synthetic_images(batch, shape, seed=1, letterbox=False):
    """NHWC U(-1,1) images (utils.py:446-447 range); optional -1 letterbox bands."""
    rng = np.random.default_rng(seed)
    h, w, c = shape
    img = rng.uniform(-1.0, 1.0, size=(batch, h, w, c)).astype(np.float32)
    if letterbox:
        band = h // 8
        img[:, :band] = -1.0
        img[:, h - band:] = -1.0
    return img


OBJECTNESS_THRESHOLD = 0.5                   # vtd.py:41
CLASSIFICATION_CONFIDENCE_THRESHOLD = 0.5    # vtd.py:43


def detection_mask(decoded, obj_thr=OBJECTNESS_THRESHOLD,
                   cls_thr=CLASSIFICATION_CONFIDENCE_THRESHOLD):
    """MeanAveragePrecision.update_state's prediction test (vtd.py:1359-1384) on the
    output of transform_predictions: category = tf.round(class) (half to even, as
    np.round), confidence = (0.5 - |class - category|) / 0.5, valid = objectness > 0.5
    and confidence > 0.5.  Returns (category int32, valid bool)."""
    d = np.asarray(decoded, dtype=np.float64)
    cat = np.round(d[..., 1])
    conf = (0.5 - np.abs(d[..., 1] - cat)) / 0.5
    valid = (d[..., 0] > obj_thr) & (conf > cls_thr)
    return cat.astype(np.int32), valid
