"""Whole-forward parity of the path the bench times, at the configurations' real batch
sizes (VERDICT r1 "what's weak" #1).

The B=1 goldens in test_gpu_model.py run the small-problem kernels (128-tile GEMM, the
row-statistics pass, one stream).  Here the golden images (tests/golden/batched_forward.json,
fp64 oracle logits per image, made by `make_golden.py batched`) are placed among random
filler images in a batch of the config's real size, so the forward takes the default
large-batch path:

  * C2 B=256 (the headline): 256x256 ping-pong GEMMs (pp2), LayerNorm folded into the
    query/key/value and first MLP GEMMs with the statistics emitted by the producing GEMMs
    (centred partials + finalize), the bf16 residual stream, and the two-stream split
    (two halves of 128 images on the caller's stream and the internal stream);
  * C2 B=64 (one stream, 49 row tiles), C3 B=32 (N = 1600, two streams), C5 B=128
    (ViT-L, two streams) in bf16, the MX-fp8 mode and the f32 parity mode.

Every golden row is compared to its fp64 oracle logits (oracle/vtd_numpy.py:190-222 ->
vtd.py:498-583) with the tolerances of test_gpu_model.py:
  float32 1e-3 (north_star), bf16x3 (split-bf16 parity mode) 1e-4, bfloat16 3e-2,
  float8 1e-1, in the form
  |y - ref| <= tol |ref| + tol max|ref| per image.
Filler images differ from the goldens, so a row that read another image's data fails.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import vtd_numpy as V

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL = {"float32": 1e-3, "bf16x3": 1e-4, "bfloat16": 3e-2, "float8": 1e-1}

# (case, batch, golden positions in the batch): both micro-batch halves, their edges, and
# rows in the middle
CASES = {
    "c2_b256": ("c2_vitb16_imgs8", 256, [0, 1, 97, 127, 128, 200, 254, 255]),
    "c2_b64": ("c2_vitb16_imgs8", 64, [0, 13, 31, 32, 45, 50, 62, 63]),
    "c3_b32": ("c3_vitb16_640_imgs3", 32, [0, 16, 31]),
    "c5_b128": ("c5_vitl16_384_imgs3", 128, [0, 64, 127]),
}
PARAMS = [("c2_b256", "bfloat16"), ("c2_b256", "float32"), ("c2_b256", "float8"),
          ("c2_b256", "bf16x3"),
          ("c2_b64", "bfloat16"), ("c2_b64", "float32"), ("c2_b64", "bf16x3"),
          ("c3_b32", "bfloat16"), ("c3_b32", "float8"), ("c3_b32", "float32"),
          ("c3_b32", "bf16x3"),
          ("c5_b128", "bfloat16"), ("c5_b128", "float8"), ("c5_b128", "float32"),
          ("c5_b128", "bf16x3")]

_spec_cache = {}
_weight_cache = {}


def _spec(name):
    if not _spec_cache:
        _spec_cache.update(json.load(open(os.path.join(GOLD, "batched_forward.json"))))
    return _spec_cache[name]


def _weights(spec):
    key = (json.dumps(spec["kwargs"], sort_keys=True), spec["weight_seed"])
    if key not in _weight_cache:
        _weight_cache.clear()                 # one preset's fp32 weights at a time
        kw = dict(spec["kwargs"])
        _weight_cache[key] = V.init_weights(seed=spec["weight_seed"], perturb=spec["perturb"],
                                            **kw)
    return _weight_cache[key]


def within(y, ref, tol):
    y, ref = np.asarray(y, np.float64), np.asarray(ref, np.float64)
    bound = tol * np.abs(ref) + tol * np.abs(ref).max()
    return bool(np.all(np.abs(y - ref) <= bound)), float(np.abs(y - ref).max() / np.abs(ref).max())


@pytest.fixture(scope="module")
def vtd(cuda):
    import vision_transformer_detector_amd as m
    return m


@pytest.mark.parametrize("case,dtype", PARAMS)
def test_batched_forward_matches_golden(vtd, cuda, case, dtype):
    name, batch, pos = CASES[case]
    spec = _spec(name)
    kw = dict(spec["kwargs"])
    kw["input_shape"] = tuple(kw["input_shape"])
    shape = V.resolve_kwargs(**kw)["input_shape"]
    imgs = V.synthetic_images(spec["n"], shape, seed=spec["image_seed"],
                              letterbox=spec["letterbox"])
    import hashlib
    assert hashlib.sha256(np.ascontiguousarray(imgs, np.float32).tobytes()).hexdigest() == \
        spec["images_sha256"], "golden images no longer regenerate from their seed"
    w = _weights(spec)
    model = vtd.create_vision_transformer_detector(**kw, dtype=dtype, device=cuda)
    model.set_weights(w)
    gen = torch.Generator(device=cuda).manual_seed(77)
    x = torch.rand((batch,) + tuple(shape), generator=gen, device=cuda) * 2 - 1
    for i, p in enumerate(pos):
        x[p] = torch.from_numpy(imgs[i]).to(cuda)
    logits, dets = model.detect(x)              # the bench's step: forward + fused decode
    torch.cuda.synchronize()
    y = logits.cpu().numpy()
    d = dets.cpu().numpy()
    worst = 0.0
    for i, p in enumerate(pos):
        ref = np.asarray(spec["logits"][i])
        ok, rel = within(y[p], ref, TOL[dtype])
        worst = max(worst, rel)
        assert ok, f"{case} {dtype}: image {i} at row {p}: max rel err {rel:.3e}"
        if dtype in ("float32", "bf16x3"):
            np.testing.assert_allclose(d[p], V.transform_predictions(ref[None])[0],
                                       rtol=1e-3, atol=1e-3 * 608)
    assert np.isfinite(y).all()
    print(f"{case} {dtype}: worst max-rel err over {len(pos)} golden rows {worst:.3e}")
