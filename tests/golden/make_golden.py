"""Generates the golden fixtures in tests/golden/ from the fp64 NumPy oracle.

The reference (TF 2.9 / Keras / tfa) cannot be imported in this pipeline (SURVEY.md §8c:
ModuleNotFoundError, no network), so the vectors come from the oracle restatement
(`oracle/vtd_numpy.py`), cross-checked against the independent torch restatement when
they are generated.  Inputs and weights are regenerated from seeds (numpy PCG64 is
platform-stable) for the large C1/C2 cases; tiny cases store everything explicitly.

Run:  python tests/golden/make_golden.py [seeded case names ...]
      python tests/golden/make_golden.py batched [batched case names ...]
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import torch  # noqa: E402

from oracle import vtd_numpy as V  # noqa: E402
from oracle import vtd_torch_cpu as T  # noqa: E402

TINY = {
    # small Mish model: SAME padding on both axes (40 = 5*8, 36 -> 5 cols, pad 4)
    "tiny_mish": dict(kw=dict(input_shape=(40, 36, 3), patch_size=8, embedding_dim=24,
                              encoder_num_heads=3, encoder_key_dim=10,
                              encoder_mlp_quantities=3, encoder_repeat_times=2,
                              mlp_head_last_units=8, mlp_head_dense_layers_quantity=3),
                      batch=3, seed=11),
    # GELU, odd sizes everywhere, head block repeats 2
    "tiny_gelu": dict(kw=dict(input_shape=(33, 50, 3), patch_size=7, embedding_dim=20,
                              encoder_num_heads=2, encoder_key_dim=12,
                              encoder_mlp_quantities=2, encoder_repeat_times=2,
                              mlp_head_last_units=4, mlp_head_dense_layers_quantity=5,
                              mlp_head_dense_mish_block_repeats=2, use_mish=False),
                      batch=2, seed=12),
    # long-ish sequence (N = 20*20 = 400 tokens > one KV tile), heads*dk odd
    "tiny_seq400": dict(kw=dict(input_shape=(80, 80, 3), patch_size=4, embedding_dim=32,
                                encoder_num_heads=3, encoder_key_dim=16,
                                encoder_mlp_quantities=2, encoder_repeat_times=1,
                                mlp_head_last_units=16, mlp_head_dense_layers_quantity=2),
                        batch=2, seed=13),
}

SEEDED = {
    # reference default config (ipynb:394-403), one image, weights/images from seeds
    "c1_default_b1": dict(kw={}, batch=1, wseed=0, iseed=1, letterbox=True),
    # ViT-B/16 preset, one image
    "c2_vitb16_b1": dict(kw=dict(input_shape=(224, 224, 3), patch_size=16, embedding_dim=768,
                                 encoder_num_heads=12, encoder_key_dim=64,
                                 encoder_repeat_times=12, encoder_mlp_quantities=3,
                                 use_mish=False), batch=1, wseed=0, iseed=1, letterbox=False),
    # C3: ViT-B/16 preset at 640x640 (N = 1600 tokens: long-sequence attention)
    "c3_vitb16_640_b1": dict(kw="vit_b16_640", batch=1, wseed=0, iseed=1, letterbox=True),
    # C5: ViT-L/16 preset at 384x384 (D 1024, 16 heads, 24 layers)
    "c5_vitl16_384_b1": dict(kw="vit_l16_384", batch=1, wseed=0, iseed=1, letterbox=True),
}

# Multi-image cases for the batched parity tests (tests/test_gpu_batch_parity.py): the
# same weights as the b1 case of the preset, `n` distinct images from one seed, each
# image's fp64 logits stored.  The GPU test places them among random filler images in a
# batch of the config's real size (C2 B=256 / 64, C3 B=32, C5 B=128), so the timed
# kernels (256-tile GEMMs, producer LayerNorm statistics, two streams) are what is checked.
BATCHED = {
    "c2_vitb16_imgs8": dict(kw="vit_b16_224", n=8, wseed=0, iseed=100, letterbox=True),
    "c3_vitb16_640_imgs3": dict(kw="vit_b16_640", n=3, wseed=0, iseed=101, letterbox=True),
    "c5_vitl16_384_imgs3": dict(kw="vit_l16_384", n=3, wseed=0, iseed=102, letterbox=True),
}


def make_batched(names=None):
    from vision_transformer_detector_amd import presets
    path = os.path.join(HERE, "batched_forward.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name, c in BATCHED.items():
        if names and name not in names:
            continue
        kw = dict(presets.PRESETS[c["kw"]])
        shape = V.resolve_kwargs(**kw)["input_shape"]
        w = V.init_weights(seed=c["wseed"], perturb=0.02, **kw)
        x = V.synthetic_images(c["n"], shape, seed=c["iseed"], letterbox=c["letterbox"])
        ys = [V.forward(w, x[i:i + 1], **kw)[0] for i in range(c["n"])]
        y2 = T.TorchCpuDetector(w, dtype=torch.float64, **kw)(x[:1]).numpy()[0]
        assert np.abs(ys[0] - y2).max() < 1e-12, name
        out[name] = dict(preset=c["kw"], kwargs=kw, n=c["n"], weight_seed=c["wseed"],
                         perturb=0.02, image_seed=c["iseed"], letterbox=c["letterbox"],
                         images_sha256=digest(x),
                         weights_sha256=digest(np.concatenate([v.ravel() for v in w.values()])),
                         logits=[y.tolist() for y in ys])
        print(name, float(max(np.abs(y).max() for y in ys)), flush=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


def main(only=None):
    """only: names of SEEDED cases to (re)compute, merged into the existing JSON (the
    tiny fixtures are then left untouched)."""
    from vision_transformer_detector_amd import presets
    for name, c in TINY.items():
        if only:
            break
        kw = c["kw"]
        w = V.init_weights(seed=c["seed"], perturb=0.02, **kw)
        x = V.synthetic_images(c["batch"], V.resolve_kwargs(**kw)["input_shape"],
                               seed=c["seed"] + 100)
        y = V.forward(w, x, **kw)
        y2 = T.TorchCpuDetector(w, dtype=torch.float64, **kw)(x).numpy()
        assert np.abs(y - y2).max() < 1e-12, name
        arrays = {f"w:{k}": v for k, v in w.items()}
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), images=x, logits=y,
                            dets=V.transform_predictions(y),
                            kwargs=np.array(json.dumps(kw)), **arrays)
        print(name, y.shape, float(np.abs(y).max()))
    path = os.path.join(HERE, "seeded_forward.json")
    seeded = json.load(open(path)) if only else {}
    for name, c in SEEDED.items():
        if only and name not in only:
            continue
        kw = c["kw"] if isinstance(c["kw"], dict) else dict(presets.PRESETS[c["kw"]])
        shape = V.resolve_kwargs(**kw)["input_shape"]
        w = V.init_weights(seed=c["wseed"], perturb=0.02, **kw)
        x = V.synthetic_images(c["batch"], shape, seed=c["iseed"], letterbox=c["letterbox"])
        y = V.forward(w, x, **kw)
        y2 = T.TorchCpuDetector(w, dtype=torch.float64, **kw)(x).numpy()
        assert np.abs(y - y2).max() < 1e-12, name
        seeded[name] = dict(kwargs=kw, batch=c["batch"], weight_seed=c["wseed"],
                            perturb=0.02, image_seed=c["iseed"], letterbox=c["letterbox"],
                            images_sha256=digest(x),
                            weights_sha256=digest(np.concatenate(
                                [v.ravel() for v in w.values()])),
                            logits=y.tolist())
        print(name, float(np.abs(y).max()))
    with open(path, "w") as f:
        json.dump(seeded, f, indent=1)
    if only:
        return
    shapes = V.layer_output_shapes()
    with open(os.path.join(HERE, "oracle_layer_shapes_c1.json"), "w") as f:
        json.dump({k: list(v) for k, v in shapes.items()}, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1:2] == ["batched"]:
        make_batched(sys.argv[2:] or None)
    else:
        main(sys.argv[1:] or None)
