"""Writes tests/golden/tiny_keras.h5: the Keras 2.9 HDF5 layout of `model.save('*.keras')`
(vtd.py:2146, 2179) for the smoke-size detector config, with the oracle's seeded weights
(oracle.vtd_numpy.init_weights(seed=3)) under the Keras weight names of SURVEY App. B.3
and the layer names of the reference's plot_model diagram (tests/golden/plot_model_shapes.json).

No h5py / TF here, so the file is produced by tests/golden/h5_writer.py, which writes the
structures h5py writes at its default settings: PARITY UNPINNED against a file saved by
Keras itself (none ships with the reference).

  python tests/golden/make_keras_h5.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from h5_writer import write_keras_model  # noqa: E402
from oracle import vtd_numpy as ref  # noqa: E402

TINY = dict(input_shape=(40, 36, 3), patch_size=8, embedding_dim=24, encoder_num_heads=3,
            encoder_key_dim=10, encoder_mlp_quantities=3, encoder_repeat_times=2,
            mlp_head_last_units=8, mlp_head_dense_layers_quantity=3)
SEED = 3


def keras_layers(kw, weights):
    """Layer names in model order (vtd.py:498-583; names as in plot_model_shapes.json) and
    {layer: [(weight name + ':0', array)]} grouped by each weight's owning layer."""
    order = ["images", "split_image_into_patches", "flatten_patches", "linear_projection",
             "position_encoding", "embedded_patches"]
    act = 0
    for i in range(1, kw["encoder_repeat_times"] + 1):
        order += ["layer_normalization" if i == 1 else f"layer_normalization_{2 * i - 2}",
                  "multi_head_attention" if i == 1 else f"multi_head_attention_{i - 1}",
                  f"residual_connection_{i}_1", f"layer_normalization_{2 * i - 1}"]
        for j in range(1, kw["encoder_mlp_quantities"] + 1):
            order += [f"MLP_{i}_{j}", "mish_activation" if act == 0 else f"mish_activation_{act}"]
            act += 1
        order.append(f"residual_connection_{i}_2")
    order += ["dense", "reshape"]
    n_head = sum(1 for k in weights if k.startswith("dense_") and k.endswith("/kernel"))
    for j in range(1, n_head + 1):
        order += [f"dense_{j}", f"mish_activation_{act}"]
        act += 1
    order.append("MLP_Head_no_Sigmoid")
    grouped = {}
    for name, arr in weights.items():
        grouped.setdefault(name.split("/")[0], []).append((name + ":0", arr))
    missing = set(grouped) - set(order)
    assert not missing, missing
    return order, grouped


def main(path=os.path.join(os.path.dirname(os.path.abspath(__file__)), "tiny_keras.h5")):
    kw = ref.resolve_kwargs(**TINY)
    w = ref.init_weights(seed=SEED, **TINY)
    order, grouped = keras_layers(kw, w)
    cfg = {"class_name": "Functional", "config": {"name": "vision_transformer_detector"},
           "_note": "stand-in model_config (the reference's get_config JSON is not reproduced)"}
    write_keras_model(path, grouped, order, model_config=cfg)
    print(path, os.path.getsize(path), "bytes,", len(w), "weights")


if __name__ == "__main__":
    main()
