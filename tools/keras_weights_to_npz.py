"""Export the weights of a reference Keras model (vision_transformer_detector.py, TF 2.9)
to the name-keyed .npz this package loads with Model.load_weights.

Run where TensorFlow / tensorflow-addons are installed (not in this repo's pipeline):
  python tools/keras_weights_to_npz.py checkpoints/highest_ap_vision_transformer_detector.keras out.npz

The reference saves with model.save('*.keras') (vtd.py:2146, 2179), which TF 2.x writes as
HDF5; loading needs the custom layers as custom_objects (cf. SaveModelHighestAP,
vtd.py:2118-2125).
"""
import sys

import numpy as np


def main(src, dst):
    from tensorflow import keras  # noqa: F401  (reference environment only)
    import vision_transformer_detector as vtd  # the reference module
    model = keras.models.load_model(src, compile=False, custom_objects={
        "MishActivation": vtd.MishActivation, "PositionEncoding": vtd.PositionEncoding,
        "ExtractImagePatches": vtd.ExtractImagePatches, "ClipWeight": vtd.ClipWeight})
    np.savez(dst, **{w.name.split(":")[0]: w.numpy() for w in model.weights})
    print(f"wrote {len(model.weights)} arrays to {dst}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
