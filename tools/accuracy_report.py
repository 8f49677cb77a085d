"""Max relative logit error of every golden case per dtype (GPU): the numbers behind the
model-parity tolerances.  `VTD_RESID_F32=1 python tools/accuracy_report.py` measures the
f32 residual stream in the bf16 / fp8 modes for comparison.
  python tools/accuracy_report.py [--out FILE]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import vtd_numpy as V  # noqa: E402
import vision_transformer_detector_amd as vtd  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def rel(y, ref):
    y, ref = np.asarray(y, np.float64), np.asarray(ref, np.float64)
    return float(np.abs(y - ref).max() / np.abs(ref).max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    res = {"resid_f32_env": os.environ.get("VTD_RESID_F32", "0")}
    seeded = json.load(open(os.path.join(GOLD, "seeded_forward.json")))
    for dtype in ("float32", "bf16x3", "bfloat16", "float8"):
        for name in ("tiny_mish", "tiny_gelu", "tiny_seq400"):
            z = np.load(os.path.join(GOLD, f"{name}.npz"))
            kw = json.loads(str(z["kwargs"]))
            if "input_shape" in kw:
                kw["input_shape"] = tuple(kw["input_shape"])
            m = vtd.create_vision_transformer_detector(**kw, dtype=dtype)
            m.set_weights({k[2:]: z[k] for k in z.files if k.startswith("w:")})
            res[f"{name}/{dtype}"] = rel(m(torch.from_numpy(z["images"]).to(dev)).cpu().numpy(),
                                         z["logits"])
        for case, spec in seeded.items():
            kw = dict(spec["kwargs"])
            if "input_shape" in kw:
                kw["input_shape"] = tuple(kw["input_shape"])
            w = V.init_weights(seed=spec["weight_seed"], perturb=spec["perturb"], **kw)
            shape = V.resolve_kwargs(**kw)["input_shape"]
            x = V.synthetic_images(spec["batch"], shape, seed=spec["image_seed"],
                                   letterbox=spec["letterbox"])
            m = vtd.create_vision_transformer_detector(**kw, dtype=dtype)
            m.set_weights(w)
            res[f"{case}/{dtype}"] = rel(m(torch.from_numpy(x).to(dev)).cpu().numpy(),
                                         np.array(spec["logits"]))
            del m
            torch.cuda.empty_cache()
        print(dtype, {k: f"{v:.2e}" for k, v in res.items() if k.endswith(dtype)}, flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
