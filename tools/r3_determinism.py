"""Round 3 check: repeatability of the C2 forward (128 images, bf16) and the effect of the
A/B switches VTD_LN_FINALIZE / VTD_SPLITK on the logits (max abs diff)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vision_transformer_detector_amd as vtd  # noqa: E402
from oracle import vtd_numpy as V  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
spec = json.load(open(os.path.join(GOLD, "seeded_forward.json")))["c2_vitb16_b1"]
kw = dict(spec["kwargs"])
w = V.init_weights(seed=spec["weight_seed"], perturb=spec["perturb"], **kw)
shape = V.resolve_kwargs(**kw)["input_shape"]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
x = torch.from_numpy(V.synthetic_images(B, shape, seed=5)).to("cuda")
model = vtd.create_vision_transformer_detector(**kw, dtype="bfloat16")
model.set_weights(w)


def run(**env):
    for k in ("VTD_LN_FINALIZE", "VTD_SPLITK", "VTD_STREAMS"):
        os.environ.pop(k, None)
    os.environ.update(env)
    y = model(x).clone()
    torch.cuda.synchronize()
    return y


a1, a2 = run(), run()
s1, s2 = run(VTD_LN_FINALIZE="1"), run(VTD_LN_FINALIZE="1")
k1 = run(VTD_SPLITK="0")
o1 = run(VTD_STREAMS="1")
o2 = run(VTD_STREAMS="1", VTD_LN_FINALIZE="1")
d = lambda p, q: float((p - q).abs().max())
print(json.dumps({"B": B, "fused_repeat": d(a1, a2), "sep_repeat": d(s1, s2), "fused_vs_sep": d(a1, s1),
                  "splitk_off_vs_on": d(a1, k1), "one_stream_fused_vs_sep": d(o1, o2),
                  "one_vs_two_stream": d(a1, o1), "max_abs_logit": float(a1.abs().max())}))
