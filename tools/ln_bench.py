"""LayerNorm pass bandwidth through the C-ABI (C5: 73728 rows x 1024, bf16 stream in): the
MX-fp8 LayerNorm (vtd_layernorm_mx8, the fp8 mode's LN pass), the bf16 LayerNorm and, as the
attainable reference for a read + write stream of the same bytes, torch's bf16 -> fp8-sized copy.
  python tools/ln_bench.py [--reps 20] [--rows 73728] [--D 1024]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_transformer_detector_amd import _lib as L  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rows", type=int, default=73728)
    ap.add_argument("--D", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    R, D = a.rows, a.D
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(R, D, generator=g, device=dev) * 3 + 1).to(torch.bfloat16)
    gamma = torch.ones(D, device=dev)
    beta = torch.zeros(D, device=dev)
    s_rows = -(-R // 4) * 4
    q = torch.empty(R, D, dtype=torch.uint8, device=dev)
    s = torch.empty(D // 128 * s_rows * 4, dtype=torch.uint8, device=dev)
    h = torch.empty(R, D, dtype=torch.bfloat16, device=dev)
    st = L.stream_ptr()
    mx = lambda: L.check(L.lib.vtd_layernorm_mx8(x.data_ptr(), L.BF16, R, D, D, gamma.data_ptr(),
                                                 beta.data_ptr(), 1e-3, q.data_ptr(), D, D,
                                                 s.data_ptr(), s_rows, st), "ln_mx8")
    bf = lambda: L.check(L.lib.vtd_layernorm(x.data_ptr(), L.BF16, R, D, D, gamma.data_ptr(),
                                             beta.data_ptr(), 1e-3, h.data_ptr(), D, L.BF16, st),
                         "ln")
    cp2 = lambda: h.copy_(x)                             # read + write R*D*2 B each
    res = {"rows": R, "D": D}
    for name, fn, nbytes in (("ln_mx8", mx, R * D * 3 + R * D // 32),
                             ("ln_bf16", bf, R * D * 4),
                             ("torch_copy_bf16", cp2, R * D * 4)):
        us = timed(fn, a.reps)
        res[name] = {"us": round(us, 2), "TBps": round(nbytes / us / 1e6, 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
