"""Attention kernel micro-benchmark through the C-ABI at the C2 shape (B=256, N=196, 12
heads x 64, bf16), for rocprofv3 PMC passes and variant A/B (knob VTD_KNOB_ATTN_VARIANT,
interleaved rounds in one process).
  python tools/attn_bench.py [--reps 20] [--B 256] [--N 196] [--flush] [--variants 4,5] [--rounds 3]"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_transformer_detector_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--N", type=int, default=196)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--flush", action="store_true", help="evict the MALL between reps")
    ap.add_argument("--variants", default="-1")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32", "x3"],
                    help="x3: the split-bf16 kernel (f32 qkv in, [hi | lo] out)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, N, H, dkp = a.B, a.N, a.H, 64
    ld = 3 * H * dkp
    g = torch.Generator(device=dev).manual_seed(0)
    code = {"bf16": L.BF16, "f32": L.F32, "x3": L.BF16X3}[a.dtype]
    qkv = torch.randn(B * N, ld, generator=g, device=dev) * 1.5
    if a.dtype == "bf16":
        qkv = qkv.to(torch.bfloat16)
    ldo = 2 * H * dkp if a.dtype == "x3" else H * dkp
    out = torch.empty(B * N, ldo, device=dev,
                      dtype=torch.float32 if a.dtype == "f32" else torch.bfloat16)
    junk = torch.empty(512 << 20, dtype=torch.uint8, device=dev) if a.flush else None
    st = L.stream_ptr()
    call = lambda: L.check(L.lib.vtd_attention(qkv.data_ptr(), B, N, H, dkp, ld, 1 / math.sqrt(64),
                                               out.data_ptr(), ldo, code, st))
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(a.rounds):
        for v in [int(x) for x in a.variants.split(",")]:
            with L.knob(L.KNOB_ATTN_VARIANT, v):
                for _ in range(3):
                    call()
                ms = 0.0
                for _ in range(a.reps):
                    if junk is not None:
                        junk.fill_(1)
                    t0.record()
                    call()
                    t1.record()
                    torch.cuda.synchronize()
                    ms += t0.elapsed_time(t1)
            us = 1e3 * ms / a.reps
            byts = B * N * (ld * qkv.element_size() + ldo * out.element_size())
            print(json.dumps({"dtype": a.dtype, "variant": v, "round": rnd, "B": B, "N": N,
                              "flush": a.flush, "us": round(us, 2),
                              "hbm_tbs": round(byts / us / 1e6, 2),
                              "tflops": round(4.0 * B * H * N * N * 64 / us / 1e6, 1)}), flush=True)

if __name__ == "__main__":
    main()
