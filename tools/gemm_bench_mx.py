"""MX-fp8 GEMM micro-benchmark through the C-ABI (vtd_gemm_mx8): TFLOP/s per C5 encoder shape
(ViT-L/16 @384, B=128: M = 73728) for A/B-ing the MX kernels (VTD_MX_VARIANT) in one
process.  Operands are quantized once with vtd_quantize_mx8.

  python tools/gemm_bench_mx.py [--variants 1,2] [--reps 10] [--shapes qkv,mlp2]
"""
import argparse
import ctypes
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_transformer_detector_amd import _lib as L  # noqa: E402

SHAPES = {  # name: (M, N, K, act, out (1 bf16, 2 MX-fp8), resid)
    "qkv": (73728, 3072, 1024, 0, 1, False),
    "attn_out": (73728, 1024, 1024, 0, 1, True),
    "mlp1": (73728, 4096, 1024, 1, 2, False),
    "mlp2": (73728, 2048, 4096, 1, 2, False),
    "mlp3": (73728, 1024, 2048, 1, 1, True),
    "sq8192": (8192, 8192, 8192, 0, 1, False),
}


def quantize(x):
    rows, K = x.shape
    s_rows = -(-rows // 4) * 4
    q = torch.empty(rows, K, dtype=torch.uint8, device=x.device)
    s = torch.empty(K // 128 * s_rows * 4, dtype=torch.uint8, device=x.device)
    L.check(L.lib.vtd_quantize_mx8(x.data_ptr(), L.BF16, rows, K, K, K, q.data_ptr(), K,
                                   s.data_ptr(), s_rows, L.stream_ptr()), "quantize_mx8")
    return q, s, s_rows


def run(name, spec, reps, variants, dev):
    M, N, K, act, od, res = spec
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand(N, K, generator=g, device=dev) * 2 - 1) / math.sqrt(K)).to(torch.bfloat16)
    qa, sa, sar = quantize(A)
    qb, sb, sbr = quantize(W)
    del A, W
    bias = torch.zeros(N, device=dev)
    e = L.VtdEpilogue()
    e.bias, e.act, e.ldo = bias.data_ptr(), act, N
    if od == 2:
        out = torch.empty(M, N, device=dev, dtype=torch.uint8)
        so = torch.empty(N // 128 * sar * 4, device=dev, dtype=torch.uint8)
        e.out, e.out_dtype, e.scale_out, e.scale_rows = out.data_ptr(), 2, so.data_ptr(), sar
    else:
        out = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        e.out, e.out_dtype = out.data_ptr(), 1
        if res:
            e.resid, e.ldr = out.data_ptr(), N
    st = L.stream_ptr()
    call = lambda: L.check(L.lib.vtd_gemm_mx8(M, N, K, qa.data_ptr(), K, sa.data_ptr(), sar,
                                              qb.data_ptr(), K, sb.data_ptr(), sbr,
                                              ctypes.byref(e), st), "gemm_mx8")
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out_rows = []
    for v in variants:
        os.environ["VTD_MX_VARIANT"] = v
        for _ in range(2):
            call()
        t0.record()
        for _ in range(reps):
            call()
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / reps
        out_rows.append({"shape": name, "variant": v, "dg": os.environ.get("VTD_X4_DG", "0"),
                         "us": round(ms * 1e3, 1),
                         "tflops": round(2 * M * N * K / ms / 1e9, 1)})
    return out_rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="1,2")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for name in args.shapes.split(","):
        for r in run(name, SHAPES[name], args.reps, args.variants.split(","), dev):
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
