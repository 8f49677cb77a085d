"""Tile-tail experiment through the C-ABI (C2 at B = 64: 49 row tiles of 256).

A GEMM whose 256 x 256 tile count leaves a small last round (mlp2 at B = 64: 294 tiles = one
round + 38) timed three ways on one stream:
  plain   -- vtd_gemm over all rows;
  tail    -- the rows of the last m-tiles first as split-K partials (vtd_gemm_splitk with
             ksplit pieces: its partial launch + reduce), then vtd_gemm over the leading m-tiles
             (whole rounds only);
  splitk  -- vtd_gemm_splitk over all rows.
  python tools/tail_bench.py [--reps 20]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_transformer_detector_amd import _lib as L  # noqa: E402

# name: (M, N, K, act)  -- C2 B = 64 encoder layers without residual / statistics
SHAPES = {"mlp2_b64": (12544, 1536, 3072, 1), "mlp1_b64": (12544, 3072, 768, 1),
          "qkv_b64": (12544, 2304, 768, 0), "mlp3_b64_nost": (12544, 768, 1536, 1),
          "attn_out_b64_nost": (12544, 768, 768, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    st = L.stream_ptr()
    for name in args.shapes.split(","):
        M, N, K, act = SHAPES[name]
        g = torch.Generator(device=dev).manual_seed(0)
        A = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        Bt = (torch.rand(N, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        bias = torch.zeros(N, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        part = torch.empty(8 * M * N, device=dev, dtype=torch.float32)

        def epi(row0):
            e = L.VtdEpilogue()
            e.bias, e.act = bias.data_ptr(), act
            e.out, e.ldo, e.out_dtype = out.data_ptr() + row0 * N * 2, N, L.BF16
            return e

        tm, tn = M // 256, (N + 255) // 256
        calls = {"plain": lambda: L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K,
                                                        L.BF16, ctypes.byref(epi(0)), st))}
        for ks in (2, 3, 4):
            calls[f"splitk{ks}"] = (lambda ks=ks: L.check(L.lib.vtd_gemm_splitk(
                M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16, ctypes.byref(epi(0)), part.data_ptr(),
                part.numel() * 4, ks, st)))
        # leading m-tiles: whole rounds of 256 tiles; the rest split-K near one round
        full = (tm * tn) // 256
        if full >= 1:
            m_main = (full * 256) // tn
            m_rem = tm - m_main
            for ks in (2, 3, 4, 6, 8):
                if m_rem * tn * ks > 288 or K // 64 < 4 * ks:
                    continue
                r0 = m_main * 256

                def tail(ks=ks, r0=r0, m_rem=m_rem, m_main=m_main):
                    L.check(L.lib.vtd_gemm_splitk(m_rem * 256, N, K, A.data_ptr() + r0 * K * 2, K,
                                                  Bt.data_ptr(), K, L.BF16, ctypes.byref(epi(r0)),
                                                  part.data_ptr(), part.numel() * 4, ks, st))
                    L.check(L.lib.vtd_gemm(m_main * 256, N, K, A.data_ptr(), K, Bt.data_ptr(), K,
                                           L.BF16, ctypes.byref(epi(0)), st))
                calls[f"tail_m{m_main}_ks{ks}"] = tail
        res = {"shape": name, "tiles": tm * tn}
        ref = None
        for label, call in calls.items():
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(args.reps):
                call()
            t1.record()
            torch.cuda.synchronize()
            res[label] = round(t0.elapsed_time(t1) / args.reps * 1e3, 1)
            o = out.float()
            if ref is None:
                ref = o.clone()
            else:
                res[label + "_maxdiff"] = float((o - ref).abs().max())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
