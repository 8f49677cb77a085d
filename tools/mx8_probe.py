"""Probe of the MX-fp8 GEMM's operand / scale conventions on the GPU (debug aid):
runs vtd_gemm_mx8 on hand-built e4m3 bytes and scale patterns and prints the max error
against the fp64 product for each experiment.
  python tools/mx8_probe.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import mx8 as MX  # noqa: E402
from vision_transformer_detector_amd import _lib as L  # noqa: E402


def run(qa, sa, qb, sb, M, N, K):
    dev = torch.device("cuda:0")
    ta, tsa = torch.from_numpy(qa).to(dev), torch.from_numpy(sa).to(dev)
    tb, tsb = torch.from_numpy(qb).to(dev), torch.from_numpy(sb).to(dev)
    out = torch.zeros(M, N, device=dev)
    bias = torch.zeros(N, device=dev)
    e = L.VtdEpilogue()
    e.bias, e.out, e.ldo, e.out_dtype = bias.data_ptr(), out.data_ptr(), N, 0
    L.check(L.lib.vtd_gemm_mx8(M, N, K, ta.data_ptr(), K, tsa.data_ptr(), M, tb.data_ptr(), K,
                               tsb.data_ptr(), N, ctypes.byref(e), L.stream_ptr()), "mx8")
    torch.cuda.synchronize()
    return out.cpu().numpy().astype(np.float64)


def main():
    rng = np.random.default_rng(0)
    M = N = 256
    K = 256
    # bytes of small e4m3 values: exponent field 6..8 (0.5 .. 3.75), random mantissa/sign
    def rnd_bytes(r, c):
        ex = rng.integers(6, 9, size=(r, c))
        return ((rng.integers(0, 2, size=(r, c)) << 7) | (ex << 3) | rng.integers(0, 8, size=(r, c))).astype(np.uint8)
    qa, qb = rnd_bytes(M, K), rnd_bytes(N, K)
    A, B = MX.decode_e4m3(qa), MX.decode_e4m3(qb)
    ones_a = np.full(K // 128 * M * 4, 127, np.uint8)
    ones_b = np.full(K // 128 * N * 4, 127, np.uint8)
    ref = A @ B.T
    got = run(qa, ones_a, qb, ones_b, M, N, K)
    print("unit scales: max abs err", np.abs(got - ref).max(), "max|ref|", np.abs(ref).max())
    # scale 2^1 on A block (row r, kblock b) for one block at a time
    for (r, kb) in [(0, 0), (0, 1), (5, 2), (17, 3), (100, 5)]:
        sa = ones_a.copy().reshape(K // 128, M, 4)
        sa[kb // 4, r, kb % 4] = 128
        Ae = A.copy()
        Ae[r, 32 * kb:32 * kb + 32] *= 2
        got = run(qa, sa.reshape(-1), qb, ones_b, M, N, K)
        err = np.abs(got - Ae @ B.T)
        print(f"A scale x2 at row {r} block {kb}: max err {err.max():.3g}, rows with err:",
              np.unique(np.argwhere(err > 1e-3)[:, 0])[:8])
        # solve got[r] - ref[r] = sum_k d_k B[n][k] for d_k = (f_k - 1) A[r][k]
        d = np.linalg.lstsq(B, got[r] - A[r] @ B.T, rcond=None)[0]
        f = 1 + d / np.where(A[r] != 0, A[r], 1)
        chg = np.argwhere(np.abs(f - 1) > 1e-3)[:, 0]
        print("   k with factor != 1:", chg[:4], "...", chg[-4:], "count", len(chg),
              "factors", np.unique(np.round(f[chg], 3))[:6])
        # which 32-block (or which factor) was actually scaled
        for b2 in range(K // 32):
            for f in (2.0, 4.0, 0.5):
                A3 = A.copy()
                A3[r, 32 * b2:32 * b2 + 32] *= f
                if np.abs(got[r] - A3[r] @ B.T).max() < 1e-3:
                    print(f"   -> matches block {b2} x{f}")
        for f in (2.0, 4.0, 0.5):
            if np.abs(got[r] - f * (A[r] @ B.T)).max() < 1e-3:
                print(f"   -> matches whole row x{f}")
            A4 = A.copy()
            ks = (kb // 4) * 128
            A4[r, ks:ks + 128] *= f
            if np.abs(got[r] - A4[r] @ B.T).max() < 1e-3:
                print(f"   -> matches whole K-step x{f}")
    # which k does A element (row 0, k) pair with: perturb one byte
    for k in [0, 1, 15, 16, 31, 32, 63, 64, 100, 127, 128]:
        qa2 = qa.copy()
        qa2[0, k] = 0
        A2 = MX.decode_e4m3(qa2)
        got = run(qa2, ones_a, qb, ones_b, M, N, K)
        print(f"zero A[0,{k}]: max err {np.abs(got - A2 @ B.T).max():.3g}")


if __name__ == "__main__":
    main()
