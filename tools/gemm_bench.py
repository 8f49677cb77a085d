"""GEMM micro-benchmark through the C-ABI: TFLOP/s per encoder shape (C2, B=256) and a
square reference shape, for A/B-ing kernel variants (VTD_GEMM_VARIANT) in one process.

  python tools/gemm_bench.py [--variants 0,1] [--reps 20]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_transformer_detector_amd import _lib as L  # noqa: E402

SHAPES = {  # name: (M, N, K, act, out_dtype, resid)
    "qkv": (50176, 2304, 768, 0, 1, False),
    "attn_out": (50176, 768, 768, 0, 1, True),     # bf16 residual stream (the forward's)
    "mlp1": (50176, 3072, 768, 1, 1, False),
    "mlp2": (50176, 1536, 3072, 1, 1, False),
    "mlp3": (50176, 768, 1536, 1, 1, True),
    "head1": (4352, 8704, 256, 1, 1, False),
    "head2": (4352, 4352, 8704, 1, 1, False),
    "sq8192": (8192, 8192, 8192, 0, 1, False),
    # the head's skinny-kernel layers per micro-batch half (B = 128: 2176 rows), padded widths
    "det17": (25088, 17, 768, 0, 1, False),
    "head272": (2176, 320, 576, 1, 1, False),
    "head136": (2176, 192, 320, 1, 1, False),
    "head6": (2176, 6, 192, 0, 0, False),
    # diagnostics: the activation's share of an epilogue (mlp1 / mlp2 without GELU)
    "mlp1_noact": (50176, 3072, 768, 0, 1, False),
    "mlp2_noact": (50176, 1536, 3072, 0, 1, False),
    # the forward's own epilogues: residual layers emitting the next LayerNorm's partial
    # statistics (statout), LayerNorm-folded consumers (lnstat / colsum)
    "attn_out_st": (50176, 768, 768, 0, 1, True),
    "mlp3_st": (50176, 768, 1536, 1, 1, True),
    "qkv_ln": (50176, 2304, 768, 0, 1, False),
    "mlp1_ln": (50176, 3072, 768, 1, 1, False),
    # the micro-batch halves of the two-stream forward (B = 128 each)
    "attn_out_h": (25088, 768, 768, 0, 1, True),
    "mlp3_h": (25088, 768, 1536, 1, 1, True),
    "qkv_h": (25088, 2304, 768, 0, 1, False),
    "mlp1_h": (25088, 3072, 768, 1, 1, False),
    "mlp2_h": (25088, 1536, 3072, 1, 1, False),
}
STATOUT = {"attn_out_st", "mlp3_st"}
LNFOLD = {"qkv_ln", "mlp1_ln"}


def stamp_summary(call, M, N):
    """Diagnostic library, VTD_PP2_DG=16: per-workgroup s_memtime stamps of one launch
    (start, prologue landed, main loop done, epilogue issued; shader clocks) -> mean phase
    lengths and, per XCC, the gap between a workgroup's end and the next start on the XCC."""
    import numpy as np
    fn = L.lib.vtd_diag_read_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    nwg = ((M + 255) // 256) * ((N + 255) // 256)
    call()
    torch.cuda.synchronize()
    buf = np.zeros((nwg, 6), np.uint64)
    assert fn(buf.ctypes.data, nwg) == 0
    t = buf[:, :4].astype(np.int64)
    pro, main, epi = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    r0, r1 = buf[:, 4].astype(np.int64), buf[:, 5].astype(np.int64)   # 100 MHz real time
    clk_ghz = float(np.median((t[:, 3] - t[:, 0]) / np.maximum(r1 - r0, 1))) / 10.0
    span_us = (r1.max() - r0.min()) / 100.0
    busy_us = (r1 - r0).sum() / 100.0
    # running workgroups over time: the mean over the launch span, the share of the span with
    # >= 240 of the 256 CUs busy
    ev = np.concatenate([np.stack([r0, np.ones_like(r0)], 1), np.stack([r1, -np.ones_like(r1)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    run, full, last = 0, 0, ev[0, 0]
    for tt, d in ev:
        if run >= 240:
            full += tt - last
        run += d
        last = tt
    return {"stamp_cycles": {"prologue": int(np.median(pro)), "mainloop": int(np.median(main)),
                             "epilogue": int(np.median(epi)),
                             "tile": int(np.median(t[:, 3] - t[:, 0]))},
            "clock_ghz": round(clk_ghz, 3), "span_us": round(span_us, 1),
            "mean_running_wg": round(busy_us / max(span_us, 1e-9), 1),
            "full_share": round(full / 100.0 / max(span_us, 1e-9), 3),
            "tile_us": round(float(np.median(r1 - r0)) / 100.0, 2)}


def run(name, spec, reps, dev):
    M, N, K, act, od, res = spec
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    Bt = (torch.rand(N, K, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    bias = torch.zeros(N, device=dev)
    out = torch.empty(M, N, device=dev, dtype=torch.float32 if od == 0 else torch.bfloat16)
    e = L.VtdEpilogue()
    e.bias = bias.data_ptr()
    e.act = act
    e.out, e.ldo, e.out_dtype = out.data_ptr(), N, od
    if res:
        e.resid, e.ldr = out.data_ptr(), N
    keep = []
    if name in STATOUT:
        # slot-major planes (stat_ld = M, round 5); VTD_STAT_ROWMAJOR=1 for a library built
        # before (stat_ld = N / 64): the same buffer size either way
        stat = torch.empty(M, N // 64, 2, device=dev)
        keep.append(stat)
        e.statout = stat.data_ptr()
        e.stat_ld = N // 64 if os.environ.get("VTD_STAT_ROWMAJOR") == "1" else M
    if name in LNFOLD:
        lnstat = torch.stack([torch.zeros(M, device=dev), torch.ones(M, device=dev)], 1).contiguous()
        colsum = Bt.float().sum(1).contiguous()
        keep += [lnstat, colsum]
        e.lnstat, e.colsum = lnstat.data_ptr(), colsum.data_ptr()
    st = L.stream_ptr()
    call = lambda: L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K,
                                          L.BF16, ctypes.byref(e), st))
    for _ in range(3):
        call()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        call()
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / reps
    res = {"shape": name, "us": round(ms * 1e3, 1), "tflops": round(2 * M * N * K / ms / 1e9, 1)}
    if os.environ.get("VTD_PP2_DG") == "16":
        res.update(stamp_summary(call, M, N))
    if os.environ.get("VTD_GEMM_SPLIT2"):
        # the same problem as two M-halves on two streams at once (the forward's two-stream
        # micro-batching), and the two halves back to back on one stream
        h = (M // 2 // 256) * 256
        s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
        e1, e2 = L.VtdEpilogue(), L.VtdEpilogue()
        for ee, r0 in ((e1, 0), (e2, h)):
            ee.bias, ee.act, ee.ldo, ee.out_dtype = e.bias, e.act, N, e.out_dtype
            ee.out = out.data_ptr() + r0 * N * out.element_size()
            if res:
                ee.resid, ee.ldr = ee.out, N

        def halves(st_a, st_b):
            for ee, r0, mm, stv in ((e1, 0, h, st_a), (e2, h, M - h, st_b)):
                L.check(L.lib.vtd_gemm(mm, N, K, A.data_ptr() + r0 * K * 2, K, Bt.data_ptr(), K,
                                       L.BF16, ctypes.byref(ee), stv.cuda_stream))
        cur = torch.cuda.current_stream()
        for label, (sa, sb) in (("two_streams", (s1, s2)), ("one_stream", (s1, s1))):
            for _ in range(3):
                halves(sa, sb)
            torch.cuda.synchronize()
            t0.record(cur)
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            for _ in range(reps):
                halves(sa, sb)
            cur.wait_stream(s1)
            cur.wait_stream(s2)
            t1.record(cur)
            torch.cuda.synchronize()
            res["halves_" + label + "_us"] = round(t0.elapsed_time(t1) / reps * 1e3, 1)
    if os.environ.get("VTD_GEMM_REF_LIB"):
        # vendor-library reference (torch.matmul -> hipBLASLt), timing comparison only
        Bk = Bt.t()
        o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(A, Bk, out=o)
        t0.record()
        for _ in range(reps):
            torch.matmul(A, Bk, out=o)
        t1.record()
        torch.cuda.synchronize()
        ms2 = t0.elapsed_time(t1) / reps
        res["vendor_lib_tflops"] = round(2 * M * N * K / ms2 / 1e9, 1)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for name in args.shapes.split(","):
        print(json.dumps({"variant": os.environ.get("VTD_GEMM_VARIANT", "default"),
                          **run(name, SHAPES[name], args.reps, dev)}), flush=True)


if __name__ == "__main__":
    main()
