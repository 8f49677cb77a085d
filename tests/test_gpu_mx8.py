"""MX-fp8 path of the VTD_FP8 mode on the GPU, through the C-ABI:
  - vtd_quantize_mx8 against the CPU restatement oracle/mx8.py, element for element
    (e4m3 values and E8M0 block exponents must be identical);
  - vtd_gemm_mx8 against the fp64 product of the DEQUANTIZED device operands, so the
    check isolates the block-scaled MFMA + fp32 accumulation + epilogue; the 8-wave
    ping-pong kernel (and, with the diagnostic library, VTD_MX_VARIANT 2 = x4, one wave per
    SIMD).  Tolerance
    5e-4 relative for f32 outputs: the instruction reduces each 128-element K-step
    inside the matrix core before the fp32 accumulate (measured max 1.1e-4 at K <= 1536,
    6x the 2e-5 of the bf16 MFMA's exact fp32 fma chain); 8e-3 for bf16 outputs.
"""
import ctypes
import math

import numpy as np
import pytest
import torch

from oracle import mx8 as MX
from oracle import vtd_numpy as ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L(cuda):
    from vision_transformer_detector_amd import _lib
    return _lib


def _need_variant(L, variant):
    """VTD_MX_VARIANT 2 / 3 (the x4 kernel) exist in the diagnostic library only."""
    if variant != "1" and not hasattr(L.lib, "vtd_diag_build"):
        pytest.skip("the x4 kernel is in the diagnostic build only (make diag)")


def _quantize(L, x, Kq, s_rows=None):
    rows, K = x.shape
    s_rows = s_rows or -(-rows // 4) * 4
    q = torch.full((rows, Kq), 0x7f, dtype=torch.uint8, device=x.device)
    s = torch.full((Kq // 128 * s_rows * 4,), 0xff, dtype=torch.uint8, device=x.device)
    dt = L.BF16 if x.dtype == torch.bfloat16 else L.F32
    L.check(L.lib.vtd_quantize_mx8(x.data_ptr(), dt, rows, K, x.shape[1], Kq, q.data_ptr(),
                                   Kq, s.data_ptr(), s_rows, L.stream_ptr()), "quantize_mx8")
    torch.cuda.synchronize()
    return q, s, s_rows


@pytest.mark.parametrize("rows,K,Kq,src", [(64, 256, 256, "bf16"), (37, 200, 256, "bf16"),
                                           (129, 768, 768, "f32"), (5, 96, 128, "f32")])
def test_quantize_matches_oracle(L, cuda, rows, K, Kq, src):
    g = torch.Generator(device=cuda).manual_seed(rows * K)
    x = torch.randn(rows, K, generator=g, device=cuda)
    # blocks spanning many binades: per-row magnitudes 2^-20 .. 2^20, one zero row
    x = x * torch.exp2(torch.linspace(-20, 20, rows, device=cuda))[:, None]
    x[rows // 2] = 0
    x = x.to(torch.bfloat16) if src == "bf16" else x
    q, s, s_rows = _quantize(L, x, Kq)
    vals, E = MX.quantize(x.float().cpu().numpy(), Kq)
    got = MX.decode_e4m3(q.cpu().numpy())
    np.testing.assert_array_equal(got, vals)
    s_np = s.cpu().numpy().reshape(Kq // 128, s_rows, 4)[:, :rows]
    np.testing.assert_array_equal(s_np.transpose(1, 0, 2).reshape(rows, -1).astype(int) - 127, E)
    deq = MX.dequantize(q.cpu().numpy(), s.cpu().numpy(), rows, Kq)
    xf = np.zeros((rows, Kq))
    xf[:, :K] = x.float().cpu().numpy()
    # e4m3 relative step 2^-3 -> |err| <= 2^-4 |x| (normal range of the block)
    blk = np.abs(xf).reshape(rows, -1, 32).max(axis=2, keepdims=True)
    err = np.abs(deq - xf).reshape(rows, -1, 32)
    assert np.all(err <= np.maximum(np.abs(xf.reshape(rows, -1, 32)) / 16, blk * 2.0 ** -9 + 1e-300))


@pytest.mark.parametrize("M,N,K,act,out_dtype,resid", [
    (300, 200, 256, 0, 0, False), (1000, 520, 384, 1, 1, False),
    (4096, 1024, 1024, 1, 1, False), (2600, 776, 1536, 0, 0, True),
    (513, 64, 128, 2, 0, False), (4096, 768, 1536, 1, 1, True), (1000, 520, 384, 0, 1, True),
    (2304, 1280, 640, 2, 1, False)])
@pytest.mark.parametrize("variant", ["1", "2"])
def test_gemm_mx8_matches_dequantized_fp64(L, cuda, monkeypatch, variant, M, N, K, act,
                                           out_dtype, resid):
    _need_variant(L, variant)
    monkeypatch.setenv("VTD_MX_VARIANT", variant)
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    W = torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)
    qa, sa, sa_rows = _quantize(L, A, K)
    qb, sb, sb_rows = _quantize(L, W, K)
    bias = torch.randn(N, generator=g, device=cuda)
    res = torch.randn(M, N, generator=g, device=cuda) if resid else None
    if resid and out_dtype == 1:
        res = res.to(torch.bfloat16)                # resid is read in the output's dtype
    out = torch.full((M, N), float("nan"), device=cuda,
                     dtype=torch.float32 if out_dtype == 0 else torch.bfloat16)
    e = L.VtdEpilogue()
    e.bias, e.act = bias.data_ptr(), act
    e.resid, e.ldr = (res.data_ptr(), N) if resid else (None, 0)
    e.out, e.ldo, e.out_dtype = out.data_ptr(), N, out_dtype
    L.check(L.lib.vtd_gemm_mx8(M, N, K, qa.data_ptr(), K, sa.data_ptr(), sa_rows, qb.data_ptr(),
                               K, sb.data_ptr(), sb_rows, ctypes.byref(e), L.stream_ptr()),
            "gemm_mx8")
    torch.cuda.synchronize()
    a64 = MX.dequantize(qa.cpu().numpy(), sa.cpu().numpy(), M, K)
    b64 = MX.dequantize(qb.cpu().numpy(), sb.cpu().numpy(), N, K)
    ref64 = a64 @ b64.T + bias.double().cpu().numpy()
    ref64 = {0: lambda v: v, 1: ref.gelu_tanh, 2: ref.mish}[act](ref64)
    if resid:
        ref64 = ref64 + res.double().cpu().numpy()
    got = out.double().cpu().numpy()
    tol = 5e-4 if out_dtype == 0 else 8e-3
    err = np.abs(got - ref64) / np.maximum(np.abs(ref64), 1.0)
    assert err.max() < tol, (err.max(), np.argwhere(err >= tol)[:5].tolist())


@pytest.mark.parametrize("rows,D,x_dtype", [(200, 768, "bf16"), (64, 1024, "f32"), (37, 96, "bf16"),
                                             (50, 104, "bf16"), (21, 2048, "bf16"),
                                             (9, 4000, "f32")])
def test_layernorm_mx8_equals_layernorm_then_quantize(L, cuda, rows, D, x_dtype):
    """The fused LayerNorm -> MX-fp8 pass writes exactly the bytes of vtd_layernorm (bf16 out)
    followed by vtd_quantize_mx8: the 16-columns-per-lane pair (D % 16 == 0) and the 4-column
    pair (D = 104)."""
    g = torch.Generator(device=cuda).manual_seed(rows + D)
    xdt = torch.bfloat16 if x_dtype == "bf16" else torch.float32
    x = (torch.randn(rows, D, generator=g, device=cuda) * 3 + 1).to(xdt)
    gamma = 1 + 0.2 * torch.randn(D, generator=g, device=cuda)
    beta = 0.3 * torch.randn(D, generator=g, device=cuda)
    xc = L.BF16 if x_dtype == "bf16" else L.F32
    Kq = -(-D // 128) * 128
    h = torch.zeros(rows, D, device=cuda, dtype=torch.bfloat16)
    L.check(L.lib.vtd_layernorm(x.data_ptr(), xc, rows, D, D, gamma.data_ptr(), beta.data_ptr(),
                                1e-3, h.data_ptr(), D, L.BF16, L.stream_ptr()), "ln")
    q_ref, s_ref, s_rows = _quantize(L, h, Kq)
    q = torch.full((rows, Kq), 0x7f, dtype=torch.uint8, device=cuda)
    s = torch.full_like(s_ref, 0xff)
    L.check(L.lib.vtd_layernorm_mx8(x.data_ptr(), xc, rows, D, D, gamma.data_ptr(),
                                    beta.data_ptr(), 1e-3, q.data_ptr(), Kq, Kq, s.data_ptr(),
                                    s_rows, L.stream_ptr()), "ln_mx8")
    torch.cuda.synchronize()
    assert torch.equal(q, q_ref)
    s_ref_v = s_ref.view(Kq // 128, s_rows, 4)[:, :rows]
    assert torch.equal(s.view(Kq // 128, s_rows, 4)[:, :rows], s_ref_v)


@pytest.mark.parametrize("M,N,K,act", [(4096, 1024, 1024, 1), (2560, 512, 384, 0),
                                       (1536, 2048, 768, 2)])
@pytest.mark.parametrize("variant", ["1", "2"])
def test_gemm_mx8_fp8_output_equals_quantized_bf16_output(L, cuda, monkeypatch, variant, M, N,
                                                          K, act):
    """out_dtype VTD_FP8 (the next MX GEMM's operand written by the epilogue) equals the bf16
    output of the same GEMM passed through vtd_quantize_mx8, byte for byte."""
    _need_variant(L, variant)
    monkeypatch.setenv("VTD_MX_VARIANT", variant)
    g = torch.Generator(device=cuda).manual_seed(M + N + K + 7)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    W = torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)
    qa, sa, sa_rows = _quantize(L, A, K)
    qb, sb, sb_rows = _quantize(L, W, K)
    bias = torch.randn(N, generator=g, device=cuda)
    out = torch.zeros(M, N, device=cuda, dtype=torch.bfloat16)

    def run(e):
        L.check(L.lib.vtd_gemm_mx8(M, N, K, qa.data_ptr(), K, sa.data_ptr(), sa_rows,
                                   qb.data_ptr(), K, sb.data_ptr(), sb_rows, ctypes.byref(e),
                                   L.stream_ptr()), "gemm_mx8")

    e = L.VtdEpilogue()
    e.bias, e.act, e.out, e.ldo, e.out_dtype = bias.data_ptr(), act, out.data_ptr(), N, 1
    run(e)
    q_ref, s_ref, s_rows = _quantize(L, out, N)
    q = torch.full((M, N), 0x7f, dtype=torch.uint8, device=cuda)
    s = torch.full_like(s_ref, 0xff)
    e2 = L.VtdEpilogue()
    e2.bias, e2.act, e2.out, e2.ldo, e2.out_dtype = bias.data_ptr(), act, q.data_ptr(), N, 2
    e2.scale_out, e2.scale_rows = s.data_ptr(), s_rows
    run(e2)
    torch.cuda.synchronize()
    assert torch.equal(q, q_ref)
    assert torch.equal(s, s_ref)


@pytest.mark.parametrize("M,N,K,act,resid", [(4096, 1024, 1024, 0, False),
                                              (2048, 768, 1536, 1, True),
                                              (777, 300, 384, 2, False)])
def test_gemm_mx8_x4_equals_pingpong(L, cuda, monkeypatch, M, N, K, act, resid):
    """The two MX kernels compute each output as the same sequence of 128-wide scaled MFMA
    K-steps accumulated in fp32 in K order (x4 with the operands swapped: D^T = B A^T), so
    their outputs agree bit for bit (x4: the diagnostic library only)."""
    _need_variant(L, "2")
    g = torch.Generator(device=cuda).manual_seed(M * 3 + N + K)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    W = torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)
    qa, sa, sa_rows = _quantize(L, A, K)
    qb, sb, sb_rows = _quantize(L, W, K)
    bias = torch.randn(N, generator=g, device=cuda)
    res = torch.randn(M, N, generator=g, device=cuda).to(torch.bfloat16) if resid else None
    outs = []
    for variant in ("1", "2"):
        monkeypatch.setenv("VTD_MX_VARIANT", variant)
        out = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
        e = L.VtdEpilogue()
        e.bias, e.act, e.out, e.ldo, e.out_dtype = bias.data_ptr(), act, out.data_ptr(), N, 1
        e.resid, e.ldr = (res.data_ptr(), N) if resid else (None, 0)
        L.check(L.lib.vtd_gemm_mx8(M, N, K, qa.data_ptr(), K, sa.data_ptr(), sa_rows,
                                   qb.data_ptr(), K, sb.data_ptr(), sb_rows, ctypes.byref(e),
                                   L.stream_ptr()), "gemm_mx8")
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), (outs[0].float() - outs[1].float()).abs().max().item()


@pytest.mark.parametrize("B,N,H,dkp", [(2, 196, 12, 64), (1, 576, 16, 64), (3, 100, 4, 32),
                                       (1, 70, 2, 128), (2, 1600, 4, 64)])
def test_attention_mx8_equals_attention_then_quantize(L, cuda, monkeypatch, B, N, H, dkp):
    """The attention kernel's MX-fp8 epilogue (the VTD_FP8 attention-output operand) writes
    exactly the bytes of vtd_attention (bf16 out) followed by vtd_quantize_mx8.  The MX
    epilogue rides on the streaming (per-(image, head)) kernel, so the bf16 reference is that
    kernel too (knob VTD_KNOB_ATTN_VARIANT 2: at N = 196 the default bf16 path is the persistent kernel,
    whose one-pass softmax rounds P differently)."""
    prev = L.lib.vtd_set_knob(L.KNOB_ATTN_VARIANT, 2)
    try:
        _attention_mx8_case(L, cuda, B, N, H, dkp)
    finally:
        L.lib.vtd_set_knob(L.KNOB_ATTN_VARIANT, prev)


def _attention_mx8_case(L, cuda, B, N, H, dkp):
    g = torch.Generator(device=cuda).manual_seed(B * N + H)
    ld = 3 * H * dkp
    qkv = (torch.randn(B * N, ld, generator=g, device=cuda) * 1.5).to(torch.bfloat16)
    inner, rows = H * dkp, B * N
    scale = 1.0 / math.sqrt(dkp)
    o = torch.zeros(rows, inner, device=cuda, dtype=torch.bfloat16)
    L.check(L.lib.vtd_attention(qkv.data_ptr(), B, N, H, dkp, ld, scale, o.data_ptr(), inner,
                                L.BF16, L.stream_ptr()), "attention")
    q_ref, s_ref, s_rows = _quantize(L, o, inner)
    q = torch.full((rows, inner), 0x7f, dtype=torch.uint8, device=cuda)
    s = torch.full_like(s_ref, 0xff)
    L.check(L.lib.vtd_attention_mx8(qkv.data_ptr(), B, N, H, dkp, ld, scale, q.data_ptr(), inner,
                                    s.data_ptr(), s_rows, L.stream_ptr()), "attention_mx8")
    torch.cuda.synchronize()
    assert torch.equal(q, q_ref)
    v = s.view(inner // 128, s_rows, 4)[:, :rows]
    assert torch.equal(v, s_ref.view(inner // 128, s_rows, 4)[:, :rows])


@pytest.mark.parametrize("M,N,K,act,out_dtype,resid", [
    (4096, 1024, 1024, 1, 2, False), (1536, 2048, 768, 2, 2, False), (2304, 1280, 640, 2, 1, False),
    (4096, 768, 1536, 1, 1, True), (1000, 520, 384, 1, 0, False)])
def test_gemm_mx8_transposed_equals_staged(L, cuda, M, N, K, act, out_dtype, resid):
    """Activation layers without a residual take the transposed-accumulator MX kernel
    (operands swapped in the scaled MFMA, permuted B rows with their scales, register-direct
    epilogue incl. the MX-fp8 output); knob VTD_KNOB_GEMM_TR = 0 keeps the staged epilogue
    (the residual case checks the knob is harmless where no transposed kernel exists).  The same products in the
    same order: the outputs (and the MX-fp8 scales) are identical."""
    g = torch.Generator(device=cuda).manual_seed(M + N + K + 11)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    W = torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)
    qa, sa, sa_rows = _quantize(L, A, K)
    qb, sb, sb_rows = _quantize(L, W, K)
    bias = torch.randn(N, generator=g, device=cuda)
    res0 = torch.randn(M, N, generator=g, device=cuda).to(
        torch.float32 if out_dtype == 0 else torch.bfloat16)

    def run():
        if out_dtype == 2:
            out = torch.full((M, N), 0x7f, dtype=torch.uint8, device=cuda)
            s = torch.full((N // 128 * sa_rows * 4,), 0xff, dtype=torch.uint8, device=cuda)
        else:
            out = res0.clone() if resid else torch.zeros_like(res0)
            s = None
        e = L.VtdEpilogue()
        e.bias, e.act, e.out, e.ldo, e.out_dtype = bias.data_ptr(), act, out.data_ptr(), N, out_dtype
        if resid:
            e.resid, e.ldr = out.data_ptr(), N
        if s is not None:
            e.scale_out, e.scale_rows = s.data_ptr(), sa_rows
        L.check(L.lib.vtd_gemm_mx8(M, N, K, qa.data_ptr(), K, sa.data_ptr(), sa_rows,
                                   qb.data_ptr(), K, sb.data_ptr(), sb_rows, ctypes.byref(e),
                                   L.stream_ptr()), "gemm_mx8")
        torch.cuda.synchronize()
        return out, s

    got, gs = run()
    with L.knob(L.KNOB_GEMM_TR, 0):
        ref_out, rs = run()
    assert torch.equal(got, ref_out)
    if gs is not None:
        assert torch.equal(gs, rs)
