"""Split-bf16 parity mode (dtype VTD_BF16X3 / "bf16x3"; include/vtd.h "Split-bf16 operands").

An f32 value v is held as hi = bf16(v) (round to nearest even) and lo = bf16(v - hi); a Dense
layer runs as ONE bf16 MFMA GEMM over K' = 3 K on the activation rows stored [hi | lo] and read
as [hi | lo | hi] (A: the K loop returns to column 0 after 2 K) against the weight rows
[hi | hi | lo] (B), i.e. hi.hi + lo.hi + hi.lo summed in fp32 accumulators.  Checks:
  * the split itself is bit-exact against a numpy restatement (split_np below);
  * every producer that writes the split operand directly -- the GEMM epilogues (generic,
    LDS-staged fast, register-direct transposed; the head's Reshape scatter; split-K), the
    LayerNorm kernels, patch extraction -- writes exactly split_np of its f32 result;
  * a split-bf16 GEMM is within 2e-5 of the fp64 product of the f32 operands (the dropped
    lo.lo term is <= 2^-18 of each product).
The whole-forward goldens for this mode are in test_gpu_model.py / test_gpu_batch_parity.py
(tolerance 1e-4)."""
import ctypes
import math

import numpy as np
import pytest
import torch

from oracle import vtd_numpy as ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L(cuda):
    from vision_transformer_detector_amd import _lib
    return _lib


def bf16_rne(x):
    """f32 -> bf16 bits (uint16) by round to nearest even (finite inputs)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def bf16_to_f32(b):
    return (b.astype(np.uint32) << 16).view(np.float32)


def split_np(x, P, role):
    """f32 [rows][K] -> uint16: role 0 [hi | lo] ([rows][2P]), role 1 [hi | hi | lo] ([rows][3P])."""
    x = np.asarray(x, np.float32)
    rows, K = x.shape
    xp = np.zeros((rows, P), np.float32)
    xp[:, :K] = x
    hi = bf16_rne(xp)
    lo = bf16_rne(xp - bf16_to_f32(hi))
    return np.concatenate([hi, lo] if role == 0 else [hi, hi, lo], axis=1)


def as_u16(t):
    return t.cpu().view(torch.int16).numpy().view(np.uint16)


def split_dev(L, x, P, role):
    rows, K = x.shape
    w = (3 if role else 2) * P
    y = torch.full((rows, w), -1, dtype=torch.int16, device=x.device)
    L.check(L.lib.vtd_split_bf16x3(x.data_ptr(), rows, K, x.shape[1], y.data_ptr(), w, role,
                                   L.stream_ptr()), "split")
    torch.cuda.synchronize()
    return y.view(torch.bfloat16)


@pytest.mark.parametrize("rows,K,P", [(5, 64, 64), (33, 100, 128), (7, 13, 24), (256, 768, 768)])
@pytest.mark.parametrize("role", [0, 1])
def test_split_bit_exact(L, cuda, rows, K, P, role):
    g = torch.Generator().manual_seed(rows + K + role)
    x = torch.randn(rows, K, generator=g) * torch.logspace(-6, 6, K)    # wide exponent range
    x[0, :min(K, 4)] = torch.tensor([0.0, -0.0, 1e-30, -3.0e38])[:min(K, 4)]
    y = split_dev(L, x.to(cuda), P, role)
    assert np.array_equal(as_u16(y), split_np(x.numpy(), P, role))


def _epi(L, out, ldo, out_dtype, bias=None, act=0, scatter=0, resid=None):
    e = L.VtdEpilogue()
    e.bias, e.act = L.ptr(bias), act
    e.out, e.ldo, e.out_dtype = L.ptr(out), ldo, out_dtype
    e.scatter_tokens = scatter
    e.resid = L.ptr(resid)
    e.ldr = resid.shape[1] if resid is not None else 0
    return e


def _gemm_x3(L, A32, W32, N=None, **kw):
    """split-bf16 GEMM of f32 operands A [M][K], W^T [N][K] (K % 64 == 0)."""
    M, K = A32.shape
    a3 = split_dev(L, A32, K, 0)
    b3 = split_dev(L, W32, K, 1)
    return a3, b3


@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (300, 200, 192), (1024, 768, 768),
                                   (8192, 1024, 256), (512, 17, 256), (300, 512, 192),
                                   (2048, 2048, 3072), (2176, 2176, 1088), (588, 17, 768),
                                   (200, 300, 1024)])
def test_split_gemm_vs_fp64(L, cuda, M, N, K):
    """A split-bf16 GEMM (dtype VTD_BF16X3: bf16 kernels over K' = 3K, A read with the wrap --
    the 256-tile pp2 kernel for the larger shapes, the 128-tile kernel (1024 x 768, 300 x 512)
    and the skinny kernel for the narrow ones, which stages only the [hi | lo] columns of the
    weights: the head's Dense(17) at K = 768, N = 300 at K = 1024 -- 2048 staged columns, its
    LDS limit) against the fp64 product of the f32 operands;
    where the forward would split K (vtd_gemm_splitk_choice), the split-K form too, whose
    ranges start before, across and past the wrap (2176 x 2176 x 1088: 4 x 13 K-steps, wrap
    at 34)."""
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / math.sqrt(K)
    a3, b3 = _gemm_x3(L, A.to(cuda), W.to(cuda))
    ref64 = A.double() @ W.double().T
    out = torch.full((M, N), float("nan"), device=cuda)
    e = _epi(L, out, N, L.F32)
    L.check(L.lib.vtd_gemm(M, N, 3 * K, a3.data_ptr(), 2 * K, b3.data_ptr(), 3 * K, L.BF16X3,
                           ctypes.byref(e), L.stream_ptr()), "gemm")
    ks = L.lib.vtd_gemm_splitk_choice(M, N, 3 * K, L.BF16X3)
    outs = [out]
    if ks > 1:
        out2 = torch.full((M, N), float("nan"), device=cuda)
        e2 = _epi(L, out2, N, L.F32)
        part = torch.empty(ks * M * N, device=cuda)
        L.check(L.lib.vtd_gemm_splitk(M, N, 3 * K, a3.data_ptr(), 2 * K, b3.data_ptr(), 3 * K,
                                      L.BF16X3, ctypes.byref(e2), part.data_ptr(),
                                      part.numel() * 4, ks, L.stream_ptr()), "splitk")
        outs.append(out2)
    torch.cuda.synchronize()
    for o in outs:
        err = (o.cpu().double() - ref64).abs().max().item()
        assert err <= 2e-5 * ref64.abs().max().item(), (len(outs), err)


@pytest.mark.parametrize("M,N,K,act", [(8192, 1024, 256, 0), (4096, 3072, 256, 1),
                                       (8000, 1024, 256, 2), (512, 1536, 256, 2),
                                       (300, 200, 192, 1), (64, 6, 128, 0),
                                       (4352, 1088, 2176, 1)])
def test_split_output_equals_split_of_f32_output(L, cuda, M, N, K, act):
    """out_dtype VTD_BF16X3 (EPI_S3 on the fast pp2 epilogues, the generic epilogue on partial
    tiles and small problems, split-K for the head's few-tile long-K shape) writes exactly
    split_np of the same GEMM's f32 output (same accumulators, same bias / activation)."""
    g = torch.Generator().manual_seed(N + act)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).to(cuda)
    W = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(torch.bfloat16).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    f32 = torch.empty(M, N, device=cuda)
    P = ((N + 63) // 64) * 64
    s3 = torch.full((M, 2 * P), -1, dtype=torch.int16, device=cuda)
    for out, ldo, od in ((f32, N, L.F32), (s3, 2 * P, L.BF16X3)):
        e = _epi(L, out, ldo, od, bias=bias, act=act)
        ks = L.lib.vtd_gemm_splitk_choice(M, N, K, L.BF16)
        if ks > 1:
            part = torch.empty(ks * M * N, device=cuda)
            L.check(L.lib.vtd_gemm_splitk(M, N, K, A.data_ptr(), K, W.data_ptr(), K, L.BF16,
                                          ctypes.byref(e), part.data_ptr(), part.numel() * 4, ks,
                                          L.stream_ptr()), "splitk")
        else:
            L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, W.data_ptr(), K, L.BF16,
                                   ctypes.byref(e), L.stream_ptr()), "gemm")
    torch.cuda.synchronize()
    v = f32.cpu().numpy()
    want = split_np(v, P, 0)
    got = as_u16(s3)
    # columns [N, P) of each piece are not written
    if N < P:
        assert (got[:, N:P] == 0xFFFF).all() and (got[:, P + N:] == 0xFFFF).all()
    if act == 0:
        for piece in range(2):
            sl = slice(piece * P, piece * P + N)
            assert np.array_equal(got[:, sl], want[:, sl]), piece
    else:
        # the activation's f32 arithmetic may be contracted differently in the two kernel
        # instantiations (a few f32 ulps), which the lo piece shows: compare hi + lo with the
        # f32 output at the split's own precision (2^-17 relative)
        recon = bf16_to_f32(got[:, :N]).astype(np.float64) + bf16_to_f32(got[:, P:P + N])
        err = np.abs(recon - v) / np.maximum(np.abs(v), 1e-30)
        assert err.max() <= 2 ** -16, err.max()
        assert (got[:, :N] != want[:, :N]).mean() < 1e-3


def test_split_scatter_epilogue(L, cuda):
    """The head's Dense(17) + Reshape scatter (vtd.py:454-463) with a split-bf16 output."""
    B, T, K = 3, 196, 768
    g = torch.Generator().manual_seed(17)
    A = torch.randn(B * T, K, generator=g).to(torch.bfloat16).to(cuda)
    W = (torch.randn(17, K, generator=g) / math.sqrt(K)).to(torch.bfloat16).to(cuda)
    bias = torch.randn(17, generator=g).to(cuda)
    P = 256
    f32 = torch.zeros(B * 17, P, device=cuda)
    s3 = torch.zeros(B * 17, 2 * P, dtype=torch.int16, device=cuda)
    for out, ldo, od in ((f32, P, L.F32), (s3, 2 * P, L.BF16X3)):
        e = _epi(L, out, ldo, od, bias=bias, scatter=T)
        L.check(L.lib.vtd_gemm(B * T, 17, K, A.data_ptr(), K, W.data_ptr(), K, L.BF16,
                               ctypes.byref(e), L.stream_ptr()), "gemm")
    torch.cuda.synchronize()
    assert np.array_equal(as_u16(s3), split_np(f32.cpu().numpy(), P, 0))


@pytest.mark.parametrize("rows,D,P", [(300, 768, 768), (77, 28, 64), (64, 1024, 1024),
                                      (9, 100, 128), (9, 30, 64)])
@pytest.mark.parametrize("xdt", ["f32", "bf16"])
def test_layernorm_split_output(L, cuda, rows, D, P, xdt):
    """vtd_layernorm with dtype VTD_BF16X3 = split_np of its f32 output (the 16-column, the
    4-column and the generic kernels)."""
    g = torch.Generator().manual_seed(rows + D)
    x = (torch.randn(rows, P, generator=g) * 3 + 1)
    x[:, D:] = 0
    tdt, code = (torch.float32, L.F32) if xdt == "f32" else (torch.bfloat16, L.BF16)
    x = x.to(tdt).to(cuda)
    gamma = (1 + 0.1 * torch.randn(P, generator=g)).to(cuda)
    beta = (0.1 * torch.randn(P, generator=g)).to(cuda)
    f32 = torch.empty(rows, P, device=cuda)
    s3 = torch.full((rows, 2 * P), -1, dtype=torch.int16, device=cuda)
    for out, ldy, od in ((f32, P, L.F32), (s3, 2 * P, L.BF16X3)):
        L.check(L.lib.vtd_layernorm(x.data_ptr(), code, rows, D, P, gamma.data_ptr(),
                                    beta.data_ptr(), 1e-3, out.data_ptr(), ldy, od,
                                    L.stream_ptr()), "layernorm")
    torch.cuda.synchronize()
    assert np.array_equal(as_u16(s3), split_np(f32.cpu().numpy(), P, 0))


@pytest.mark.parametrize("H,W,p,P", [(224, 224, 16, 768), (40, 36, 8, 192), (608, 608, 17, 896)])
def test_patches_split_output(L, cuda, H, W, p, P):
    g = torch.Generator().manual_seed(H + p)
    img = (torch.rand(2, H, W, 3, generator=g) * 2 - 1).to(cuda)
    gh, gw = -(-H // p), -(-W // p)
    rows = 2 * gh * gw
    f32 = torch.empty(rows, P, device=cuda)
    s3 = torch.full((rows, 2 * P), -1, dtype=torch.int16, device=cuda)
    for out, ldo, od in ((f32, P, L.F32), (s3, 2 * P, L.BF16X3)):
        L.check(L.lib.vtd_extract_patches(img.data_ptr(), 2, H, W, 3, p, out.data_ptr(), ldo, od,
                                          L.stream_ptr()), "patches")
    torch.cuda.synchronize()
    assert np.array_equal(as_u16(s3), split_np(f32.cpu().numpy(), P, 0))
    want = ref.extract_patches_same(img.cpu().numpy().astype(np.float64), p).reshape(rows, -1)
    assert np.array_equal(f32.cpu().numpy()[:, :want.shape[1]], want.astype(np.float32))


def test_split_arguments_validated(L, cuda):
    x = torch.zeros(4, 64, device=cuda)
    y = torch.zeros(4, 192, dtype=torch.int16, device=cuda)
    split = L.lib.vtd_split_bf16x3
    assert split(x.data_ptr(), 4, 64, 64, y.data_ptr(), 129, 0, None) == -1   # 2 P, odd
    assert split(x.data_ptr(), 4, 64, 64, y.data_ptr(), 120, 0, None) == -1   # P < K
    assert split(x.data_ptr(), 4, 64, 64, y.data_ptr(), 190, 1, None) == -1   # 3 P
    assert split(x.data_ptr(), 4, 64, 64, y.data_ptr(), 180, 1, None) == -1   # P < K
    assert split(x.data_ptr(), 4, 64, 64, y.data_ptr(), 192, 2, None) == -1   # role
    out = torch.zeros(4, 192, dtype=torch.int16, device=cuda)
    e = _epi(L, out, 191, L.BF16X3)
    assert L.lib.vtd_gemm(4, 64, 64, x.data_ptr(), 64, x.data_ptr(), 64, L.BF16, ctypes.byref(e),
                          None) == -1            # split output: ldo % 2
    e = _epi(L, out, 192, L.BF16X3)
    assert L.lib.vtd_gemm(4, 64, 64, x.data_ptr(), 64, x.data_ptr(), 64, L.F32, ctypes.byref(e),
                          None) == -1            # split output needs bf16 operands
    f = torch.zeros(4, 64, device=cuda)
    e = _epi(L, f, 64, L.F32)
    gemm = L.lib.vtd_gemm
    assert gemm(4, 64, 128, x.data_ptr(), 128, x.data_ptr(), 128, L.BF16X3, ctypes.byref(e),
                None) == -1                      # split A: K = 3 P
    assert gemm(4, 64, 192, x.data_ptr(), 120, x.data_ptr(), 192, L.BF16X3, ctypes.byref(e),
                None) == -1                      # split A: lda >= 2 P


def _attn_ref64(qkv, B, N, H, dk, dkp):
    q = qkv[:, :H * dkp].reshape(B, N, H, dkp)[..., :dk]
    k = qkv[:, H * dkp:2 * H * dkp].reshape(B, N, H, dkp)[..., :dk]
    v = qkv[:, 2 * H * dkp:3 * H * dkp].reshape(B, N, H, dkp)[..., :dk]
    s = np.einsum("bqhd,bkhd->bhqk", q, k) / math.sqrt(dk)
    p = ref.softmax(s, axis=-1)
    return np.einsum("bhqk,bkhd->bqhd", p, v)


@pytest.mark.parametrize("B,N,H,dk", [(2, 196, 3, 64), (1, 70, 2, 40), (1, 1, 1, 32),
                                      (1, 333, 2, 128), (2, 1600, 2, 64), (3, 576, 3, 64),
                                      (40, 196, 12, 64), (1, 64, 4, 20), (1, 129, 2, 100),
                                      (2, 17, 3, 64), (1, 1, 2, 64), (3, 33, 2, 64)])
@pytest.mark.parametrize("variant", [-1, 10])
def test_attention_split_vs_fp64(L, cuda, B, N, H, dk, variant):
    """vtd_attention with dtype VTD_BF16X3 (vtd.py:364-369 in the split-bf16 parity mode): f32
    query / key / value in, every product as hi.hi + lo.hi + hi.lo on the bf16 MFMA with fp32
    softmax statistics, the output written as the attention-output Dense's split-bf16 A operand
    [hi | lo].  hi + lo against the fp64 attention of the same f32 inputs: within 2e-5
    of max |O| (the f32 kernel's bound in test_gpu_kernels.test_attention)."""
    dkp = 32 if dk <= 32 else (64 if dk <= 64 else 128)
    ld = 3 * H * dkp + 8
    g = np.random.default_rng(N * 10 + dk)
    qkv = np.zeros((B * N, ld), np.float32)
    for part in range(3):
        for h in range(H):
            c0 = part * H * dkp + h * dkp
            qkv[:, c0:c0 + dk] = g.normal(0, 1.5, size=(B * N, dk))
    P = H * dkp + 64
    out = torch.full((B * N, 2 * P), -1, dtype=torch.int16, device=cuda)
    qkv_d = torch.from_numpy(qkv).to(cuda)
    if variant == 10 and dkp != 64:
        pytest.skip("knob 10 (64-key chunks, one workgroup per CU) is a dkp-64 variant")
    with L.knob(L.KNOB_ATTN_VARIANT, variant):
        L.check(L.lib.vtd_attention(qkv_d.data_ptr(), B, N, H, dkp, ld, 1.0 / math.sqrt(dk),
                                    out.data_ptr(), 2 * P, L.BF16X3, L.stream_ptr()), "attention")
    torch.cuda.synchronize()
    got = as_u16(out)
    inner = H * dkp
    assert (got[:, inner:P] == 0xFFFF).all()                              # not written
    assert (got[:, P + inner:] == 0xFFFF).all()
    hi = bf16_to_f32(got[:, :inner]).astype(np.float64)
    lo = bf16_to_f32(got[:, P:P + inner]).astype(np.float64)
    # the lo piece is the split of the f32 value hi + lo: |lo| <= half an ulp of bf16(hi)
    assert (np.abs(lo) <= np.abs(hi) * 2.0 ** -7 + 1e-38).all()
    o = (hi + lo).reshape(B, N, H, dkp)
    exp = _attn_ref64(qkv.astype(np.float64), B, N, H, dk, dkp)
    assert np.abs(o[..., :dk] - exp).max() < 2e-5 * max(1.0, np.abs(exp).max())
    assert (o[..., dk:] == 0).all()


def test_attention_split_arguments_validated(L, cuda):
    x = torch.zeros(196, 3 * 64, device=cuda)
    y = torch.zeros(196, 2 * 64 + 1, dtype=torch.int16, device=cuda)
    assert L.lib.vtd_attention(x.data_ptr(), 1, 196, 1, 64, 192, 0.125, y.data_ptr(), 129,
                               L.BF16X3, None) == -1        # ldo % 2 != 0
    assert L.lib.vtd_attention(x.data_ptr(), 1, 196, 1, 64, 192, 0.125, y.data_ptr(), 96,
                               L.BF16X3, None) == -1        # piece narrower than heads * dkp
