"""Per-kernel parity on the GPU, through the C-ABI (include/vtd.h).

Each HIP kernel is compared with the fp64 oracle op it replaces (oracle/vtd_numpy.py)
or a plain fp64 torch restatement of the same op, on seeded inputs.  bf16 operands are
rounded to bf16 BEFORE the reference runs, so GEMM checks measure accumulation error
only.  Tolerances are written per test.
"""
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


def _dt(L, name):
    return {"f32": (L.F32, torch.float32), "bf16": (L.BF16, torch.bfloat16)}[name]


def _gemm(L, A, Bt, dtype, N=None, bias=None, rowadd=None, rowadd_period=1,
          rowadd_ncols=0, act=0, resid=None, out=None, out_dtype=0, out2=None,
          scatter_tokens=0, ldo=None):
    M, K = A.shape
    N = N if N is not None else Bt.shape[0]
    e = L.VtdEpilogue()
    e.bias = L.ptr(bias)
    e.rowadd = L.ptr(rowadd)
    e.rowadd_period, e.rowadd_ncols = rowadd_period, rowadd_ncols
    e.act = act
    e.resid = L.ptr(resid)
    e.ldr = resid.shape[1] if resid is not None else 0
    e.out = L.ptr(out)
    e.ldo = ldo if ldo is not None else out.shape[-1]
    e.out_dtype = out_dtype
    e.out2 = L.ptr(out2)
    e.ldo2 = out2.shape[1] if out2 is not None else 0
    e.scatter_tokens = scatter_tokens
    L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), A.shape[1], Bt.data_ptr(), Bt.shape[1],
                           dtype, ctypes.byref(e), L.stream_ptr()), "vtd_gemm")
    torch.cuda.synchronize()


def _np_act(act, x):
    return {0: lambda v: v, 1: ref.gelu_tanh, 2: ref.mish}[act](x)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (300, 200, 192), (1, 17, 64),
                                   (515, 770, 128), (64, 6, 256)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_gemm_bias_act(L, cuda, dtype, M, N, K, act):
    code, tdt = _dt(L, dtype)
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K + act)
    A = torch.randn(M, K, generator=g).to(tdt)
    Bt = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(tdt)
    bias = torch.randn(N, generator=g)
    ref64 = A.double() @ Bt.double().T + bias.double()
    ref64 = torch.from_numpy(_np_act(act, ref64.numpy()))
    out = torch.full((M, N), float("nan"), device=cuda)
    _gemm(L, A.to(cuda), Bt.to(cuda), code, bias=bias.to(cuda), act=act, out=out)
    err = (out.cpu().double() - ref64).abs().max().item()
    # f32: exact fp32 fma chain, <= ~1e-6 relative to the row norms; bf16 inputs are
    # exact in fp32, so only accumulation order differs.
    assert err <= 2e-5 * max(1.0, ref64.abs().max().item()), err


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_gemm_epilogue_rowadd_resid_out2(L, cuda, dtype):
    code, tdt = _dt(L, dtype)
    M, N, K, T = 392, 192, 128, 196
    g = torch.Generator().manual_seed(5)
    A = torch.randn(M, K, generator=g).to(tdt)
    Bt = (torch.randn(N, K, generator=g) / 12).to(tdt)
    bias = torch.randn(N, generator=g)
    pos = torch.randn(T, generator=g)
    resid = torch.randn(M, N, generator=g)
    ncols = 150
    ref64 = A.double() @ Bt.double().T + bias.double()
    rows = torch.arange(M) % T
    ref64[:, :ncols] += pos.double()[rows][:, None]
    ref64 = torch.from_numpy(ref.mish(ref64.numpy())) + resid.double()
    out = resid.clone().to(cuda)              # in-place residual like the encoder
    out2 = torch.zeros(M, N, dtype=torch.bfloat16, device=cuda)
    _gemm(L, A.to(cuda), Bt.to(cuda), code, bias=bias.to(cuda), rowadd=pos.to(cuda),
          rowadd_period=T, rowadd_ncols=ncols, act=2, resid=out, out=out, out2=out2)
    assert (out.cpu().double() - ref64).abs().max().item() < 1e-4
    assert torch.equal(out2.cpu(), out.cpu().to(torch.bfloat16))


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_gemm_bf16_output(L, cuda, dtype):
    code, tdt = _dt(L, dtype)
    M, N, K = 256, 384, 64
    g = torch.Generator().manual_seed(9)
    A = torch.randn(M, K, generator=g).to(tdt)
    Bt = torch.randn(N, K, generator=g).to(tdt)
    out = torch.zeros(M, N, dtype=torch.bfloat16, device=cuda)
    _gemm(L, A.to(cuda), Bt.to(cuda), code, out=out, out_dtype=1)
    ref64 = A.double() @ Bt.double().T
    rel = ((out.cpu().double() - ref64).abs() / ref64.abs().clamp_min(1e-3)).max().item()
    assert rel < 8e-3     # one bf16 rounding of the output (2^-8)


@pytest.mark.parametrize("M,N,K,act,out_dtype,resid", [
    (2176, 320, 576, 2, 1, False),     # the head's Dense(272) per C2 micro-batch, mish
    (2176, 192, 320, 1, 1, False),     # Dense(136), gelu
    (2176, 6, 192, 0, 0, False),       # MLP_Head_no_Sigmoid
    (25088, 17, 768, 0, 1, False),     # Dense(17) (without the scatter)
    (1000, 100, 2048, 1, 0, True),     # the largest K, ragged M and N, f32 residual
    (33, 64, 64, 2, 1, True),          # one K-step pair, bf16 residual in place
    (777, 257, 1088, 0, 0, False),     # ragged column block
    (2176, 576, 1088, 1, 1, False)])   # Dense(544): skinny only with the threshold knob (640)
@pytest.mark.parametrize("skinny", [1, 0, 640])
def test_gemm_skinny(L, cuda, M, N, K, act, out_dtype, resid, skinny):
    """The skinny bf16 kernel (N <= 320, below the 256-tile threshold; knob value 640 raises the
    threshold) against fp64, and the 128 x 128 kernel it replaces (knob VTD_KNOB_SKINNY = 0):
    both fp32 accumulation of bf16 products, so they agree to fp32 summation order."""
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    odt = torch.float32 if out_dtype == 0 else torch.bfloat16
    out = torch.randn(M, N, generator=g, device=cuda).to(odt)
    x0 = out.clone()
    with L.knob(L.KNOB_SKINNY, skinny):
        _gemm(L, A, Bt, L.BF16, bias=bias, act=act, resid=out if resid else None, out=out,
              out_dtype=out_dtype)
    ref64 = _np_act(act, (A.double() @ Bt.double().T + bias.double()).cpu().numpy())
    if resid:
        ref64 = ref64 + x0.double().cpu().numpy()
    got = out.double().cpu().numpy()
    tol = 2e-5 if out_dtype == 0 else 8e-3
    err = np.abs(got - ref64) / np.maximum(np.abs(ref64), 1.0)
    assert err.max() < tol, (err.max(), np.argwhere(err >= tol)[:5].tolist())


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("T", [196, 37, 1])
@pytest.mark.parametrize("K", [64, 768, 1024])
def test_gemm_head_reshape_scatter(L, cuda, dtype, T, K):
    """Dense(17) + keras Reshape((17, -1)) (vtd.py:454-463) as a scatter epilogue:
    must equal the row-major reinterpretation, NOT a transpose.
    bf16 with K = 768 / 1024 takes the skinny (N <= 32) kernel."""
    code, tdt = _dt(L, dtype)
    B = 3
    g = torch.Generator().manual_seed(T)
    A = torch.randn(B * T, K, generator=g).to(tdt)
    Bt = torch.randn(17, K, generator=g).to(tdt)
    bias = torch.randn(17, generator=g)
    ld = ((T + 63) // 64) * 64
    out = torch.full((B * 17, ld), 7.0, device=cuda)
    out[:, T:] = 0
    _gemm(L, A.to(cuda), Bt.to(cuda), code, bias=bias.to(cuda), out=out, N=17,
          scatter_tokens=T, ldo=ld)
    t = (A.double() @ Bt.double().T + bias.double()).reshape(B, T, 17)
    u = t.reshape(B, 17, T)                     # row-major reshape
    got = out.cpu().double()[:, :T].reshape(B, 17, T)
    assert (got - u).abs().max().item() < 1e-4 * max(1.0, math.sqrt(K / 64))
    assert (out.cpu()[:, T:] == 0).all()


@pytest.mark.parametrize("x_dtype", ["f32", "bf16"])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("D,ld", [(768, 768), (28, 64), (30, 64), (1024, 1024), (4100, 4160)])
def test_layernorm(L, cuda, dtype, x_dtype, D, ld):
    """Input: the f32 residual stream, or the bf16 one of the bf16 / fp8 modes (the
    expected value is computed from the bf16-rounded input)."""
    code, tdt = _dt(L, dtype)
    xcode, xdt = _dt(L, x_dtype)
    rows = 37
    g = torch.Generator().manual_seed(D)
    x = torch.zeros(rows, ld)
    x[:, :D] = torch.randn(rows, D, generator=g) * 3 + 1
    x = x.to(xdt).float()
    gamma = torch.zeros(ld); gamma[:D] = 1 + 0.1 * torch.randn(D, generator=g)
    beta = torch.zeros(ld); beta[:D] = 0.1 * torch.randn(D, generator=g)
    y = torch.full((rows, ld), float("nan"), dtype=tdt, device=cuda)
    xd, gd, bd = x.to(xdt).to(cuda), gamma.to(cuda), beta.to(cuda)   # keep device copies alive
    L.check(L.lib.vtd_layernorm(xd.data_ptr(), xcode, rows, D, ld, gd.data_ptr(), bd.data_ptr(),
                                1e-3, y.data_ptr(), ld, code, L.stream_ptr()), "ln")
    torch.cuda.synchronize()
    exp = ref.layer_norm(x[:, :D].double().numpy(), gamma[:D].double().numpy(),
                         beta[:D].double().numpy())
    got = y.cpu().double().numpy()
    tol = 1e-5 if dtype == "f32" else 1.6e-2
    assert np.abs(got[:, :D] - exp).max() < tol * max(1, np.abs(exp).max())
    assert (got[:, D:] == 0).all()


def test_layernorm_epsilon_kat(L, cuda):
    """variance 1e-3 must be scaled by 1/sqrt(2e-3)."""
    D = 64
    x = torch.tensor([(-1) ** i * math.sqrt(1e-3) for i in range(D)], dtype=torch.float32)
    y = torch.zeros(1, D, device=cuda)
    one, zero = torch.ones(D, device=cuda), torch.zeros(D, device=cuda)
    xd = x.to(cuda)
    L.check(L.lib.vtd_layernorm(xd.data_ptr(), L.F32, 1, D, D, one.data_ptr(),
                                zero.data_ptr(), 1e-3, y.data_ptr(), D, L.F32, L.stream_ptr()))
    torch.cuda.synchronize()
    assert abs(y[0, 0].item() - math.sqrt(1e-3) / math.sqrt(2e-3)) < 1e-5


def _attn_ref(qkv, B, N, H, dk, dkp):
    q = qkv[:, :H * dkp].reshape(B, N, H, dkp)[..., :dk]
    k = qkv[:, H * dkp:2 * H * dkp].reshape(B, N, H, dkp)[..., :dk]
    v = qkv[:, 2 * H * dkp:3 * H * dkp].reshape(B, N, H, dkp)[..., :dk]
    s = np.einsum("bqhd,bkhd->bhqk", q, k) / math.sqrt(dk)
    p = ref.softmax(s, axis=-1)
    return np.einsum("bhqk,bkhd->bqhd", p, v)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("B,N,H,dk", [(2, 196, 3, 64), (1, 70, 2, 40), (1, 1, 1, 32),
                                      (1, 333, 2, 128), (1, 1296, 1, 40), (1, 64, 4, 20),
                                      # persistent kernel (dkp 64, 128 < N <= 256): several
                                      # pairs per workgroup, N not a multiple of 32 / 8
                                      (40, 196, 12, 64), (3, 129, 5, 64), (2, 256, 2, 64),
                                      (1, 200, 3, 50), (700, 131, 1, 64), (2, 224, 3, 64),
                                      # 16-query persistent kernel (N in (192, 208])
                                      (300, 193, 1, 64), (3, 208, 5, 64),
                                      # trimmed last key block: 11 / 26 keys in it
                                      (2, 203, 3, 64), (1, 218, 2, 64),
                                      # long-sequence LDS-DMA kernel (dkp 64, N > 256): C3's
                                      # N = 1600 (5 waves per workgroup), C5's 576 (6), ragged
                                      (2, 1600, 2, 64), (3, 576, 3, 64), (1, 300, 2, 64),
                                      (2, 257, 1, 64), (1, 1100, 1, 48)])
@pytest.mark.parametrize("variant", [-1, 5, 6])
def test_attention(L, cuda, dtype, B, N, H, dk, variant):
    if variant == 5 and (dtype != "bf16" or dk > 64 or not 192 < N <= 256):
        pytest.skip("the variant applies to bf16, dkp 64, N in (192, 256] only")
    if variant == 6 and (dtype != "bf16" or not 32 < dk <= 64):
        pytest.skip("the long-sequence kernels apply to bf16, dkp 64 (any N when forced)")
    code, tdt = _dt(L, dtype)
    dkp = 32 if dk <= 32 else (64 if dk <= 64 else 128)
    ld = 3 * H * dkp + 8
    g = np.random.default_rng(N * 10 + dk)
    qkv = np.zeros((B * N, ld), np.float32)
    for part in range(3):
        for h in range(H):
            c0 = part * H * dkp + h * dkp
            qkv[:, c0:c0 + dk] = g.normal(0, 1.5, size=(B * N, dk))
    qkv_t = torch.from_numpy(qkv).to(tdt)
    ldo = H * dkp
    out = torch.full((B * N, ldo), float("nan"), dtype=tdt, device=cuda)
    qkv_d = qkv_t.to(cuda)
    with L.knob(L.KNOB_ATTN_VARIANT, variant):
        L.check(L.lib.vtd_attention(qkv_d.data_ptr(), B, N, H, dkp, ld,
                                    1.0 / math.sqrt(dk), out.data_ptr(), ldo, code,
                                    L.stream_ptr()), "attention")
    torch.cuda.synchronize()
    exp = _attn_ref(qkv_t.double().numpy(), B, N, H, dk, dkp)
    got = out.cpu().double().numpy().reshape(B, N, H, dkp)
    # f32: exact-f32 MFMA + fp32 softmax; bf16: P rounded to bf16 before P.V
    tol = 2e-5 if dtype == "f32" else 2e-2
    assert np.abs(got[..., :dk] - exp).max() < tol * max(1.0, np.abs(exp).max())
    assert (got[..., dk:] == 0).all()


@pytest.mark.parametrize("B,N,H", [(256, 196, 12), (5, 129, 7), (3, 224, 4), (1, 161, 1),
                                   (7, 193, 3), (2, 208, 2)])
def test_attention_persistent_equals_per_pair_kernel(L, cuda, monkeypatch, B, N, H):
    """The persistent short-sequence kernel (knob VTD_KNOB_ATTN_VARIANT 4, the default for dkp 64 and
    128 < N <= 256) against the per-(image, head) kernel, at the C2 shape (3072 pairs, 12 per
    workgroup) and ragged ones.  Its softmax takes the row's true max in one pass (all keys
    are in LDS) where the streaming kernel keeps a deferred running max, so P rounds to bf16
    differently: equal to within bf16 rounding of P (both are checked against fp64 in
    test_attention)."""
    dkp = 64
    ld = 3 * H * dkp + 8
    g = torch.Generator().manual_seed(N + H)
    qkv = (torch.randn(B * N, ld, generator=g) * 1.5).to(torch.bfloat16).to(cuda)
    outs = []
    for variant in (2, 4, 5):
        o = torch.full((B * N, H * dkp + 16), float("nan"), dtype=torch.bfloat16, device=cuda)
        with L.knob(L.KNOB_ATTN_VARIANT, variant):
            L.check(L.lib.vtd_attention(qkv.data_ptr(), B, N, H, dkp, ld, 0.125, o.data_ptr(),
                                        H * dkp + 16, L.BF16, L.stream_ptr()), "attention")
        torch.cuda.synchronize()
        outs.append(o.cpu())
    a = outs[0][:, :H * dkp].float()
    for o in outs[1:]:
        b = o[:, :H * dkp].float()
        assert torch.isfinite(b).all()
        assert (a - b).abs().max().item() <= 1e-2 * max(1.0, a.abs().max().item())
        assert torch.isnan(o[:, H * dkp:].float()).all()     # nothing written past ldo's heads


@pytest.mark.parametrize("B,N,H", [(4, 1600, 12), (6, 576, 16), (3, 1100, 5), (2, 300, 3)])
def test_attention_long_sequence_equals_streaming_kernel(L, cuda, B, N, H):
    """The long-sequence LDS-DMA kernel (knob 6, opt-in) against the
    register-staged streaming kernel (knob 2) at the C3 / C5 shapes and ragged ones: the same
    64-key chunks and deferred-rescale online softmax, so equal to within bf16 rounding of P
    (both against fp64 in test_attention)."""
    dkp = 64
    ld = 3 * H * dkp + 8
    g = torch.Generator().manual_seed(N + H)
    qkv = (torch.randn(B * N, ld, generator=g) * 1.5).to(torch.bfloat16).to(cuda)
    outs = []
    for variant in (2, 6):
        o = torch.full((B * N, H * dkp + 16), float("nan"), dtype=torch.bfloat16, device=cuda)
        with L.knob(L.KNOB_ATTN_VARIANT, variant):
            L.check(L.lib.vtd_attention(qkv.data_ptr(), B, N, H, dkp, ld, 0.125, o.data_ptr(),
                                        H * dkp + 16, L.BF16, L.stream_ptr()), "attention")
        torch.cuda.synchronize()
        outs.append(o.cpu())
    a = outs[0][:, :H * dkp].float()
    for o in outs[1:]:
        b = o[:, :H * dkp].float()
        assert torch.isfinite(b).all()
        assert (a - b).abs().max().item() <= 1e-2 * max(1.0, a.abs().max().item())
        assert torch.isnan(o[:, H * dkp:].float()).all()


def test_attention_uniform_kat(L, cuda):
    """with Q = 0 the softmax is uniform -> O = mean over keys of V."""
    B, N, H, dkp = 1, 100, 2, 64
    g = torch.Generator().manual_seed(1)
    qkv = torch.zeros(B * N, 3 * H * dkp)
    qkv[:, H * dkp:] = torch.randn(B * N, 2 * H * dkp, generator=g)
    out = torch.zeros(B * N, H * dkp, device=cuda)
    qkv_d = qkv.to(cuda)
    L.check(L.lib.vtd_attention(qkv_d.data_ptr(), B, N, H, dkp, 3 * H * dkp, 0.125,
                                out.data_ptr(), H * dkp, L.F32, L.stream_ptr()))
    torch.cuda.synchronize()
    v = qkv[:, 2 * H * dkp:].double()
    assert (out.cpu().double() - v.mean(0, keepdim=True)).abs().max() < 1e-5


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("H,W,p", [(5, 5, 2), (608, 608, 17), (224, 224, 16), (40, 36, 8),
                                   (13, 7, 4), (384, 384, 16), (64, 32, 8)])
def test_extract_patches(L, cuda, dtype, H, W, p):
    """Generic gather kernel and (unpadded, bf16, P % 64 == 0: 224/16, 384/16, 64x32/8)
    the row-segment copy kernel."""
    code, tdt = _dt(L, dtype)
    B, C = 2, 3
    img = ref.synthetic_images(B, (H, W, C), seed=H + W)
    exp = ref.extract_patches_same(img, p)
    P = p * p * C
    ld = ((P + 63) // 64) * 64
    out = torch.full((B * exp.shape[1], ld), float("nan"), dtype=tdt, device=cuda)
    img_d = torch.from_numpy(img).to(cuda)
    L.check(L.lib.vtd_extract_patches(img_d.data_ptr(), B, H, W, C,
                                      p, out.data_ptr(), ld, code, L.stream_ptr()))
    torch.cuda.synchronize()
    got = out.cpu()
    exp_t = torch.from_numpy(exp.reshape(-1, P)).to(tdt)
    assert torch.equal(got[:, :P], exp_t)            # pure data movement: bit-exact
    assert (got[:, P:] == 0).all()


def test_decode_matches_oracle(L, cuda):
    g = np.random.default_rng(3)
    logits = g.normal(0, 4, size=(5, 17, 6)).astype(np.float32)
    logits[0, 0] = 0.0
    dets = torch.zeros(5, 17, 6, device=cuda)
    logits_d = torch.from_numpy(logits).to(cuda)
    L.check(L.lib.vtd_decode(logits_d.data_ptr(), 5 * 17,
                             dets.data_ptr(), L.stream_ptr()))
    torch.cuda.synchronize()
    exp = ref.transform_predictions(logits)
    assert np.abs(dets.cpu().numpy() - exp).max() < 1e-3
    # a zero logit decodes to [0.5, 39.5, 304, 304, 304, 304]
    np.testing.assert_allclose(dets[0, 0].cpu().numpy(), [0.5, 39.5, 304, 304, 304, 304],
                               rtol=1e-6)


def test_bad_args_raise_value_error(L, cuda):
    e = L.VtdEpilogue()
    with pytest.raises(ValueError):
        L.check(L.lib.vtd_gemm(16, 16, 30, 1, 32, 1, 32, L.BF16, ctypes.byref(e),
                               L.stream_ptr()), "gemm")


@pytest.mark.parametrize("M,N,K,act,out_dtype", [
    (4100, 2100, 192, 0, 0), (4100, 2100, 192, 1, 1), (8192, 1024, 64, 2, 0),
    (3000, 3000, 320, 1, 1), (4352, 8704, 256, 1, 1), (4100, 2104, 192, 0, 0),
    (2600, 776, 1536, 1, 1), (6272, 768, 768, 0, 0), (3000, 3000, 320, 2, 0),
    (5000, 2304, 128, 0, 1), (3000, 1544, 3072, 1, 1), (6400, 2304, 2048, 0, 1),
    (2100, 512, 4096, 2, 1)])
def test_gemm_bf16_256_tile_path(L, cuda, M, N, K, act, out_dtype):
    """Large problems (>= 128 tiles of 256 x 256) take the DMA-staged 256-tile kernel (pp2,
    vtd_gemm.hip); ragged M / N exercise the clamped loads and the masked epilogue."""
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    resid = torch.randn(M, N, generator=g, device=cuda) if out_dtype == 0 else None
    out = torch.full((M, N), float("nan"), device=cuda,
                     dtype=torch.float32 if out_dtype == 0 else torch.bfloat16)
    _gemm(L, A, Bt, L.BF16, bias=bias, act=act, resid=resid, out=out, out_dtype=out_dtype)
    ref64 = (A.double() @ Bt.double().T + bias.double()).cpu().numpy()
    ref64 = _np_act(act, ref64)
    if resid is not None:
        ref64 = ref64 + resid.double().cpu().numpy()
    got = out.double().cpu().numpy()
    tol = 2e-5 if out_dtype == 0 else 8e-3
    err = np.abs(got - ref64) / np.maximum(np.abs(ref64), 1.0)
    bad = np.argwhere(err >= tol)
    assert err.max() < tol, (err.max(), len(bad), bad[:5].tolist())


@pytest.mark.parametrize("M,N,K,act,resid", [
    (12544, 2304, 768, 0, False),    # the fp32 mode's query/key/value at C2 B = 64
    (6272, 3072, 768, 1, False),     # mlp1 (gelu), transposed-accumulator epilogue
    (12544, 768, 1536, 2, True),     # mish + f32 residual in place
    (4100, 2100, 192, 0, True),      # ragged M / N: generic epilogue on the split tiles
    (4096, 4096, 64, 1, False)])     # one K-step pair
def test_gemm_f32_256_tile_path(L, cuda, M, N, K, act, resid):
    """The fp32 parity mode's 256-tile kernel (v_mfma_f32_16x16x4_f32, exact fp32 fma
    chains) against fp64 and against the 128 x 128 kernel (knob VTD_KNOB_F32_PP2 = 0)."""
    g = torch.Generator(device=cuda).manual_seed(M + N + K + act)
    A = torch.randn(M, K, generator=g, device=cuda)
    Bt = torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)
    bias = torch.randn(N, generator=g, device=cuda)
    x0 = torch.randn(M, N, generator=g, device=cuda)
    outs = {}
    for v in (1, 0):
        x = x0.clone()
        with L.knob(L.KNOB_F32_PP2, v):
            _gemm(L, A, Bt, L.F32, bias=bias, act=act, resid=x if resid else None, out=x,
                  out_dtype=0)
        outs[v] = x
    ref64 = _np_act(act, (A.double() @ Bt.double().T + bias.double()).cpu().numpy())
    if resid:
        ref64 = ref64 + x0.double().cpu().numpy()
    for v, x in outs.items():
        err = np.abs(x.double().cpu().numpy() - ref64) / np.maximum(np.abs(ref64), 1.0)
        assert err.max() < 2e-5, (v, err.max(), np.argwhere(err >= 2e-5)[:5].tolist())


@pytest.mark.parametrize("M,N,K,act,resid", [
    (50176, 768, 768, 0, True),      # attn_out at C2 B=256: 588 tiles = 2.3 rounds
    (50176, 768, 1536, 1, True),     # mlp3
    (12544, 1536, 3072, 1, False),   # mlp2 at B=64: 294 tiles
    (4352, 4352, 8704, 1, False),    # head2: 289 tiles, 136 K-steps
    (4352, 2176, 4352, 2, False),    # head3: 153 tiles (< one round), mish
    (3000, 1544, 3072, 1, False),    # ragged M and N: generic epilogue on split tiles
    (4100, 776, 768, 0, True),       # ragged, residual, no activation
    (2100, 512, 256, 0, False),      # 4 K-steps only
    (4096, 2048, 64, 1, False),      # one K-step (no steady-state loop)
    (4096, 2048, 128, 0, False)])    # two K-steps
def test_gemm_variants_w4_pp2(L, cuda, monkeypatch, M, N, K, act, resid):
    """The 256-tile bf16 kernel (pp2, 8-wave ping-pong) against fp64 with an in-place
    residual; with the diagnostic library (`make diag`, VTD_LIB_PATH) also the w4 kernel
    (VTD_GEMM_VARIANT 12, one wave per SIMD, persistent; VTD_W4_SCHED 1 / 2) against fp64 and
    against pp2 (same K order of the fp32 accumulation: within bf16 output rounding)."""
    variants = ("10", "12", "12s2") if hasattr(L.lib, "vtd_diag_build") else ("10",)
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    x0 = (4 * torch.randn(M, N, generator=g, device=cuda)).to(torch.bfloat16)
    outs = {}
    for v in variants:
        monkeypatch.setenv("VTD_GEMM_VARIANT", v[:2])
        monkeypatch.setenv("VTD_W4_SCHED", "2" if v.endswith("s2") else "1")
        x = x0.clone()
        _gemm(L, A, Bt, L.BF16, bias=bias, act=act, resid=x if resid else None, out=x,
              out_dtype=1)
        outs[v] = x
    ref64 = _np_act(act, (A.double() @ Bt.double().T + bias.double()).cpu().numpy())
    if resid:
        ref64 = ref64 + x0.double().cpu().numpy()
    for v in variants:
        got = outs[v].double().cpu().numpy()
        err = np.abs(got - ref64) / np.maximum(np.abs(ref64), 1.0)
        assert err.max() < 8e-3, (v, err.max(), np.argwhere(err >= 8e-3)[:5].tolist())
    if len(variants) == 1:
        return
    d = (outs["12"].float() - outs["10"].float()).abs() / outs["10"].float().abs().clamp(min=1.0)
    assert d.max().item() < 1.6e-2        # <= 2 bf16 ulps
    assert torch.equal(outs["12"], outs["12s2"])     # the schedules differ in timing only


@pytest.mark.parametrize("act,resid,fold,stat", [(0, False, True, False), (1, False, True, False),
                                                 (0, True, False, True), (1, True, False, True),
                                                 (2, False, False, False)])
@pytest.mark.parametrize("tr", [0, 1])
def test_gemm_accumulator_layouts(L, cuda, act, resid, fold, stat, tr):
    """The 256-tile kernel's two accumulator layouts (knob VTD_KNOB_GEMM_TR: 0 = LDS-staged
    row vectors, 1 = transposed accumulators, register-direct epilogue) on the forward's
    epilogue combinations -- LayerNorm fold (row statistics from the wave's LDS table),
    residual + partial statistics, activations -- against fp64."""
    M, N, K = 12544, 768, 768
    g = torch.Generator(device=cuda).manual_seed(7 + act + 2 * tr)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    x0 = torch.randn(M, N, generator=g, device=cuda).to(torch.bfloat16)
    x = x0.clone()
    e = L.VtdEpilogue()
    e.bias, e.act, e.out, e.ldo, e.out_dtype = bias.data_ptr(), act, x.data_ptr(), N, 1
    keep = []
    if resid:
        e.resid, e.ldr = x.data_ptr(), N
    if fold:
        mean = torch.randn(M, generator=g, device=cuda) * 0.1
        rstd = torch.rand(M, generator=g, device=cuda) + 0.5
        lnstat = torch.stack([mean, rstd], 1).contiguous()
        colsum = Bt.float().sum(1).contiguous()
        keep += [lnstat, colsum]
        e.lnstat, e.colsum = lnstat.data_ptr(), colsum.data_ptr()
    if stat:
        st_planes = torch.full((N // 64, M, 2), float("nan"), device=cuda)   # slot-major statout
        st = st_planes.permute(1, 0, 2)
        keep.append(st_planes)
        e.statout, e.stat_ld = st_planes.data_ptr(), M
    with L.knob(L.KNOB_GEMM_TR, tr):
        L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16,
                               ctypes.byref(e), L.stream_ptr()), "vtd_gemm")
    torch.cuda.synchronize()
    acc = A.double() @ Bt.double().T
    if fold:
        acc = (acc - lnstat[:, :1].double() * colsum.double()[None, :]) * lnstat[:, 1:].double()
    ref64 = _np_act(act, (acc + bias.double()).cpu().numpy())
    if resid:
        ref64 = ref64 + x0.double().cpu().numpy()
    got = x.double().cpu().numpy()
    err = np.abs(got - ref64) / np.maximum(np.abs(ref64), 1.0)
    assert err.max() < 8e-3, (err.max(), np.argwhere(err >= 8e-3)[:5].tolist())
    if stat:
        blocks = x.float().view(M, N // 64, 64)
        assert torch.allclose(st[..., 0], blocks.mean(-1), rtol=1e-5, atol=1e-5)
        m2 = ((blocks - blocks.mean(-1, keepdim=True)) ** 2).sum(-1)
        assert torch.allclose(st[..., 1], m2, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("variant", ["10", "12", "12s2"])
def test_gemm_statout_variants(L, cuda, monkeypatch, variant):
    """The producer-side LayerNorm partial statistics on the 256-tile kernels (w4: the
    diagnostic library only)."""
    if variant != "10" and not hasattr(L.lib, "vtd_diag_build"):
        pytest.skip("the w4 kernel is in the diagnostic build only (make diag)")
    monkeypatch.setenv("VTD_GEMM_VARIANT", variant[:2])
    monkeypatch.setenv("VTD_W4_SCHED", "2" if variant.endswith("s2") else "1")
    M, N, K = 50176, 768, 768
    g = torch.Generator(device=cuda).manual_seed(5)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    stat_planes = torch.full((N // 64, M, 2), float("nan"), device=cuda)   # slot-major statout
    stat = stat_planes.permute(1, 0, 2)
    e = L.VtdEpilogue()
    e.bias, e.out, e.ldo, e.out_dtype = bias.data_ptr(), out.data_ptr(), N, 1
    e.statout, e.stat_ld = stat_planes.data_ptr(), M
    L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16,
                           ctypes.byref(e), L.stream_ptr()), "vtd_gemm")
    torch.cuda.synchronize()
    r64 = A.double() @ Bt.double().T + bias.double()
    assert ((out.double() - r64).abs() / r64.abs().clamp(min=1.0)).max().item() < 8e-3
    blocks = out.float().view(M, N // 64, 64)
    assert torch.allclose(stat[..., 0], blocks.mean(-1), rtol=1e-5, atol=1e-5)
    m2 = ((blocks - blocks.mean(-1, keepdim=True)) ** 2).sum(-1)
    assert torch.allclose(stat[..., 1], m2, rtol=1e-4, atol=1e-4)


def test_decode_detections_matches_oracle(L, cuda):
    """Fused decode + the MeanAveragePrecision prediction test (vtd.py:1359-1384)."""
    from vision_transformer_detector_amd import decode_detections
    g = np.random.default_rng(11)
    logits = g.normal(0, 3, size=(64, 17, 6)).astype(np.float32)
    dets, cat, valid = decode_detections(torch.from_numpy(logits).to(cuda))
    exp = ref.transform_predictions(logits)
    ecat, evalid = ref.detection_mask(exp)
    assert np.abs(dets.cpu().numpy() - exp).max() < 1e-3
    # ignore slots within float rounding of a threshold / a .5 class boundary
    conf = (0.5 - np.abs(exp[..., 1] - np.round(exp[..., 1]))) / 0.5
    frac = np.abs(exp[..., 1] - np.floor(exp[..., 1]) - 0.5)
    safe = (np.abs(exp[..., 0] - 0.5) > 1e-4) & (np.abs(conf - 0.5) > 1e-4) & (frac > 1e-4)
    assert safe.mean() > 0.95
    np.testing.assert_array_equal(cat.cpu().numpy()[safe], ecat[safe])
    np.testing.assert_array_equal(valid.cpu().numpy()[safe], evalid[safe])
    assert 0 < evalid.sum() < evalid.size        # both outcomes exercised


@pytest.mark.parametrize("M,N,K,act", [
    (6272, 768, 768, 0), (6272, 768, 1536, 1), (4100, 776, 768, 0), (4100, 776, 1536, 2),
    (300, 200, 256, 1)])
def test_gemm_bf16_residual_in_place(L, cuda, M, N, K, act):
    """The bf16 residual stream of the bf16 / fp8 modes: out_dtype bf16 with resid aliasing
    out (resid is read in the output's dtype) on the 256-tile fast epilogues (act 0: pp2b,
    act > 0: transposed pp2t), their ragged-tile generic epilogue, and the 128-tile kernel."""
    g = torch.Generator(device=cuda).manual_seed(M + N + K + act)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    x = (4 * torch.randn(M, N, generator=g, device=cuda)).to(torch.bfloat16)
    x0 = x.double().cpu().numpy()
    _gemm(L, A, Bt, L.BF16, bias=bias, act=act, resid=x, out=x, out_dtype=1)
    ref64 = _np_act(act, (A.double() @ Bt.double().T + bias.double()).cpu().numpy()) + x0
    err = np.abs(x.double().cpu().numpy() - ref64) / np.maximum(np.abs(ref64), 1.0)
    assert err.max() < 8e-3, err.max()


@pytest.mark.parametrize("act", [0, 1])
def test_gemm_256_rowadd_out2_fast_path(L, cuda, act):
    """The 256-tile kernels' fast epilogues with the two once-per-forward modes: the
    position-embedding row add (vtd.py:305, columns < rowadd_ncols) and the bf16 copy
    out2 of the last residual (the head's input)."""
    M, N, K, T = 6272, 768, 768, 196
    g = torch.Generator(device=cuda).manual_seed(17 + act)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    rowadd = torch.randn(T, generator=g, device=cuda)
    resid = torch.randn(M, N, generator=g, device=cuda)
    out = resid.clone()
    out2 = torch.zeros(M, N, device=cuda, dtype=torch.bfloat16)
    _gemm(L, A, Bt, L.BF16, bias=bias, rowadd=rowadd, rowadd_period=T, rowadd_ncols=700,
          act=act, resid=out, out=out, out_dtype=0, out2=out2)
    ref64 = (A.double() @ Bt.double().T + bias.double()).cpu().numpy()
    ra = rowadd.double().cpu().numpy()[np.arange(M) % T]
    ref64[:, :700] += ra[:, None]
    ref64 = _np_act(act, ref64) + resid.double().cpu().numpy()
    err = np.abs(out.double().cpu().numpy() - ref64) / np.maximum(np.abs(ref64), 1.0)
    assert err.max() < 2e-5, err.max()
    err2 = np.abs(out2.double().cpu().numpy() - ref64) / np.maximum(np.abs(ref64), 1.0)
    assert err2.max() < 8e-3, err2.max()


# ---- LayerNorm fold (bf16 mode): vtd_layernorm_stats + vtd_fold_layernorm + lnstat epilogue
@pytest.mark.parametrize("x_dtype", ["f32", "bf16"])
@pytest.mark.parametrize("D,ld", [(768, 768), (30, 64), (4100, 4160)])
def test_layernorm_stats(L, cuda, x_dtype, D, ld):
    xcode, xdt = _dt(L, x_dtype)
    rows = 53
    g = torch.Generator().manual_seed(D + 1)
    x = torch.zeros(rows, ld)
    x[:, :D] = torch.randn(rows, D, generator=g) * 2 + 3
    x = x.to(xdt)
    xd = x.to(cuda)
    st = torch.full((rows, 2), float("nan"), device=cuda)
    L.check(L.lib.vtd_layernorm_stats(xd.data_ptr(), xcode, rows, D, ld, 1e-3, st.data_ptr(),
                                      L.stream_ptr()), "ln_stats")
    torch.cuda.synchronize()
    x64 = x[:, :D].double().numpy()
    mu = x64.mean(1)
    rstd = 1 / np.sqrt(((x64 - mu[:, None]) ** 2).mean(1) + 1e-3)
    got = st.cpu().double().numpy()
    assert np.abs(got[:, 0] - mu).max() < 1e-5 * np.abs(mu).max()
    assert np.abs(got[:, 1] - rstd).max() < 1e-5 * rstd.max()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_fold_layernorm(L, cuda, dtype):
    code, tdt = _dt(L, dtype)
    N, K, ldo = 200, 96, 128
    g = torch.Generator().manual_seed(5)
    w = torch.randn(N, K, generator=g)
    gamma, beta = 1 + 0.2 * torch.randn(K, generator=g), 0.3 * torch.randn(K, generator=g)
    b = torch.randn(N, generator=g)
    wd, gd, bd, bid = w.to(cuda), gamma.to(cuda), beta.to(cuda), b.to(cuda)
    wo = torch.full((N, ldo), float("nan"), device=cuda).to(tdt)
    bo = torch.zeros(N, device=cuda)
    cs = torch.zeros(N, device=cuda)
    L.check(L.lib.vtd_fold_layernorm(wd.data_ptr(), N, K, K, gd.data_ptr(), bd.data_ptr(),
                                     bid.data_ptr(), wo.data_ptr(), ldo, code, bo.data_ptr(),
                                     cs.data_ptr(), L.stream_ptr()), "fold")
    torch.cuda.synchronize()
    exp_w = (w * gamma[None, :]).to(tdt)
    assert torch.equal(wo[:, :K].cpu(), exp_w)          # same rounding (RNE) as torch
    assert (wo[:, K:].cpu().float() == 0).all()
    np.testing.assert_allclose(bo.cpu().double().numpy(),
                               b.double().numpy() + w.double().numpy() @ beta.double().numpy(),
                               rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(cs.cpu().double().numpy(), exp_w.double().sum(1).numpy(),
                               rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("M,N,K,act,dtype,offset", [
    (6272, 2304, 768, 0, "bf16", 8), (6272, 3072, 768, 1, "bf16", 8),
    (4100, 776, 768, 2, "bf16", 8), (300, 200, 256, 1, "bf16", 8), (300, 200, 128, 0, "f32", 8),
    # |mean| / std ~ 1e2: the folded epilogue (acc - mean colsum) rstd cancels a
    # mean * colsum term 1e2 times the result's scale.  (At 1e3 the bf16 stream itself has
    # no digits left for the row's spread -- its spacing at the mean is ~4 std -- so the
    # statistics test above covers that ratio on the stored values.)
    (6272, 2304, 768, 0, "bf16", 200), (6272, 3072, 768, 1, "bf16", 200)])
def test_gemm_layernorm_fold(L, cuda, M, N, K, act, dtype, offset):
    """LN(x) W + b computed as a GEMM on the raw rows x with the folded weights and the
    lnstat epilogue, against fp64 LN -> Dense -> act.  Paths: 256-tile fast epilogues
    (act 0: pp2b staged, act > 0: transposed direct), ragged tiles (generic), the 128-tile
    kernel, f32 mode.  Rows have a large common offset (mean >> std in some rows)."""
    code, tdt = _dt(L, dtype)
    g = torch.Generator(device=cuda).manual_seed(M + N + K + act)
    x = (torch.randn(M, K, generator=g, device=cuda) * 2
         + offset * torch.randn(M, 1, generator=g, device=cuda)).to(tdt)
    w = torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)
    gamma = 1 + 0.2 * torch.randn(K, generator=g, device=cuda)
    beta = 0.3 * torch.randn(K, generator=g, device=cuda)
    b = torch.randn(N, generator=g, device=cuda)
    wo = torch.zeros(N, K, device=cuda).to(tdt)
    bo, cs = torch.zeros(N, device=cuda), torch.zeros(N, device=cuda)
    L.check(L.lib.vtd_fold_layernorm(w.data_ptr(), N, K, K, gamma.data_ptr(), beta.data_ptr(),
                                     b.data_ptr(), wo.data_ptr(), K, code, bo.data_ptr(),
                                     cs.data_ptr(), L.stream_ptr()), "fold")
    st = torch.zeros(M, 2, device=cuda)
    L.check(L.lib.vtd_layernorm_stats(x.data_ptr(), code, M, K, K, 1e-3, st.data_ptr(),
                                      L.stream_ptr()), "stats")
    out = torch.full((M, N), float("nan"), device=cuda, dtype=tdt)
    e = L.VtdEpilogue()
    e.bias, e.act, e.out, e.ldo, e.out_dtype = bo.data_ptr(), act, out.data_ptr(), N, code
    e.lnstat, e.colsum = st.data_ptr(), cs.data_ptr()
    L.check(L.lib.vtd_gemm(M, N, K, x.data_ptr(), K, wo.data_ptr(), K, code, ctypes.byref(e),
                           L.stream_ptr()), "gemm")
    torch.cuda.synchronize()
    h = ref.layer_norm(x.double().cpu().numpy(), gamma.double().cpu().numpy(),
                       beta.double().cpu().numpy())
    ref64 = _np_act(act, h @ w.double().cpu().numpy().T + b.double().cpu().numpy())
    err = np.abs(out.double().cpu().numpy() - ref64) / np.maximum(np.abs(ref64), 1.0)
    # bf16: the W' = W * gamma rounding (2^-9 relative per weight, sigma ~1.1e-3 on unit
    # outputs, the max over 1.4e7 outputs ~6 sigma) + the bf16 output rounding (2^-9);
    # the unfolded path has the same budget (h and W rounded to bf16).  f32: exact-ish.
    tol = 1.6e-2 if dtype == "bf16" else 1e-4
    assert err.max() < tol, err.max()


@pytest.mark.parametrize("N,K,act,resid,offset", [
    (768, 768, 0, True, 3.0), (768, 1536, 1, True, 3.0), (1024, 512, 0, False, 3.0),
    (512, 256, 2, False, 3.0),
    # adversarial rows: |mean| / std ~ 1e2 and 1e3 (trained-weight outlier rows)
    (768, 768, 0, True, 2e2), (768, 768, 0, False, 2e3), (768, 1536, 1, True, 2e2)])
def test_gemm_statout_and_finalize(L, cuda, N, K, act, resid, offset):
    """Producer side of the LayerNorm fold: the bf16 fast epilogues (act 0: pp2b staged,
    act > 0: transposed direct) emit per-(row, 64-column block) centred partials (block
    mean, sum of squared deviations) of the STORED bf16 outputs;
    vtd_layernorm_stats_finalize merges them (Chan) into (mean, rstd).  With offset 2e3
    and std ~2 the rows have |mean| / std ~ 1e3, where a one-pass sum(x^2)/D - mean^2
    in fp32 loses every digit of the variance."""
    M = 256 * 64                       # >= 128 tiles: the 256-tile kernels
    g = torch.Generator(device=cuda).manual_seed(N + K + act + int(offset))
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    if not resid:                      # the offset then rides on the bias (act 0 only)
        bias += offset if act == 0 else 0.0
    x = (offset + 2 * torch.randn(M, N, generator=g, device=cuda)).to(torch.bfloat16)
    slots = N // 64
    part_planes = torch.full((slots, M, 2), float("nan"), device=cuda)   # slot-major statout
    part = part_planes.permute(1, 0, 2)
    e = L.VtdEpilogue()
    e.bias, e.act, e.out, e.ldo, e.out_dtype = bias.data_ptr(), act, x.data_ptr(), N, 1
    if resid:
        e.resid, e.ldr = x.data_ptr(), N
    e.statout, e.stat_ld = part_planes.data_ptr(), M
    L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16, ctypes.byref(e),
                           L.stream_ptr()), "gemm")
    st = torch.zeros(M, 2, device=cuda)
    L.check(L.lib.vtd_layernorm_stats_finalize(part_planes.data_ptr(), M, slots, N, 1e-3, st.data_ptr(),
                                               L.stream_ptr()), "finalize")
    # the grid-stride form (knob VTD_KNOB_FIN_WGS, few 1024-thread workgroups): same bits
    st2 = torch.full((M, 2), float("nan"), device=cuda)
    with L.knob(L.KNOB_FIN_WGS, 3):
        L.check(L.lib.vtd_layernorm_stats_finalize(part_planes.data_ptr(), M, slots, N, 1e-3,
                                                   st2.data_ptr(), L.stream_ptr()), "finalize")
    torch.cuda.synchronize()
    assert torch.equal(st, st2)
    xs = x.double().cpu().numpy().reshape(M, slots, 64)
    got = part.double().cpu().numpy()
    bm = xs.mean(2)
    bm2 = ((xs - bm[..., None]) ** 2).sum(2)
    np.testing.assert_allclose(got[..., 0], bm, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(got[..., 1], bm2, rtol=1e-4, atol=1e-4 * bm2.mean())
    x64 = xs.reshape(M, N)
    mu = x64.mean(1)
    rstd = 1 / np.sqrt(x64.var(1) + 1e-3)
    s = st.double().cpu().numpy()
    assert np.abs(s[:, 0] - mu).max() < 1e-6 * max(1, np.abs(mu).max())
    # rstd relative to each row's own value (the rows' variances differ widely when the
    # offset quantizes the stored bf16 values)
    assert (np.abs(s[:, 1] - rstd) / rstd).max() < 1e-4


def test_layernorm_stats_finalize_needs_full_blocks(L, cuda):
    part = torch.zeros(4, 2, 2, device=cuda)
    st = torch.zeros(4, 2, device=cuda)
    with pytest.raises(ValueError):                # VTD_ERR_INVALID_ARG
        L.check(L.lib.vtd_layernorm_stats_finalize(part.data_ptr(), 4, 2, 100, 1e-3,
                                                   st.data_ptr(), L.stream_ptr()), "finalize")


def test_gemm_statout_unsupported_shape(L, cuda):
    """statout only on full tiles: a ragged M is refused (the forward then runs the
    row-statistics pass instead)."""
    M, N, K = 256 * 64 + 8, 768, 256
    A = torch.zeros(M, K, device=cuda, dtype=torch.bfloat16)
    Bt = torch.zeros(N, K, device=cuda, dtype=torch.bfloat16)
    out = torch.zeros(M, N, device=cuda, dtype=torch.bfloat16)
    bias = torch.zeros(N, device=cuda)
    part_planes = torch.zeros(N // 64, M, 2, device=cuda)     # slot-major statout
    e = L.VtdEpilogue()
    e.bias, e.out, e.ldo, e.out_dtype = bias.data_ptr(), out.data_ptr(), N, 1
    e.statout, e.stat_ld = part_planes.data_ptr(), M
    with pytest.raises(L.VtdError):
        L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16, ctypes.byref(e),
                               L.stream_ptr()), "gemm")


@pytest.mark.parametrize("M,N,K,ksplit,act,out_dtype", [
    (2176, 4352, 8704, 2, 1, 1), (2176, 2176, 4352, 4, 1, 1), (2176, 1088, 2176, 4, 2, 1),
    (300, 520, 1088, 3, 0, 0), (1000, 136, 640, 5, 1, 0), (257, 264, 192, 3, 0, 1)])
def test_gemm_splitk(L, cuda, M, N, K, ksplit, act, out_dtype):
    """vtd_gemm_splitk (the head's few-tile, long-K layers): fp32 partial sums of ksplit K
    ranges summed in split order + the epilogue, against fp64 and within fp32 summation-order
    noise of the unsplit kernel; ragged M / N take the masked partial tiles."""
    g = torch.Generator(device=cuda).manual_seed(M + N + K + ksplit)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    resid = torch.randn(M, N, generator=g, device=cuda) if out_dtype == 0 else None
    odt = torch.float32 if out_dtype == 0 else torch.bfloat16
    out = torch.full((M, N), float("nan"), device=cuda, dtype=odt)
    part = torch.full((ksplit, M, N), float("nan"), device=cuda)
    e = L.VtdEpilogue()
    e.bias, e.act, e.out, e.ldo, e.out_dtype = L.ptr(bias), act, L.ptr(out), N, out_dtype
    e.resid, e.ldr = L.ptr(resid), (N if resid is not None else 0)
    L.check(L.lib.vtd_gemm_splitk(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16,
                                  ctypes.byref(e), part.data_ptr(), part.numel() * 4, ksplit,
                                  L.stream_ptr()),
            "vtd_gemm_splitk")
    torch.cuda.synchronize()
    ref64 = _np_act(act, (A.double() @ Bt.double().T + bias.double()).cpu().numpy())
    if resid is not None:
        ref64 = ref64 + resid.double().cpu().numpy()
    got = out.double().cpu().numpy()
    tol = 2e-5 if out_dtype == 0 else 8e-3
    err = np.abs(got - ref64) / np.maximum(np.abs(ref64), 1.0)
    assert err.max() < tol, err.max()
    # the unsplit kernel on the same operands: equal up to fp32 summation order (f32 out)
    # or one bf16 rounding step (bf16 out)
    out1 = torch.full((M, N), float("nan"), device=cuda, dtype=odt)
    _gemm(L, A, Bt, L.BF16, bias=bias, act=act, resid=resid, out=out1, out_dtype=out_dtype)
    d = (out1.double() - out.double()).abs().cpu().numpy() / np.maximum(np.abs(ref64), 1.0)
    assert d.max() < (1e-5 if out_dtype == 0 else 8e-3), d.max()


def test_gemm_splitk_choice_and_args(L, cuda):
    """The forward's split counts for the C2 head (B x 17 = 2176 rows per micro-batch) and
    argument checks (ksplit < 2, short partial buffer, an empty split)."""
    c = L.lib.vtd_gemm_splitk_choice
    assert c(2176, 4352, 8704, L.BF16) == 2
    assert c(2176, 2176, 4352, L.BF16) == 4
    assert c(2176, 8704, 256, L.BF16) == 1          # short K
    assert c(50176, 768, 768, L.BF16) == 1          # many tiles
    assert c(2176, 4352, 8704, L.F32) == 1          # bf16 only
    e = L.VtdEpilogue()
    for ks, nbytes, K in ((1, 1 << 30, 512), (2, 16, 512), (9, 1 << 30, 512)):
        with pytest.raises(ValueError):
            L.check(L.lib.vtd_gemm_splitk(64, 64, K, 1, K, 1, K, L.BF16, ctypes.byref(e), 1,
                                          nbytes, ks, L.stream_ptr()), "gemm_splitk")


def test_gemm_statout_needs_a_specialised_epilogue(L, cuda):
    """Partial LayerNorm statistics are written only by the specialised 256-tile epilogues:
    a combination without one (the fold + residual + statistics of a single-layer MLP) is
    refused with VTD_ERR_UNSUPPORTED instead of returning OK with the statistics unwritten
    (ADVICE r3); the same GEMM without the fold still emits them."""
    M, N, K = 32768, 512, 512
    g = torch.Generator(device=cuda).manual_seed(3)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    colsum = Bt.float().sum(1).contiguous()
    lnstat = torch.stack([A.float().mean(1), torch.ones(M, device=cuda)], 1).contiguous()
    x = torch.randn(M, N, generator=g, device=cuda).to(torch.bfloat16)
    stat_planes = torch.full((N // 64, M, 2), float("nan"), device=cuda)   # slot-major statout
    stat = stat_planes.permute(1, 0, 2)
    e = L.VtdEpilogue()
    e.bias, e.act, e.out, e.ldo, e.out_dtype = bias.data_ptr(), L.ACT_GELU_TANH, x.data_ptr(), N, 1
    e.resid, e.ldr = x.data_ptr(), N
    e.lnstat, e.colsum = lnstat.data_ptr(), colsum.data_ptr()
    e.statout, e.stat_ld = stat_planes.data_ptr(), M
    rc = L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16, ctypes.byref(e),
                        L.stream_ptr())
    assert rc == -2, (rc, L.lib.vtd_last_error())
    e.lnstat, e.colsum = None, None
    L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16, ctypes.byref(e),
                           L.stream_ptr()), "vtd_gemm")
    torch.cuda.synchronize()
    assert torch.isfinite(stat).all()
    blocks = x.float().view(M, N // 64, 64)
    assert torch.allclose(stat[..., 0], blocks.mean(-1), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M,N,K,act,mode", [
    (4100, 2100, 192, 1, "bf16"),         # ragged M / N: generic epilogue on edge tiles
    (8192, 1024, 64, 1, "bf16"),          # one K-step: the prefetched stage is the whole loop
    (12544, 768, 768, 0, "stat"),         # residual + partial statistics (attention_output)
    (12544, 768, 768, 1, "fold"),         # LayerNorm fold + gelu (mlp1)
    (12544, 2304, 768, 0, "fold"),        # LayerNorm fold (query/key/value)
    (6000, 1544, 3072, 1, "bf16")])       # (all >= 128 tiles: the pp2 kernels)
@pytest.mark.parametrize("tpw", [2, 3, 5])
def test_gemm_tiles_per_workgroup(L, cuda, M, N, K, act, mode, tpw):
    if not hasattr(L.lib, "vtd_diag_build"):
        pytest.skip("the multi-tile kernel is in the diagnostic build only (VTD_LIB_PATH=libvtd_diag.so)")
    """Several output tiles per pp2 workgroup (knob VTD_KNOB_GEMM_TPW, gemm_tn_bf16_pp2_mt_kernel
    for the forward's epilogue codes; the next tile's first K-stage is loaded during the
    current tile's epilogue): every tile is computed by the same instructions, so the outputs
    (and statistics) equal the one-tile launch bit for bit -- tile counts not divisible by
    tpw, ragged edges and one-K-step loops included."""
    g = torch.Generator(device=cuda).manual_seed(M + K + act)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    f32 = mode == "f32resid"
    r0 = torch.randn(M, N, generator=g, device=cuda)
    if not f32:
        r0 = r0.to(torch.bfloat16)
    keep = []

    def run():
        x = r0.clone()
        e = L.VtdEpilogue()
        e.bias, e.act, e.out, e.ldo, e.out_dtype = bias.data_ptr(), act, x.data_ptr(), N, 0 if f32 else 1
        st = None
        if mode in ("f32resid", "stat"):
            e.resid, e.ldr = x.data_ptr(), N
        if mode == "stat":
            st_planes = torch.full((N // 64, M, 2), float("nan"), device=cuda)   # slot-major statout
            st = st_planes.permute(1, 0, 2)
            e.statout, e.stat_ld = st_planes.data_ptr(), M
        if mode == "fold":
            gg = torch.Generator(device=cuda).manual_seed(3)
            lnstat = torch.stack([torch.randn(M, generator=gg, device=cuda) * 0.1,
                                  torch.rand(M, generator=gg, device=cuda) + 0.5], 1).contiguous()
            colsum = Bt.float().sum(1).contiguous()
            keep.extend([lnstat, colsum])
            e.lnstat, e.colsum = lnstat.data_ptr(), colsum.data_ptr()
        L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16,
                               ctypes.byref(e), L.stream_ptr()), "vtd_gemm")
        torch.cuda.synchronize()
        return x, st

    with L.knob(L.KNOB_GEMM_TPW, 1):
        x1, s1 = run()
    with L.knob(L.KNOB_GEMM_TPW, tpw):
        x2, s2 = run()
    assert not torch.isnan(x1.float()).any()
    assert torch.equal(x1, x2)
    if s1 is not None:
        assert torch.equal(s1, s2)


@pytest.mark.parametrize("M,N,K,ks", [(1568, 2304, 768, 3), (196, 3072, 768, 6)])
def test_gemm_splitk_layernorm_fold(L, cuda, M, N, K, ks):
    """vtd_gemm_splitk with the LayerNorm fold (epilogue.lnstat / colsum, applied in the
    reduction's epilogue: what vtd_forward's small-batch query/key/value and first MLP layers
    run) against the unsplit kernel on the same operands: equal up to fp32 summation order."""
    g = torch.Generator(device=cuda).manual_seed(M + N + ks)
    A = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    Bt = (torch.randn(N, K, generator=g, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=cuda)
    mean = torch.randn(M, generator=g, device=cuda) * 0.1
    rstd = torch.rand(M, generator=g, device=cuda) + 0.5
    lnstat = torch.stack([mean, rstd], 1).contiguous()
    colsum = Bt.float().sum(1).contiguous()
    outs = []
    for split in (1, ks):
        out = torch.full((M, N), float("nan"), device=cuda)
        e = L.VtdEpilogue()
        e.bias, e.act, e.out, e.ldo, e.out_dtype = L.ptr(bias), 1, L.ptr(out), N, 0
        e.lnstat, e.colsum = lnstat.data_ptr(), colsum.data_ptr()
        if split == 1:
            L.check(L.lib.vtd_gemm(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16,
                                   ctypes.byref(e), L.stream_ptr()), "vtd_gemm")
        else:
            part = torch.empty(split * M * N, device=cuda)
            L.check(L.lib.vtd_gemm_splitk(M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, L.BF16,
                                          ctypes.byref(e), part.data_ptr(), part.numel() * 4,
                                          split, L.stream_ptr()), "vtd_gemm_splitk")
        outs.append(out)
    torch.cuda.synchronize()
    d = (outs[0].double() - outs[1].double()).abs().max().item()
    assert d <= 1e-5 * max(1.0, outs[0].abs().max().item()), d
