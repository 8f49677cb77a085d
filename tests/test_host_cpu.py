"""CPU tests of the C-ABI library and the host mirror (no GPU, no compute calls):
libvtd.so loads and exports every symbol include/vtd.h declares, the ctypes structs have
the C layout, graph shapes / weight names agree with the oracle, and invalid arguments
come back as ValueError like Keras would raise.
"""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from oracle import vtd_numpy as V

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vtd.h")


@pytest.fixture(scope="module")
def L():
    from vision_transformer_detector_amd import _lib
    return _lib


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vtd_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(L):
    names = declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(L.lib, n), f"libvtd.so does not export {n}"
        assert n in L.SIGNATURES, f"ctypes binding missing for {n}"
    assert L.lib.vtd_abi_version() == L.ABI_VERSION


def test_removed_switches_are_not_read_by_the_library(L):
    """The round-2 diagnostic switches (VTD_ATTN_DIAG, VTD_PP3_DIAG, VTD_LN_FUSE) are gone
    from the product library: their names are not in libvtd.so's strings, so no getenv can
    read them (the GPU test checks the logits with them set)."""
    blob = open(L.lib._name, "rb").read()
    for name in (b"VTD_ATTN_DIAG", b"VTD_PP3_DIAG", b"VTD_LN_FUSE", b"VTD_W4_DG",
                 b"VTD_DIAG_NOFIN", b"VTD_DIAG_NOATTN", b"VTD_DIAG_NOHEAD",
                 # round 4: w4 / x4 and their switches live in the diagnostic build only
                 b"VTD_GEMM_VARIANT", b"VTD_MX_VARIANT", b"VTD_W4_SCHED", b"VTD_X4_SCHED"):
        assert name + b"\0" not in blob, name
    assert b"gemm_tn_bf16_w4" not in blob and b"gemm_mx8_x4" not in blob
    # round 4: measured-negative / neutral kernels kept for the diagnostic build only
    assert b"gemm_tn_bf16_pp2_mt_kernel" not in blob and b"attention_bf16_ps16_kernel" not in blob
    assert not hasattr(L.lib, "vtd_diag_build")
    # the run-time knobs are read from the environment once per process (vtd_set_knob)
    for name in (b"VTD_ATTN_VARIANT", b"VTD_ATTN_GRID", b"VTD_GEMM_NGW", b"VTD_SPLITK",
                 b"VTD_JPEG_CHUNK_BITS", b"VTD_SKINNY", b"VTD_F32_PP2", b"VTD_STAGGER", b"VTD_GEMM_TR",
                 b"VTD_FIN_WGS", b"VTD_GEMM_TPW"):
        assert name + b"\0" in blob, name


def test_knobs_set_get_and_restore(L):
    """vtd_set_knob returns the previous value; out-of-range knobs are rejected."""
    for k in range(L.KNOB_GEMM_TPW + 1):
        prev = L.lib.vtd_get_knob(k)
        assert L.lib.vtd_set_knob(k, 7) == prev
        assert L.lib.vtd_get_knob(k) == 7
        with L.knob(k, 3):
            assert L.lib.vtd_get_knob(k) == 3
        assert L.lib.vtd_get_knob(k) == 7
        assert L.lib.vtd_set_knob(k, prev) == 7
    assert L.lib.vtd_set_knob(99, 1) == -1 and L.lib.vtd_get_knob(-1) == -1


def test_ctypes_struct_layout_matches_c(L):
    """Compile a probe against include/vtd.h with gcc and compare sizeof/offsetof."""
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "vtd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu\n", sizeof(vtd_config), sizeof(vtd_dims),
         sizeof(vtd_layer_weights), sizeof(vtd_weights), sizeof(vtd_epilogue));
  printf("%zu %zu %zu %zu\n", offsetof(vtd_dims, rows), offsetof(vtd_weights, layers),
         offsetof(vtd_weights, w_final), offsetof(vtd_epilogue, scatter_tokens));
  return 0;
}'''
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "p.c"), os.path.join(d, "p")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.dirname(HEADER), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    sizes = [int(v) for v in out]
    assert sizes[:5] == [ctypes.sizeof(s) for s in (L.VtdConfig, L.VtdDims, L.VtdLayerWeights,
                                                     L.VtdWeights, L.VtdEpilogue)]
    assert sizes[5:] == [L.VtdDims.rows.offset, L.VtdWeights.layers.offset,
                         L.VtdWeights.w_final.offset, L.VtdEpilogue.scatter_tokens.offset]


def _cfg(L, kw, batch=2, dtype=1):
    k = V.resolve_kwargs(**kw)
    h, w, c = k["input_shape"]
    return L.VtdConfig(batch=batch, image_h=h, image_w=w, channels=c,
                       patch_size=k["patch_size"], embedding_dim=k["embedding_dim"],
                       num_heads=k["encoder_num_heads"], key_dim=k["encoder_key_dim"],
                       mlp_quantities=k["encoder_mlp_quantities"],
                       repeat_times=k["encoder_repeat_times"],
                       head_last_units=k["mlp_head_last_units"],
                       head_layers=k["mlp_head_dense_layers_quantity"],
                       head_repeats=k["mlp_head_dense_mish_block_repeats"],
                       use_mish=int(k["use_mish"]), dtype=dtype)


CONFIGS = [
    {},                                                                  # C1 default
    dict(input_shape=(224, 224, 3), patch_size=16, embedding_dim=768, encoder_num_heads=12,
         encoder_key_dim=64, encoder_repeat_times=12, encoder_mlp_quantities=3,
         use_mish=False),                                                # C2
    dict(input_shape=(640, 640, 3), patch_size=16, embedding_dim=768, encoder_num_heads=12,
         encoder_key_dim=64, encoder_repeat_times=12, encoder_mlp_quantities=3),   # C3
    dict(input_shape=(33, 50, 3), patch_size=7, embedding_dim=20, encoder_num_heads=2,
         encoder_key_dim=12, encoder_mlp_quantities=2, encoder_repeat_times=2,
         mlp_head_last_units=4, mlp_head_dense_layers_quantity=5,
         mlp_head_dense_mish_block_repeats=2, use_mish=False),
]


@pytest.mark.parametrize("kw", CONFIGS)
def test_derived_dims_match_oracle_shapes(L, kw):
    d = L.VtdDims()
    L.check(L.lib.vtd_derive_dims(ctypes.byref(_cfg(L, kw)), ctypes.byref(d)))
    shapes = V.layer_output_shapes(**kw)
    _, gh, gw, pdim = shapes["split_image_into_patches"]
    assert (d.grid_h, d.grid_w, d.tokens, d.patch_dim) == (gh, gw, gh * gw, pdim)
    k = V.resolve_kwargs(**kw)
    for j in range(k["encoder_mlp_quantities"]):
        assert d.mlp_units[j] == shapes[f"MLP_1_{j + 1}"][-1]
    heads = [s[-1] for n, s in shapes.items() if n.startswith("dense_")]
    assert [d.head_units[j] for j in range(d.n_head)] == heads
    for v, vp in [(d.patch_dim, d.patch_dim_p), (d.d, d.d_p), (d.tokens, d.tokens_p)]:
        assert vp >= v and vp % L.KALIGN == 0
    assert d.key_dim_p >= k["encoder_key_dim"] and (d.inner_p % L.KALIGN == 0)
    h, w, _ = k["input_shape"]
    p = k["patch_size"]
    assert d.pad_top == ((gh - 1) * p + p - h) // 2 and d.pad_left == ((gw - 1) * p + p - w) // 2


@pytest.mark.parametrize("kw", CONFIGS)
def test_weight_names_match_oracle(L, kw):
    from vision_transformer_detector_amd.detector import keras_weight_names
    d = L.VtdDims()
    L.check(L.lib.vtd_derive_dims(ctypes.byref(_cfg(L, kw)), ctypes.byref(d)))
    got = keras_weight_names(V.resolve_kwargs(**kw), d)
    assert list(got.items()) == list(V.weight_shapes(**kw).items())


def test_workspace_grows_with_batch(L):
    sizes = []
    for b in (1, 8, 64):
        n = ctypes.c_size_t()
        L.check(L.lib.vtd_workspace_bytes(ctypes.byref(_cfg(L, CONFIGS[1], batch=b)),
                                          ctypes.byref(n)))
        sizes.append(n.value)
    assert sizes[0] < sizes[1] < sizes[2]
    assert sizes[2] < 64 * sizes[0] * 1.01


@pytest.mark.parametrize("field,value", [("batch", 0), ("patch_size", 0), ("key_dim", 200),
                                         ("mlp_quantities", 17), ("dtype", 7),
                                         ("head_layers", 0)])
def test_invalid_config_raises_value_error(L, field, value):
    cfg = _cfg(L, CONFIGS[0])
    setattr(cfg, field, value)
    d = L.VtdDims()
    with pytest.raises(ValueError):
        L.check(L.lib.vtd_derive_dims(ctypes.byref(cfg), ctypes.byref(d)), "derive")
    assert L.lib.vtd_last_error()


def test_invalid_op_args_raise_before_any_launch(L):
    # K not a multiple of VTD_KALIGN, null pointers: rejected on the host, no GPU needed
    e = L.VtdEpilogue()
    with pytest.raises(ValueError):
        L.check(L.lib.vtd_gemm(16, 16, 30, 1, 32, 1, 32, L.BF16, ctypes.byref(e), None))
    with pytest.raises(ValueError):
        L.check(L.lib.vtd_attention(None, 1, 4, 1, 48, 144, 1.0, None, 48, L.BF16, None))
    with pytest.raises(ValueError):
        L.check(L.lib.vtd_layernorm(None, L.F32, 1, 4, 4, None, None, 1e-3, None, 4, L.F32, None))
    # split-bf16 A operand (dtype VTD_BF16X3): K = 3 P with P % 64 == 0, lda >= 2 P
    e.out, e.ldo, e.out_dtype = 1, 16, L.F32
    for K, lda in ((128, 128), (192, 120), (576, 256)):
        with pytest.raises(ValueError):
            L.check(L.lib.vtd_gemm(16, 16, K, 1, lda, 1, K, L.BF16X3, ctypes.byref(e), None))
        with pytest.raises(ValueError):
            L.check(L.lib.vtd_gemm_splitk(16, 16, K, 1, lda, 1, K, L.BF16X3, ctypes.byref(e), 16,
                                          1 << 20, 2, None))
    # partial LayerNorm statistics need bf16 operands: refused for a split-bf16 A operand
    st = L.VtdEpilogue()
    st.bias, st.out, st.ldo, st.out_dtype = 16, 16, 256, L.BF16
    st.statout, st.stat_ld = 16, 16384
    assert L.lib.vtd_gemm(16384, 256, 768, 16, 512, 16, 768, L.BF16X3, ctypes.byref(st),
                          None) == -2
    # a split-bf16 output: two ldo / 2 wide pieces
    e.ldo, e.out_dtype = 33, L.BF16X3
    with pytest.raises(ValueError):
        L.check(L.lib.vtd_gemm(16, 16, 64, 1, 64, 1, 64, L.BF16, ctypes.byref(e), None))


def test_presets_param_counts():
    from vision_transformer_detector_amd import presets
    n = sum(int(np.prod(s)) for s in V.weight_shapes(**presets.VIT_B16_224).values())
    assert abs(n / 1e6 - 180.36) < 0.01
    n = sum(int(np.prod(s)) for s in V.weight_shapes(**presets.C1_REFERENCE_DEFAULT).values())
    assert abs(n / 1e6 - 131.48) < 0.01


def test_model_requires_a_hip_device():
    import torch
    import vision_transformer_detector_amd as vtd
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(Exception):
        vtd.create_vision_transformer_detector(input_shape=(32, 32, 3), patch_size=8,
                                               embedding_dim=8, device="cpu")


def test_dropout_rates_and_training_flag():
    """dropout is the identity at inference (vtd.py:369, 405, 486 run with the call's
    training flag): any rate in [0, 1) is accepted (the GPU test checks the logits); a rate
    outside it, or a build-time training=True with dropout on, is refused before any
    device work."""
    import vision_transformer_detector_amd as vtd
    with pytest.raises(ValueError, match="dropout rate"):
        vtd.create_vision_transformer_detector(dropout=1.5)
    with pytest.raises(ValueError, match="training=True"):
        vtd.create_vision_transformer_detector(dropout=0.1, training=True)


def test_gemm_lds_swizzle_conflict_free():
    """The 256-tile GEMMs' 128-B-row LDS swizzles serve every ds_read_b128 lane group of
    their plain and permuted fragment reads without bank conflicts (tools/swizzle_check.py)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "swizzle_check.py")],
                       capture_output=True, text=True)
    assert r.returncode == 0 and "conflict-free" in r.stdout


def test_bench_golden_generators_match_oracle():
    """bench.py's parity_mode regenerates the batched golden case's weights and images without
    the oracle (golden_weights / golden_images); they must be the oracle's draws exactly."""
    import json
    import bench
    from oracle import vtd_numpy as V
    from vision_transformer_detector_amd.detector import keras_weight_names
    from vision_transformer_detector_amd import _lib as L2
    kw = dict(input_shape=(40, 36, 3), patch_size=8, embedding_dim=24, encoder_num_heads=3,
              encoder_key_dim=10, encoder_mlp_quantities=3, encoder_repeat_times=2,
              mlp_head_last_units=8, mlp_head_dense_layers_quantity=3)
    full = V.resolve_kwargs(**kw)
    cfg = L2.VtdConfig(batch=1, image_h=40, image_w=36, channels=3, patch_size=8,
                       embedding_dim=24, num_heads=3, key_dim=10, mlp_quantities=3,
                       repeat_times=2, head_last_units=8, head_layers=3, head_repeats=1,
                       use_mish=1, dtype=0)
    dims = L2.VtdDims()
    assert L2.lib.vtd_derive_dims(ctypes.byref(cfg), ctypes.byref(dims)) == 0
    names = keras_weight_names(full, dims)
    got = bench.golden_weights(names, seed=5, perturb=0.02)
    want = V.init_weights(seed=5, perturb=0.02, **kw)
    assert list(got) == list(want)
    for n in want:
        assert np.array_equal(got[n], want[n]), n
    assert np.array_equal(bench.golden_images(3, (40, 36, 3), 4, True),
                          V.synthetic_images(3, (40, 36, 3), seed=4, letterbox=True))
    spec = json.load(open(os.path.join(ROOT, "tests", "golden", "batched_forward.json")))
    assert bench.GOLDEN_CASE in spec and len(bench.GOLDEN_POS) == spec[bench.GOLDEN_CASE]["n"]


def test_enable_device_kernel_arguments_reports_effect(monkeypatch):
    """The opt-in kernel-argument placement takes effect only before the HIP runtime
    initialises: after it, the helper says so (False + a warning) instead of claiming it."""
    import torch
    import vision_transformer_detector_amd as vtd
    monkeypatch.delenv("HIP_FORCE_DEV_KERNARG", raising=False)
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    with pytest.warns(RuntimeWarning, match="already initialised"):
        assert vtd.enable_device_kernel_arguments() is False
    assert "HIP_FORCE_DEV_KERNARG" not in os.environ
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: False)
    assert vtd.enable_device_kernel_arguments() is True
    monkeypatch.setenv("HIP_FORCE_DEV_KERNARG", "0")        # an explicit setting wins
    assert vtd.enable_device_kernel_arguments() is False
